#!/bin/bash
# The engine bench from C (tools/engine_cbench.c, system HIP runtime, no torch), interleaved A/B of
# an environment toggle:  bash tools/gpu_engine_c_ab.sh VAR=value
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for round in 1 2; do
  for setting in CZ_AB_NONE=1 "$1"; do
    echo -n "$setting round $round: "
    env "$setting" timeout -k 10 120 ./tools/bin/engine_cbench || exit 5
  done
done
exit 0
