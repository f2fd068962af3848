#!/bin/bash
# Interleaved A/B of several library builds on one or more configs:
#   CFGS="4k open4k" LIBS="libcz_base.so libcz_new.so" bash tools/gpu_ab_multi.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in $CFGS; do
  echo "== A/B $cfg"
  bash tools/gpu_lib_ab.sh "--config $cfg --steps 30 --warmup 20 --no-roundtrip $EXTRA" $LIBS || exit 5
done
exit 0
