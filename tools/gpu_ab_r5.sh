#!/bin/bash
# Round-5 interleaved A/B of library builds in one process: bash tools/gpu_ab_r5.sh LOG "<spec>;<spec>..." lib1.so lib2.so ...
# (tools/ab_lib.py: every build on the same batches, rounds alternating between builds)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
LOG=$1; SPECS=$2; shift 2
args=()
IFS=';' read -ra SP <<< "$SPECS"
for s in "${SP[@]}"; do args+=(--spec "$s"); done
libs=()
for l in "$@"; do libs+=("jeromq_amd/$l"); done
timeout -k 10 900 python -u tools/ab_lib.py --rounds 10 --steps 5 "${args[@]}" "${libs[@]}" > "gpurun_out/$LOG" 2>&1
rc=$?; tail -40 "gpurun_out/$LOG"; exit $rc
