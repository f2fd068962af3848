#!/bin/bash
# Parity tests on the current build, then interleaved A/B of two library builds on several configs.
#   bash tools/gpu_ab_session.sh lib_a.so lib_b.so "4k open4k zipf 100b"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
A=$1; B=$2; CFGS=${3:-4k}
for cfg in $CFGS; do
  echo "== $cfg"
  bash tools/gpu_lib_ab.sh "--config $cfg --steps 20 --warmup 10" $A $B || exit 5
done
exit 0
