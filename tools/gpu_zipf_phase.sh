#!/bin/bash
# Zipf line-phase session: segment/dense parity, interleaved A/B against a baseline library,
# FETCH/WRITE passes for the zipf config.  usage: bash tools/gpu_zipf_phase.sh [baseline.so]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
BASE=${1:-libcz_base.so}
echo "== pytest segments + dense"
timeout -k 10 600 python -u -m pytest tests/test_gpu_segments.py tests/test_gpu_dense.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_seg.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_seg.log; [ $rc -eq 0 ] || exit $rc
echo "== A/B zipf"
bash tools/gpu_lib_ab.sh "--config zipf --steps 20 --warmup 10" $BASE libcurvezmq_mi355x.so || exit 5
echo "== A/B zipf out-align 8"
bash tools/gpu_lib_ab.sh "--config zipf --out-align 8 --steps 20 --warmup 10" $BASE libcurvezmq_mi355x.so || exit 5
bash tools/gpu_traffic.sh zipf || exit 7
exit 0
