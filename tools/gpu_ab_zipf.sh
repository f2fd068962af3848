#!/bin/bash
# Segment parity, then interleaved A/B (libcz_base.so vs libcz_new.so) on the Zipf seal.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_segments.py tests/test_gpu_dense.py tests/test_gpu_engine.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_zipf_ab.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_zipf_ab.log; [ $rc -eq 0 ] || exit $rc
for a in "--config zipf" "--config zipf --out-align 16"; do
  echo "== A/B $a"
  bash tools/gpu_lib_ab.sh "$a --steps 30 --warmup 20" libcz_base.so libcz_new.so || exit 5
done
exit 0
