#!/bin/bash
# Dense-output parity, then interleaved A/B (libcz_base.so vs libcz_new.so) on the dense 4 KiB
# seal and the Zipf seal with 8-byte and 1-byte output offsets.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== pytest dense + segments + parity"
timeout -k 10 400 python -u -m pytest tests/test_gpu_dense.py tests/test_gpu_segments.py tests/test_gpu_parity.py tests/test_gpu_engine.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_dense.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_dense.log; [ $rc -eq 0 ] || exit $rc
for a in "--config 4k_dense" "--config zipf --out-align 8 --in-align 8" "--config zipf --out-align 1"; do
  echo "== A/B $a"
  bash tools/gpu_lib_ab.sh "$a --steps 30 --warmup 20" libcz_base.so libcz_new.so || exit 5
done
exit 0
