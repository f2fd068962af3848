#!/bin/bash
# Parity (seal/open/dense/segments) on the current build, then interleaved A/B of libcz_base.so vs
# libcz_new.so on the 4k seal, 4k open and 100 B configs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== pytest parity"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dense.py tests/test_gpu_segments.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ab.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_ab.log; [ $rc -eq 0 ] || exit $rc
for cfg in "--config 4k" "--config open4k" "--config 100b" ${EXTRA_CFG:+"$EXTRA_CFG"}; do
  echo "== A/B $cfg"
  bash tools/gpu_lib_ab.sh "$cfg --steps 30 --warmup 20 --no-roundtrip" libcz_base.so libcz_new.so || exit 5
done
exit 0
