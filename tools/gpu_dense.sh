#!/bin/bash
# Shifted line emitter session: parity (dense/segments/uniform), Zipf A/B against a baseline
# library, dense-layout bench lines.  usage: bash tools/gpu_dense.sh [baseline.so]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
BASE=${1:-libcz_base.so}
echo "== pytest dense + segments + parity"
timeout -k 10 600 python -u -m pytest tests/test_gpu_dense.py tests/test_gpu_segments.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_dense.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_dense.log; [ $rc -eq 0 ] || exit $rc
echo "== A/B zipf (128-byte output slots)"
bash tools/gpu_lib_ab.sh "--config zipf --steps 20 --warmup 10" $BASE libcurvezmq_mi355x.so || exit 5
for oa in 8 1; do
  echo "== bench zipf --out-align $oa"
  timeout -k 10 300 python bench.py --config zipf --out-align $oa --no-cpu-baseline > gpurun_out/bench_zipf_oa$oa.log 2>&1 || { tail gpurun_out/bench_zipf_oa$oa.log; exit 6; }
  tail -1 gpurun_out/bench_zipf_oa$oa.log | cut -c1-420
done
for cfg in 4k_dense 4k; do
  echo "== bench $cfg"
  timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline --no-roundtrip > gpurun_out/bench_$cfg.log 2>&1 || { tail gpurun_out/bench_$cfg.log; exit 7; }
  tail -1 gpurun_out/bench_$cfg.log | cut -c1-420
done
exit 0
