#!/bin/bash
# Round 3 session 5: box-layout seal (parity + bench line), open line-0 burst (parity, A/B, FETCH).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03
export TMPDIR=/tmp
echo "== parity (box, open, full suite)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03/pytest_gpu_s5.log 2>&1
rc=$?; tail -2 gpurun_out/r03/pytest_gpu_s5.log; [ $rc -eq 0 ] || exit $rc
echo "== A/B open4k"
bash tools/gpu_lib_ab.sh "--config open4k" libcz_zclass.so libcz_open0.so || exit 5
echo "== bench 4k vs 4k_box"
for c in 4k 4k_box; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-roundtrip > gpurun_out/r03/bench_${c}_s5.log 2>&1 || { tail gpurun_out/r03/bench_${c}_s5.log; exit 4; }
  tail -1 gpurun_out/r03/bench_${c}_s5.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['roofline']['hbm_copy_GBps'], d['roofline']['frac_of_copy'])"
done
echo "== PMC open4k 4k_box"
bash tools/gpu_traffic.sh open4k 4k_box || exit 7
bash tools/gpu_valu.sh open4k 4k_box || exit 8
cp profiles/pmc_traffic.json gpurun_out/r03/pmc_traffic_s5.json
echo "== nacl single-message latency"
timeout -k 10 300 python bench.py --config nacl --steps 10 --warmup 2 > gpurun_out/r03/bench_nacl_s5.log 2>&1 || { tail gpurun_out/r03/bench_nacl_s5.log; exit 4; }
tail -1 gpurun_out/r03/bench_nacl_s5.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); [print(r) for r in d['single_shot']]"
