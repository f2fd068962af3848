#!/bin/bash
# Round 3 session 3: uniform dense emitter (EmitShiftLinesUni) parity + A/B, Zipf 8-byte layout PMC.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03
export TMPDIR=/tmp
[ -n "$SKIP_PARITY" ] || {
echo "== dense parity"
timeout -k 10 600 python -u -m pytest tests/test_gpu_layouts_full.py tests/test_gpu_dense.py tests/test_abi.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03/pytest_dense_uni.log 2>&1
rc=$?; tail -3 gpurun_out/r03/pytest_dense_uni.log; [ $rc -eq 0 ] || exit $rc; }
echo "== A/B 4k_dense"
bash tools/gpu_lib_ab.sh "--config 4k_dense" libcz_bufstore.so libcz_denseuni.so || exit 5
echo "== latency floors"
timeout -k 10 120 ./tools/diag/latency_ub > gpurun_out/r03/latency_ub.log 2>&1 || { tail gpurun_out/r03/latency_ub.log; exit 3; }
cat gpurun_out/r03/latency_ub.log
echo "== bench 4k (copy ceiling)"
timeout -k 10 300 python bench.py --config 4k --no-cpu-baseline > gpurun_out/r03/bench_4k_copyk.log 2>&1 || { tail gpurun_out/r03/bench_4k_copyk.log; exit 4; }
tail -1 gpurun_out/r03/bench_4k_copyk.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline'])"
echo "== PMC zipf 8-byte layout"
bash tools/gpu_traffic.sh zipf@ia8,oa8 4k_dense || exit 7
bash tools/gpu_valu.sh zipf@ia8,oa8 zipf 4k_dense || exit 8
bash tools/gpu_stall.sh zipf@ia8,oa8 zipf 4k_dense > gpurun_out/r03/stall_s3.log 2>&1 || { tail gpurun_out/r03/stall_s3.log; exit 9; }
cat gpurun_out/r03/stall_s3.log
cp profiles/pmc_traffic.json gpurun_out/r03/pmc_traffic_s3.json
