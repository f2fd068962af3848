#!/bin/bash
# Round 3 session 7: Zipf segment dispatch order (CZ_PLAN_ORDER) experiment, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_segments.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03/pytest_seg_s7.log 2>&1
rc=$?; tail -1 gpurun_out/r03/pytest_seg_s7.log; [ $rc -eq 0 ] || exit $rc
CZ_PLAN_ORDER=mix timeout -k 10 300 python -u -m pytest tests/test_gpu_segments.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03/pytest_seg_s7_mix.log 2>&1
rc=$?; tail -1 gpurun_out/r03/pytest_seg_s7_mix.log; [ $rc -eq 0 ] || exit $rc
for round in 1 2; do
  for order in base asc mix; do
    ev=""; [ $order != base ] && ev="CZ_PLAN_ORDER=$order"
    env $ev timeout -k 10 300 python bench.py --config zipf --no-cpu-baseline > gpurun_out/r03/zorder.log 2>&1 || { tail gpurun_out/r03/zorder.log; exit 5; }
    python3 -c "import json; d=json.loads(open('gpurun_out/r03/zorder.log').read().strip().splitlines()[-1]); print('$order round $round ->', d['value'], 'GiB/s', d['roofline']['kernel_ms'], 'ms')"
  done
done
