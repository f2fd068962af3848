#!/bin/bash
# ctx tests, then bench.py --config nacl with the small-batch segment path and without (CZ_CTX_LANES_ONLY)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "ctx or nacl" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ctx_small.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_ctx_small.log; [ $rc -eq 0 ] || exit $rc
for round in 1 2; do
  for lanes in 0 1; do
    if [ $lanes = 1 ]; then export CZ_CTX_LANES_ONLY=1; else unset CZ_CTX_LANES_ONLY; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline --config nacl > gpurun_out/naclab.log 2>&1 || { tail gpurun_out/naclab.log; exit 5; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/naclab.log').read().strip().splitlines()[-1])
print('lanes_only=$lanes round $round', [(b['batch'], b['call_us']) for b in d['batched_4k']], 'win', d['batch_beating_one_cpu_core'])"
  done
done
