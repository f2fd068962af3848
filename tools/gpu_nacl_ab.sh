#!/bin/bash
# ctx pipeline tests, then bench.py --config nacl for each library build (CZ_LIB), interleaved
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "ctx or nacl" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_nacl_ab.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_nacl_ab.log; [ $rc -eq 0 ] || exit $rc
for round in 1 2; do
  for lib in "$@"; do
    CZ_LIB=$PWD/jeromq_amd/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --config nacl > gpurun_out/naclab.log 2>&1 || { tail gpurun_out/naclab.log; exit 5; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/naclab.log').read().strip().splitlines()[-1])
print('$lib round $round', [(r['payload_bytes'], r['seal_us'], r['open_us']) for r in d['single_shot']])
print('   batched', [(b['batch'], b['call_us']) for b in d['batched_4k']], 'win', d['batch_beating_one_cpu_core'])"
  done
done
