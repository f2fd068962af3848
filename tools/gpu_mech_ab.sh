#!/bin/bash
# mechanism / engine / ctx GPU tests, then bench.py --config nacl per library build (CZ_LIB), interleaved
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_interop.py tests/test_gpu_handshake.py tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_mech.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_mech.log; [ $rc -eq 0 ] || exit $rc
for round in 1 2; do
  for lib in "$@"; do
    CZ_LIB=$PWD/jeromq_amd/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --config nacl > gpurun_out/naclab.log 2>&1 || { tail gpurun_out/naclab.log; exit 5; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/naclab.log').read().strip().splitlines()[-1])
print('$lib round $round mech', [(r['payload_bytes'], r['encode_us'], r['decode_us'], r['verified']) for r in d['mechanism_single']])
print('   single', [(r['payload_bytes'], r['seal_us'], r['open_us']) for r in d['single_shot']])"
  done
done
