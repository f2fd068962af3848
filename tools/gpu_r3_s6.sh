#!/bin/bash
# Round 3 session 6: one-launch NaCl drop-in with key/nonce in the kernel arguments.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_handshake.py tests/test_gpu_x25519.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03/pytest_nacl_s6.log 2>&1
rc=$?; tail -2 gpurun_out/r03/pytest_nacl_s6.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config nacl --steps 10 --warmup 2 > gpurun_out/r03/bench_nacl_s6.log 2>&1 || { tail gpurun_out/r03/bench_nacl_s6.log; exit 4; }
tail -1 gpurun_out/r03/bench_nacl_s6.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); [print(r) for r in d['single_shot']]; print(d['batch_beating_one_cpu_core'])"
