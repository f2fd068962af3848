#!/bin/bash
# Host-resident paths: engine tests (pipelined flush_out, wire_iov), engine / e2e / jnacl latency
# bench lines with the PCIe copy ceilings.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== pytest engine"
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_parity.py -k "engine or nacl" -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_engine.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_engine.log; [ $rc -eq 0 ] || exit $rc
echo "== engine"
CZ_ENGINE_TRACE=1 timeout -k 10 300 python bench.py --config engine > gpurun_out/bench_engine.log 2>&1 || { tail gpurun_out/bench_engine.log; exit 4; }
grep -v "^\[cz_engine\]" gpurun_out/bench_engine.log | tail -1 | cut -c1-1500
grep "flush_out" gpurun_out/bench_engine.log | tail -2
echo "== e2e4k"
timeout -k 10 300 python bench.py --config e2e4k > gpurun_out/bench_e2e4k.log 2>&1 || { tail gpurun_out/bench_e2e4k.log; exit 5; }
tail -1 gpurun_out/bench_e2e4k.log | cut -c1-1500
echo "== nacl"
timeout -k 10 300 python bench.py --config nacl > gpurun_out/bench_nacl.log 2>&1 || { tail gpurun_out/bench_nacl.log; exit 6; }
tail -1 gpurun_out/bench_nacl.log
exit 0
