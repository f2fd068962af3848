#!/bin/bash
# Engine GPU tests, then the C engine bench (tools/engine_cbench.c, no torch) interleaved between
# the in-tree library and a base build in tools/bin/base/ (LD_LIBRARY_PATH wins over RUNPATH).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_handshake.py tests/test_gpu_interop.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_engine_lib.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_engine_lib.log; [ $rc -eq 0 ] || exit $rc
for round in 1 2 3; do
  echo -n "base round $round: "; LD_LIBRARY_PATH=$PWD/tools/bin/base timeout -k 10 120 ./tools/bin/engine_cbench || exit 5
  echo -n "new  round $round: "; timeout -k 10 120 ./tools/bin/engine_cbench || exit 5
done
timeout -k 10 300 python bench.py --config engine > gpurun_out/bench_engine_rxpool.log 2>&1 || { tail gpurun_out/bench_engine_rxpool.log; exit 6; }
tail -1 gpurun_out/bench_engine_rxpool.log | cut -c1-600
CZ_ENGINE_TRACE=1 timeout -k 10 120 ./tools/bin/engine_cbench 2>&1 | tail -3
exit 0
