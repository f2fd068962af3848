#!/bin/bash
# bench.py smoke after a bench change: the 4k line and the world-size-2 rehearsal test.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_quick.log 2>&1 || { tail gpurun_out/bench_quick.log; exit 4; }
tail -1 gpurun_out/bench_quick.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_dist.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_dist.log; exit $rc
