#!/bin/bash
# Round-2 re-entry check: full -m gpu suite, smoke, headline bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail gpurun_out/smoke.log; exit 3; }
tail -1 gpurun_out/smoke.log
echo "== bench 4k"
timeout -k 10 300 python bench.py > gpurun_out/bench_4k.log 2>&1 || { tail gpurun_out/bench_4k.log; exit 4; }
tail -1 gpurun_out/bench_4k.log | cut -c1-600
exit 0
