#!/bin/bash
# Interleaved A/B of library builds on the batching-engine bench: bash tools/gpu_engine_ab.sh lib1.so lib2.so ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_engine_ab.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_engine_ab.log; [ $rc -eq 0 ] || exit $rc
for round in 1 2; do
  for lib in "$@"; do
    CZ_LIB=$PWD/jeromq_amd/$lib timeout -k 10 300 python bench.py --config engine > gpurun_out/engab.log 2>&1 || { tail gpurun_out/engab.log; exit 5; }
    python3 -c "import json; d=json.loads(open('gpurun_out/engab.log').read().strip().splitlines()[-1]); print('$lib round $round -> out', d['value'], 'in', d['open_GiBps'], d['timings_s'])"
  done
done
exit 0
