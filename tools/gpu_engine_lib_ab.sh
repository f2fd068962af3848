#!/bin/bash
# Interleaved A/B of library builds (CZ_LIB) on bench.py --config engine:
#   bash tools/gpu_engine_lib_ab.sh lib1.so lib2.so ...   (names under jeromq_amd/)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for round in 1 2 3; do
  for lib in "$@"; do
    CZ_LIB=$PWD/jeromq_amd/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --config engine > gpurun_out/engab.log 2>&1 || { tail gpurun_out/engab.log; exit 5; }
    python3 -c "import json; d=json.loads(open('gpurun_out/engab.log').read().strip().splitlines()[-1]); print('$lib round $round -> out', d['value'], 'in', d['open_GiBps'], 'GiB/s', d['timings_s']); [print('   small', r) for r in d.get('small_flush', [])]"
  done
done
exit 0
