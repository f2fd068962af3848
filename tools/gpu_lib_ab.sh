#!/bin/bash
# Interleaved A/B of library builds (CZ_LIB) on one bench config: bash tools/gpu_lib_ab.sh "<bench args>" lib1.so lib2.so ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS=$1; shift
for round in 1 2; do
  for lib in "$@"; do
    CZ_LIB=$PWD/jeromq_amd/$lib timeout -k 10 300 python bench.py --no-cpu-baseline $ARGS > gpurun_out/libab.log 2>&1 || { tail gpurun_out/libab.log; exit 5; }
    python3 -c "import json; d=json.loads(open('gpurun_out/libab.log').read().strip().splitlines()[-1]); print('$lib round $round ->', d['value'], 'GiB/s', d['roofline']['kernel_ms'], 'ms')"
  done
done
exit 0
