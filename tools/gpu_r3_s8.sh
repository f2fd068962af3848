#!/bin/bash
# Round 3 session 8: Zipf split threshold (CZ_SPLIT_PERMILLE x SEG) experiment, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03
export TMPDIR=/tmp
for round in 1 2; do
  for sp in 1500 1000 1250 2000; do
    for seg in 128 96; do
      CZ_SPLIT_PERMILLE=$sp timeout -k 10 300 python bench.py --config zipf --seg-blocks $seg --no-cpu-baseline > gpurun_out/r03/zsplit.log 2>&1 || { tail gpurun_out/r03/zsplit.log; exit 5; }
      python3 -c "import json; d=json.loads(open('gpurun_out/r03/zsplit.log').read().strip().splitlines()[-1]); print('split $sp seg $seg round $round ->', d['value'], 'GiB/s', d['roofline']['kernel_ms'], 'ms')"
    done
  done
done
