#!/bin/bash
# Zipf seal: output slot alignment A/B (16 vs 128 B) with FETCH/WRITE counters.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for al in 16 128; do
  echo "== bench zipf out-align $al"
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --config zipf --out-align $al --no-cpu-baseline > gpurun_out/bench_zipf_al$al.log 2>&1 || { tail gpurun_out/bench_zipf_al$al.log; exit 5; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/bench_zipf_al$al.log').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['kernel_ms'])"
  for pmc in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 240 rocprofv3 --pmc $pmc --output-format csv -d gpurun_out/pmc_zal${al}_$pmc -o run --kernel-include-regex "k_seal_segments" -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --config zipf --out-align $al > gpurun_out/pmc_zal${al}_$pmc.log 2>&1 || { tail -5 gpurun_out/pmc_zal${al}_$pmc.log; exit 6; }
    f=$(find gpurun_out/pmc_zal${al}_$pmc -name "*counter_collection.csv" | head -1)
    python3 -c "
import csv,sys
v=[float(r['Counter_Value']) for r in csv.DictReader(open('$f'))]
print('$pmc', 'KiB/dispatch', sorted(v)[len(v)//2], 'n', len(v))"
  done
done
exit 0
