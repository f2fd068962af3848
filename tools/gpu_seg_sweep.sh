#!/bin/bash
# Zipf segment length sweep, interleaved (2 rounds): bash tools/gpu_seg_sweep.sh 96 128 192
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for round in 1 2; do
  for sb in "$@"; do
    timeout -k 10 300 python bench.py --config zipf --no-cpu-baseline --seg-blocks $sb > gpurun_out/seg_$sb.log 2>&1 || { tail gpurun_out/seg_$sb.log; exit 5; }
    python3 -c "import json; d=json.loads(open('gpurun_out/seg_$sb.log').read().strip().splitlines()[-1]); print('seg $sb round $round ->', d['value'], 'GiB/s', d['roofline']['kernel_ms'], 'ms')"
  done
done
exit 0
