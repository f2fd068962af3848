#!/bin/bash
# Open + verify at different plaintext slot strides, interleaved on one box:
# bash tools/gpu_open_stride.sh 4096 4224 ...  (is the 4096-byte write stride a channel-camping case?)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for round in 1 2; do
  for ps in "$@"; do
    timeout -k 10 300 python bench.py --config open4k --no-cpu-baseline --plain-stride $ps > gpurun_out/openab_$ps.log 2>&1 || { tail gpurun_out/openab_$ps.log; exit 5; }
    python3 -c "import json; d=json.loads(open('gpurun_out/openab_$ps.log').read().strip().splitlines()[-1]); print('plain stride $ps round $round ->', d['value'], 'GiB/s', d['roofline']['kernel_ms'], 'ms')"
  done
done
exit 0
