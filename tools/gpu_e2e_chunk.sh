#!/bin/bash
# e2e4k (pinned host -> seal/open -> pinned host) at several pipeline chunk sizes, interleaved
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for round in 1 2; do
  for c in 4096 8192 16384 32768; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --config e2e4k --chunk-frames $c > gpurun_out/e2ec.log 2>&1 || { tail gpurun_out/e2ec.log; exit 5; }
    python3 -c "import json; d=json.loads(open('gpurun_out/e2ec.log').read().strip().splitlines()[-1]); print('chunk $c round $round -> seal', d['value'], 'open', d['open_GiBps'], 'frac', d['frac_of_bidir_ceiling'])"
  done
done
