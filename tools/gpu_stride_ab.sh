#!/bin/bash
# Slot-stride A/B on one box, interleaved (2 rounds): does a power-of-two slot stride cost
# the 4 KiB kernels anything (HBM channel camping)?  open4k plaintext slots 4096 / 4160 / 4224,
# seal output slots 4224 / 4352, seal input slots 4096 / 4224.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
one() {  # tag, bench args
  local tag=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-roundtrip "$@" > gpurun_out/strideab_$tag.log 2>&1 || { tail gpurun_out/strideab_$tag.log; exit 5; }
  python3 -c "import json; d=json.loads(open('gpurun_out/strideab_$tag.log').read().strip().splitlines()[-1]); print('$tag round $round ->', d['value'], 'GiB/s', d['roofline']['kernel_ms'], 'ms')"
}
for round in 1 2; do
  one open_p4096 --config open4k --plain-stride 4096
  one open_p4224 --config open4k --plain-stride 4224
  one open_p4160 --config open4k --plain-stride 4160
  one seal_o4224 --config 4k
  one seal_o4352 --config 4k --out-stride 4352
  one seal_i4224 --config 4k --in-stride 4224
done
exit 0
