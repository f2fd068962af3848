#!/bin/bash
# round-5 interleaved A/B of library builds (tools/ab_lib.py): bash tools/gpu_ab_r5.sh OUT lib1 lib2 ...
cd "$(dirname "$0")/.." || exit 1
out=$1; shift
timeout -k 10 900 python -u tools/ab_lib.py --rounds 10 --steps 5 \
  --spec 4k --spec 4k_dense --spec open4k --spec "open4k --out-stride 4129" \
  --spec "zipf --out-align 8 --in-align 8" --spec "zipf_open --out-align 8 --in-align 8" "$@" > "$out" 2>&1
