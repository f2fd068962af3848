#!/bin/bash
# Counter-high-word open mismatch: per-build diagnostic (tools/dbg/open_hiword.py), then the full
# -m gpu suite and lib A/Bs for the candidate that is clean:  bash tools/gpu_fold_dbg.sh base cand...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
BASE=$1; shift
for lib in $BASE "$@"; do
  echo "== $lib"
  CZ_LIB=$PWD/jeromq_amd/$lib timeout -k 10 120 python tools/dbg/open_hiword.py || exit 3
done
exit 0
