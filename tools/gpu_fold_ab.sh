#!/bin/bash
# Candidate library builds: the counter-high-word open diagnostic for each, the full -m gpu suite
# for each candidate, then interleaved lib A/Bs on the 4k seal, the 4k open and the Zipf seal:
#   bash tools/gpu_fold_ab.sh base.so cand.so [cand2.so ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
BASE=$1; shift
for lib in $BASE "$@"; do
  echo "== diag $lib"
  CZ_LIB=$PWD/jeromq_amd/$lib timeout -k 10 120 python tools/dbg/open_hiword.py > gpurun_out/diag_$lib.log 2>&1 || { tail gpurun_out/diag_$lib.log; exit 3; }
  grep -c " 0 bad frames" gpurun_out/diag_$lib.log
done
for lib in "$@"; do
  echo "== pytest -m gpu with $lib"
  CZ_LIB=$PWD/jeromq_amd/$lib timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_$lib.log 2>&1
  rc=$?; tail -1 gpurun_out/pytest_gpu_$lib.log; [ $rc -eq 0 ] || exit $rc
done
for cfg in 4k open4k zipf; do
  echo "== A/B $cfg"
  bash tools/gpu_lib_ab.sh "--config $cfg --no-roundtrip" $BASE "$@" || exit 5
done
exit 0
