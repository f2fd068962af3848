#!/bin/bash
# Parity of a candidate library build on the full -m gpu suite, then interleaved lib A/Bs on
# the 4k seal, the 4k open and the Zipf seal:  bash tools/gpu_fold_ab.sh base.so cand.so
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
BASE=$1; CAND=$2
echo "== pytest -m gpu with $CAND"
CZ_LIB=$PWD/jeromq_amd/$CAND timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_cand.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gpu_cand.log; [ $rc -eq 0 ] || exit $rc
for cfg in 4k open4k zipf; do
  echo "== A/B $cfg"
  bash tools/gpu_lib_ab.sh "--config $cfg --no-roundtrip" $BASE $CAND || exit 5
done
exit 0
