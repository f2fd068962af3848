#!/bin/bash
# GPU suite on the working build, then the in-process seal/open shift16 timing for two builds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for lib in "$@"; do
  echo "== $lib"
  CZ_LIB=$PWD/jeromq_amd/$lib timeout -k 10 400 python tools/dbg/seg_shift16_ab.py 8 128 > gpurun_out/al8_$lib.log 2>&1 || { tail gpurun_out/al8_$lib.log; exit 4; }
  grep "shift16=1" gpurun_out/al8_$lib.log
done
exit 0
