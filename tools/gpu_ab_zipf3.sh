#!/bin/bash
# Full GPU suite on the working build, then interleaved lib A/B on the three Zipf layouts:
# bash tools/gpu_ab_zipf3.sh libA.so libB.so
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== pytest -m gpu"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for args in "--config zipf" "--config zipf --in-align 8 --out-align 8" "--config zipf --out-align 1"; do
  echo "== $args"
  bash tools/gpu_lib_ab.sh "$args" "$@" || exit 5
done
exit 0
