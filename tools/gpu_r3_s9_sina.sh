#!/bin/bash
# Dense tests + full GPU suite on the working build, then bench A/B of two builds over ARGS_LIST
# (';'-separated bench.py argument sets): bash tools/gpu_r3_s9_sina.sh libA.so libB.so
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_dense.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_dense.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_dense.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_dense.log | head; exit $rc; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
IFS=";" read -ra AL <<< "${ARGS_LIST}"
for round in 1 2; do
for a in "${AL[@]}"; do
  for lib in "$@"; do
    CZ_LIB=$PWD/jeromq_amd/$lib timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 10 $a > gpurun_out/o.log 2>&1 || { tail gpurun_out/o.log; exit 3; }
    python -c "import json; d=json.loads(open('gpurun_out/o.log').read().strip().splitlines()[-1]); print('$lib $a round $round', d['value'], d['roofline']['kernel_ms'])"
  done
done
done
exit 0
