#!/bin/bash
# Run bench.py once per argument set and print value + kernel ms.
#   bash tools/gpu_bench_ab.sh [--tests <pytest file>] "<args 1>" "<args 2>" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "$1" = "--tests" ]; then
  timeout -k 10 600 python -m pytest "$2" -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_ab.log 2>&1
  rc=$?; tail -3 gpurun_out/pytest_ab.log; [ $rc -eq 0 ] || exit $rc
  shift 2
fi
i=0
for a in "$@"; do
  i=$((i+1))
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline $a > gpurun_out/ab_$i.log 2>&1 || { tail gpurun_out/ab_$i.log; exit 5; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ab_$i.log').read().strip().splitlines()[-1]); print('$a', '->', d['value'], 'GiB/s', d['roofline']['kernel_ms'], 'ms')"
done
exit 0
