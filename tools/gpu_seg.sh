#!/bin/bash
# Segmented ragged path: parity tests, zipf vs zipf_lane bench, kernel stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== pytest segments"
timeout -k 10 600 python -m pytest tests/test_gpu_segments.py -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_seg.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_seg.log; [ $rc -eq 0 ] || exit $rc
for cfg in zipf zipf_lane; do
  echo "== bench $cfg"
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --config $cfg --no-cpu-baseline > gpurun_out/bench_$cfg.log 2>&1 || { tail gpurun_out/bench_$cfg.log; exit 5; }
  tail -1 gpurun_out/bench_$cfg.log
done
echo "== rocprofv3 zipf"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_zipf -o run -- python3 bench.py --steps 5 --warmup 1 --config zipf --no-cpu-baseline > gpurun_out/prof_zipf.log 2>&1 || { tail gpurun_out/prof_zipf.log; exit 6; }
f=$(find gpurun_out/prof_zipf -name "*kernel_stats.csv" | head -1); cut -d, -f1-8 "$f"
exit 0
