#!/bin/bash
# Full measurement session on one GPU box: parity tests, smoke, bench lines for every config,
# rocprofv3 kernel-trace stats, PMC traffic (FETCH/WRITE) and VALU instruction counts.
# Every GPU step has its own time limit; a failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== pytest -m gpu"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail gpurun_out/smoke.log; exit 3; }
tail -1 gpurun_out/smoke.log
for cfg in 4k 100b zipf open4k zipf_lane; do
  echo "== bench $cfg"
  extra=""; [ $cfg = 4k ] || extra="--no-cpu-baseline"
  timeout -k 10 300 python bench.py --config $cfg $extra > gpurun_out/bench_$cfg.log 2>&1 || { tail gpurun_out/bench_$cfg.log; exit 4; }
  tail -1 gpurun_out/bench_$cfg.log | cut -c1-400
done
for cfg in e2e4k engine beforenm; do
  echo "== bench $cfg"
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --config $cfg --no-cpu-baseline > gpurun_out/bench_$cfg.log 2>&1 || { tail gpurun_out/bench_$cfg.log; exit 5; }
  tail -1 gpurun_out/bench_$cfg.log | cut -c1-300
done
for cfg in 4k zipf open4k 100b; do
  echo "== rocprofv3 kernel trace $cfg"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_$cfg -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-roundtrip --config $cfg > gpurun_out/prof_$cfg.log 2>&1 || { tail gpurun_out/prof_$cfg.log; exit 6; }
done
bash tools/gpu_traffic.sh 4k 100b zipf open4k || exit 7
bash tools/gpu_valu.sh 4k 100b zipf open4k || exit 8
exit 0
