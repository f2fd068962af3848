#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit; a crash/timeout/fault ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
echo "== device" ; (rocminfo 2>/dev/null | grep -m2 -E "gfx9|Marketing") || true
echo "== pytest -m gpu"
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu.log; ok $rc || exit $rc
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail gpurun_out/smoke.log; exit 3; }
tail -2 gpurun_out/smoke.log
echo "== bench 4k"
timeout -k 10 300 python bench.py > gpurun_out/bench_4k.log 2>&1 || { tail gpurun_out/bench_4k.log; exit 4; }
tail -1 gpurun_out/bench_4k.log
for cfg in 100b zipf zipf_lane open4k e2e4k engine beforenm; do
  echo "== bench $cfg"
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --config $cfg --no-cpu-baseline > gpurun_out/bench_$cfg.log 2>&1 || { tail gpurun_out/bench_$cfg.log; exit 5; }
  tail -1 gpurun_out/bench_$cfg.log
done
echo "== rocprofv3 kernel trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_4k -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_4k.log 2>&1 || { tail gpurun_out/prof_4k.log; exit 6; }
find gpurun_out/prof_4k -name "*stats*" | head
echo "== rocprofv3 kernel trace (zipf)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_zipf -o run -- python3 bench.py --steps 5 --warmup 1 --config zipf --no-cpu-baseline > gpurun_out/prof_zipf.log 2>&1 || { tail gpurun_out/prof_zipf.log; exit 7; }
exit 0
