#!/bin/bash
# After a kernel change: full -m gpu suite, smoke, the open diagnostic, bench lines for the 4k
# seal / open / Zipf, and the rocprofv3 kernel-trace summary of the headline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== pytest -m gpu"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail gpurun_out/smoke.log; exit 3; }
tail -1 gpurun_out/smoke.log
timeout -k 10 120 python tools/dbg/open_hiword.py > gpurun_out/diag_open.log 2>&1 || { tail gpurun_out/diag_open.log; exit 3; }
grep -c " 0 bad frames" gpurun_out/diag_open.log
for cfg in 4k open4k zipf; do
  echo "== bench $cfg"
  timeout -k 10 300 python bench.py --config $cfg > gpurun_out/bench_$cfg.log 2>&1 || { tail gpurun_out/bench_$cfg.log; exit 4; }
  tail -1 gpurun_out/bench_$cfg.log | cut -c1-200
done
echo "== rocprofv3 kernel trace 4k"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_4k -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-roundtrip --config 4k > gpurun_out/prof_4k.log 2>&1 || { tail gpurun_out/prof_4k.log; exit 6; }
exit 0
