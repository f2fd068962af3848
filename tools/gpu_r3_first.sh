cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r03
export TMPDIR=/tmp
echo "== issue_ub"
timeout -k 10 240 ./tools/diag/issue_ub 256 > gpurun_out/r03/issue_ub.log 2>&1 || { tail gpurun_out/r03/issue_ub.log; exit 2; }
cat gpurun_out/r03/issue_ub.log
echo "== pytest -m gpu"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r03/pytest_gpu_bufstore.log 2>&1
rc=$?; tail -3 gpurun_out/r03/pytest_gpu_bufstore.log; [ $rc -eq 0 ] || exit $rc
for cfg in 4k open4k zipf; do
  echo "== bench $cfg"
  timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline > gpurun_out/r03/bench_${cfg}_bufstore.log 2>&1 || { tail gpurun_out/r03/bench_${cfg}_bufstore.log; exit 4; }
  tail -1 gpurun_out/r03/bench_${cfg}_bufstore.log | cut -c1-330
done
