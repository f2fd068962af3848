cd "${GRAFT_REPO_ROOT:-.}"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for c in 4k 100b zipf open4k; do echo "== $c"; bash tools/gpu_lib_ab.sh "--config $c --steps 20 --warmup 10" lib_ab_head.so lib_ab_nounal.so libcurvezmq_mi355x.so || exit 5; done
