set -o pipefail
mkdir -p gpurun_out/r6c
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_dense.py -x -q --timeout 200 --timeout-method thread -k "carry or any_offset" > gpurun_out/r6c/pytest_dense.log 2>&1 || { tail -20 gpurun_out/r6c/pytest_dense.log; exit 3; }
tail -2 gpurun_out/r6c/pytest_dense.log
timeout -k 10 600 python tools/ab_cfg.py --rounds 8 --steps 5 "open4k --out-stride 4129 --tune open_carry=1" "open4k --out-stride 4129 --tune open_carry=3" "open4k --out-stride 4129 --tune open_carry=2" "open4k --out-stride 4136 --tune open_carry=1" "open4k --out-stride 4136 --tune open_carry=3" "open4k" > gpurun_out/r6c/ab_open_half_carry.log 2>&1 || { tail gpurun_out/r6c/ab_open_half_carry.log; exit 4; }
tail -12 gpurun_out/r6c/ab_open_half_carry.log
for kn in 1 3; do
  for pmc in FETCH_SIZE WRITE_SIZE; do
    CZ_TUNE=open_carry=$kn timeout -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d gpurun_out/r6c/fetch_os4129_k${kn}_$pmc -o run --kernel-include-regex "k_open" -- python3 bench.py --config open4k --out-stride 4129 --steps 3 --warmup 1 --ramp-ms 0 --no-cpu-baseline > gpurun_out/r6c/fetch_os4129_k${kn}_$pmc.log 2>&1 || exit 5
    CZ_TUNE=open_carry=$kn timeout -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d gpurun_out/r6c/fetch_os4136_k${kn}_$pmc -o run --kernel-include-regex "k_open" -- python3 bench.py --config open4k --out-stride 4136 --steps 3 --warmup 1 --ramp-ms 0 --no-cpu-baseline > gpurun_out/r6c/fetch_os4136_k${kn}_$pmc.log 2>&1 || exit 6
  done
done
echo done
