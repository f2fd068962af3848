#!/bin/bash
# Full measurement session on one GPU box: parity tests, smoke, bench lines for every config,
# rocprofv3 kernel-trace stats, PMC traffic (FETCH/WRITE) and VALU instruction counts.
# Every GPU step has its own time limit; a failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
# PART (space-separated): tests (pytest -m gpu, smoke), bench (every bench line), trace (rocprofv3 kernel
# traces), pmc (the PMC passes); default "tests bench trace".  Each group fits one gpurun call.
PART=${PART:-tests bench trace}
has() { case " $PART " in *" $1 "*) return 0;; esac; return 1; }
if has tests; then
echo "== pytest -m gpu"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail gpurun_out/smoke.log; exit 3; }
tail -1 gpurun_out/smoke.log
fi
if has bench; then
run() {  # name, bench args
  local name=$1; shift
  echo "== bench $name"
  timeout -k 10 300 python bench.py "$@" > gpurun_out/bench_$name.log 2>&1 || { tail gpurun_out/bench_$name.log; exit 4; }
  tail -1 gpurun_out/bench_$name.log | cut -c1-400
}
run 4k --config 4k
run 4k_dense --config 4k_dense --no-cpu-baseline
run 4k_box --config 4k_box --no-cpu-baseline
run 100b --config 100b --no-cpu-baseline
run zipf --config zipf --no-cpu-baseline
run zipf_oa8 --config zipf --in-align 8 --out-align 8 --no-cpu-baseline
run zipf_oa1 --config zipf --out-align 1 --no-cpu-baseline
run open4k --config open4k --no-cpu-baseline
run zipf_lane --config zipf_lane --no-cpu-baseline
run zipf_open --config zipf_open --no-cpu-baseline
run zipf_open_oa8 --config zipf_open --in-align 8 --out-align 8 --no-cpu-baseline
run open4k_dense --config open4k --out-stride 4129 --no-cpu-baseline
run open4k_dense8 --config open4k --out-stride 4136 --no-cpu-baseline
run open4k_ps4224 --config open4k --plain-stride 4224 --no-cpu-baseline
run 100b_packed --config 100b --in-stride 100 --no-cpu-baseline
run 4k_in4097 --config 4k --in-stride 4097 --no-cpu-baseline
for cfg in e2e4k engine beforenm nacl jni; do
  run $cfg --steps 10 --warmup 2 --config $cfg --no-cpu-baseline
done
# the N > 1 launcher, control plane and leg at 4 ranks on this one GPU (gloo; RCCL needs 4 GPUs)
echo "== bench --gpus 4 (gloo rehearsal)"
CZ_DIST_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 4 --frames 262144 --steps 5 --warmup 2 --ramp-ms 0 --cpu-seconds 1 > gpurun_out/bench_gpus4_gloo.log 2>&1 || { tail gpurun_out/bench_gpus4_gloo.log; exit 4; }
tail -1 gpurun_out/bench_gpus4_gloo.log | cut -c1-400
fi
if has trace; then
for key in 4k zipf open4k 100b 4k_dense 4k_box zipf@ia8,oa8 zipf@oa1 zipf_open@ia8,oa8 open4k@os4129 open4k@os4136; do
  args=$(python3 tools/pmc_key.py args "$key"); f=$(python3 tools/pmc_key.py file "$key")
  echo "== rocprofv3 kernel trace $key"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_$f -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-roundtrip $args > gpurun_out/prof_$f.log 2>&1 || { tail gpurun_out/prof_$f.log; exit 6; }
done
fi
if has pmc; then
bash tools/gpu_traffic.sh 4k 100b zipf open4k 4k_dense 4k_box zipf@ia8,oa8 zipf@oa1 zipf_open@ia8,oa8 open4k@os4129 open4k@os4136 || exit 7
bash tools/gpu_valu.sh 4k 100b zipf open4k 4k_dense 4k_box zipf@ia8,oa8 zipf@oa1 zipf_open@ia8,oa8 open4k@os4129 open4k@os4136 || exit 8
bash tools/gpu_stall.sh 4k open4k zipf > gpurun_out/stall_measure.log 2>&1 || { tail gpurun_out/stall_measure.log; exit 9; }
cp profiles/pmc_traffic.json gpurun_out/pmc_traffic_measure.json
fi
exit 0
