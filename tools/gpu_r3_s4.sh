#!/bin/bash
# Round 3 session 4: dense at 3 waves/SIMD (class_permute scratch in dynamic LDS), latency and copy probes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03
export TMPDIR=/tmp
echo "== dense parity"
timeout -k 10 600 python -u -m pytest tests/test_gpu_layouts_full.py tests/test_gpu_dense.py tests/test_gpu_segments.py tests/test_gpu_fuzz.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03/pytest_dense3.log 2>&1
rc=$?; tail -2 gpurun_out/r03/pytest_dense3.log; [ $rc -eq 0 ] || exit $rc
echo "== A/B 4k_dense"
bash tools/gpu_lib_ab.sh "--config 4k_dense" libcz_bufstore.so libcz_denseuni.so libcz_dense3.so || exit 5
echo "== A/B zipf 8-byte offsets"
bash tools/gpu_lib_ab.sh "--config zipf --in-align 8 --out-align 8" libcz_dense3.so libcz_zclass.so || exit 5
echo "== A/B zipf 1-byte output offsets"
bash tools/gpu_lib_ab.sh "--config zipf --out-align 1" libcz_dense3.so libcz_zclass.so || exit 5
echo "== copy variants"
timeout -k 10 120 ./tools/diag/copy_ub > gpurun_out/r03/copy_ub.log 2>&1 || { tail gpurun_out/r03/copy_ub.log; exit 3; }
cat gpurun_out/r03/copy_ub.log
echo "== latency floors"
timeout -k 10 120 ./tools/diag/latency_ub > gpurun_out/r03/latency_ub2.log 2>&1 || { tail gpurun_out/r03/latency_ub2.log; exit 3; }
timeout -k 10 120 ./tools/diag/latency_ub spin >> gpurun_out/r03/latency_ub2.log 2>&1 || { tail gpurun_out/r03/latency_ub2.log; exit 3; }
cat gpurun_out/r03/latency_ub2.log
echo "== issue probe (left-shift candidates)"
timeout -k 10 400 ./tools/diag/issue_ub2 256 > gpurun_out/r03/issue_ub3.log 2>&1 || { tail gpurun_out/r03/issue_ub3.log; exit 3; }
grep -E "lshl|lshr|ashr|b16|u16|bfrev|subrev|sdwa|dpp|imm|ldexp|cndmask|max_f32|med3|exp_f32|F15S1|F7S1" gpurun_out/r03/issue_ub3.log
