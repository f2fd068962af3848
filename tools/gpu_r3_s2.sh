#!/bin/bash
# Round 3 session 2: issue-cost probes, the full-size layout parity tests, buffer-store vs asm-store A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03
export TMPDIR=/tmp
echo "== issue_ub2"
timeout -k 10 400 ./tools/diag/issue_ub2 256 > gpurun_out/r03/issue_ub2.log 2>&1 || { tail gpurun_out/r03/issue_ub2.log; exit 2; }
cat gpurun_out/r03/issue_ub2.log
echo "== full-size layout tests"
timeout -k 10 600 python -u -m pytest tests/test_gpu_layouts_full.py tests/test_gpu_handshake.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03/pytest_layouts_full.log 2>&1
rc=$?; tail -8 gpurun_out/r03/pytest_layouts_full.log; [ $rc -eq 0 ] || exit $rc
echo "== A/B 4k"
bash tools/gpu_lib_ab.sh "--config 4k --no-roundtrip" libcz_asmstore.so libcz_bufstore.so || exit 5
echo "== A/B open4k"
bash tools/gpu_lib_ab.sh "--config open4k" libcz_asmstore.so libcz_bufstore.so || exit 5
