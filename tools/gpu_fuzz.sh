#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_fuzz.py tests/test_gpu_engine.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_fuzz.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|assert" gpurun_out/pytest_fuzz.log | tail -14; tail -1 gpurun_out/pytest_fuzz.log; exit $rc
