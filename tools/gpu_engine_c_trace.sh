#!/bin/bash
# Copy / kernel timeline of the C engine bench (rocprofv3 memory-copy + kernel trace) and the
# engine's own per-phase times (CZ_ENGINE_TRACE=1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
CZ_ENGINE_TRACE=1 timeout -k 10 120 ./tools/bin/engine_cbench > gpurun_out/engine_c_phases.log 2>&1 || { tail -5 gpurun_out/engine_c_phases.log; exit 3; }
tail -3 gpurun_out/engine_c_phases.log
timeout -k 10 300 rocprofv3 --memory-copy-trace --kernel-trace --output-format csv -d gpurun_out/engine_c_trace -o run -- ./tools/bin/engine_cbench > gpurun_out/engine_c_trace.log 2>&1 || { tail -5 gpurun_out/engine_c_trace.log; exit 4; }
find gpurun_out/engine_c_trace -name "*.csv"
exit 0
