#!/bin/bash
# Copy / kernel timeline of the engine bench (rocprofv3 memory-copy + kernel trace).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --memory-copy-trace --kernel-trace --output-format csv -d gpurun_out/engine_trace -o run -- python3 bench.py --config engine > gpurun_out/engine_trace.log 2>&1 || { tail -5 gpurun_out/engine_trace.log; exit 4; }
find gpurun_out/engine_trace -name "*.csv" | head
exit 0
