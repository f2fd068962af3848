#!/bin/bash
# Register-only Salsa20 / Poly1305 issue-rate microbenchmarks (tools/diag/salsa_ub.hip),
# then the headline bench on the same box for reference.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 ./tools/diag/salsa_ub ${NB:-32} > gpurun_out/salsa_ub.log 2>&1; rc=$?; cat gpurun_out/salsa_ub.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_4k.log 2>&1 || { tail gpurun_out/bench_4k.log; exit 4; }
tail -1 gpurun_out/bench_4k.log
exit 0
