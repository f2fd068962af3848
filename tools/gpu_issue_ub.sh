#!/bin/bash
# VALU issue-cost probes (tools/diag/issue_ub*.hip, prebuilt in-tree): per-opcode cycles, fast/slow
# mixing, Salsa20 double-round forms.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03
timeout -k 10 400 ./tools/diag/issue_ub2 ${NIT:-256} > gpurun_out/r03/issue_ub2.log 2>&1; rc=$?; cat gpurun_out/r03/issue_ub2.log; exit $rc
