#!/bin/bash
# Where the waves of a bench config's kernel spend their cycles (SQ wait / active counters),
# two PMC passes per config:  bash tools/gpu_stall.sh 4k open4k zipf
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY"
P2="SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_IFETCH SQ_BUSY_CYCLES"
for key in "$@"; do
  args=$(python3 tools/pmc_key.py args "$key"); f=$(python3 tools/pmc_key.py file "$key")
  for pass in 1 2; do
    eval "ctr=\$P$pass"
    timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/stall_${f}_$pass -o run --kernel-include-regex "k_seal|k_open" -- python3 bench.py --steps 12 --warmup 4 --no-cpu-baseline --no-roundtrip $args > gpurun_out/stall_${f}_$pass.log 2>&1 || { tail -5 gpurun_out/stall_${f}_$pass.log; exit 6; }
  done
  python3 tools/stall_summary.py gpurun_out "$key"
done
exit 0
