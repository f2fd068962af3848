#!/bin/bash
# Instruction mix, waits and clock of the headline against the dense seal (round 5):
#   bash tools/gpu_pmc_dense.sh [keys...]   (default: 4k 4k_dense); summaries in gpurun_out/pmc_dense.txt
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
keys=${*:-4k 4k_dense}
bash tools/gpu_pmc_pass.sh ins "SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH" $keys || exit $?
bash tools/gpu_pmc_pass.sh wait "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_UNALIGNED_STALL SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" $keys || exit $?
bash tools/gpu_pmc_pass.sh clk "GRBM_GUI_ACTIVE GRBM_COUNT SQ_BUSY_CYCLES SQ_WAVES" $keys || exit $?
python3 tools/pmc_pass_summary.py gpurun_out/pmc_ins_* gpurun_out/pmc_wait_* gpurun_out/pmc_clk_* > gpurun_out/pmc_dense.txt 2>&1
cat gpurun_out/pmc_dense.txt
