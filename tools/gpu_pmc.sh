#!/bin/bash
# PMC passes (one counter group per rocprofv3 run) for one bench config.
#   bash tools/gpu_pmc.sh <tag> "<bench args>"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
soft() { local rc=$1; [ "$rc" -lt 124 ]; }
TAG=${1:-seal4k}
ARGS=${2:---config 4k}
i=0
for pmc in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE" "SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_BUSY_CYCLES TA_BUSY_avr" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
  i=$((i+1))
  echo "== pmc pass $i: $pmc"
  timeout -k 10 240 rocprofv3 --pmc $pmc --output-format csv -d gpurun_out/pmc_${TAG}_$i -o run --kernel-include-regex "k_seal|k_open" -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline $ARGS > gpurun_out/pmc_${TAG}_$i.log 2>&1
  rc=$?; soft $rc || { tail -5 gpurun_out/pmc_${TAG}_$i.log; exit $rc; }
done
python3 tools/pmc_summary.py gpurun_out pmc_${TAG} > gpurun_out/pmc_${TAG}_summary.txt 2>&1; cat gpurun_out/pmc_${TAG}_summary.txt
exit 0
