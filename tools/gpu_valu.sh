#!/bin/bash
# Instruction-count PMC pass per bench config (VALU issue roofline), folded into
# profiles/pmc_traffic.json:  bash tools/gpu_valu.sh 4k 100b zipf open4k zipf@ia8,oa8 (tools/pmc_key.py keys)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for key in "$@"; do
  args=$(python3 tools/pmc_key.py args "$key"); f=$(python3 tools/pmc_key.py file "$key")
  echo "== $key VALU"
  timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/valu_${f} -o run --kernel-include-regex "k_seal|k_open" -- python3 bench.py --steps 3 --warmup 1 --ramp-ms 0 --no-cpu-baseline --no-roundtrip $args > gpurun_out/valu_${f}.log 2>&1 || { tail -5 gpurun_out/valu_${f}.log; exit 6; }
done
python3 tools/valu_update.py gpurun_out "$@"
exit 0
