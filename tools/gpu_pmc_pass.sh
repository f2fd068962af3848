#!/bin/bash
# One rocprofv3 PMC pass (<= 8 SQ counters) over the seal / open kernels of bench configs:
#   bash tools/gpu_pmc_pass.sh NAME "CTR1 CTR2 ..." key1 key2 ...   (keys as tools/pmc_key.py)
# Raw CSVs land in gpurun_out/pmc_<NAME>_<key>/; summary: python3 tools/pmc_pass_summary.py
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
name=$1; ctr=$2; shift 2
for key in "$@"; do
  args=$(python3 tools/pmc_key.py args "$key"); f=$(python3 tools/pmc_key.py file "$key")
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/pmc_${name}_$f -o run \
    --kernel-include-regex "k_seal|k_open" -- python3 bench.py --steps 12 --warmup 4 --no-cpu-baseline \
    --no-roundtrip $args > gpurun_out/pmc_${name}_$f.log 2>&1 || { tail -5 gpurun_out/pmc_${name}_$f.log; exit 6; }
done
exit 0
