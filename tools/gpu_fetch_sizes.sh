#!/bin/bash
# Read traffic by request size (round 5): TCC_EA0_RDREQ_{32B,64B,128B} give the bytes the L2 fetched
# exactly (32 n32 + 64 n64 + 128 n128), where FETCH_SIZE tallies every request at 64 B or 32 B and
# the MI355X guide's x2 correction holds only for all-128-B streams.  Plus L2 hit / miss counts.
#   bash tools/gpu_fetch_sizes.sh key1 key2 ...   (keys as tools/pmc_key.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_pmc_pass.sh rdsz "TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum" "$@" || exit $?
bash tools/gpu_pmc_pass.sh hit "TCC_HIT_sum TCC_MISS_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" "$@" || exit $?
python3 tools/pmc_pass_summary.py gpurun_out/pmc_rdsz_* gpurun_out/pmc_hit_* > gpurun_out/fetch_sizes.txt 2>&1
cat gpurun_out/fetch_sizes.txt
