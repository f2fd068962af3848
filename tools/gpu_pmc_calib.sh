#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration on kernels with known byte counts (tools/diag):
#   k_read_lanewise  : 4 GiB read, lane-wise 16 B
#   k_copy_coal4     : 4 GiB read + 4 GiB write, coalesced
#   k_write_seg<8>   : 4 GiB written as whole 128 B lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for pmc in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 240 rocprofv3 --pmc $pmc --output-format csv -d gpurun_out/calib_$pmc -o run --kernel-include-regex "k_read_lanewise|k_copy_coal4|k_write_seg" -- ./tools/diag/diag > gpurun_out/calib_$pmc.log 2>&1
  rc=$?; [ $rc -lt 124 ] || exit $rc
done
python3 - <<'PY'
import csv, glob, collections
for pmc in ("FETCH_SIZE", "WRITE_SIZE"):
    agg = collections.defaultdict(list)
    for f in glob.glob(f"gpurun_out/calib_{pmc}/*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            agg[r["Kernel_Name"][:60]].append(float(r["Counter_Value"]) * 1024)
    for k, v in sorted(agg.items()):
        print(f"{pmc:10s} {k:60s} n={len(v):2d} mean bytes={sum(v)/len(v):.4e}  (4 GiB = 4.295e9)")
PY
