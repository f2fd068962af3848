#!/bin/bash
# LDS pressure of a bench config's kernels (one PMC pass each): bash tools/gpu_lds.sh 4k_dense 4k
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
P="SQ_LDS_UNALIGNED_STALL SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
for cfg in "$@"; do
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d gpurun_out/lds_${cfg} -o run --kernel-include-regex "k_seal|k_open" -- python3 bench.py --config $cfg --steps 6 --warmup 2 --ramp-ms 0 --no-cpu-baseline --no-roundtrip > gpurun_out/lds_${cfg}.log 2>&1 || { tail -5 gpurun_out/lds_${cfg}.log; exit 6; }
  python3 - "$cfg" <<'PY'
import csv, glob, sys, collections
cfg = sys.argv[1]
f = glob.glob(f"gpurun_out/lds_{cfg}/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(float); n = collections.Counter()
for r in csv.DictReader(open(f)):
    acc[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
d = {k: acc[k] / n[k] for k in acc}
w = d.get("SQ_WAVE_CYCLES", 1)
print(cfg, {k: f"{v:.3e}" for k, v in sorted(d.items())})
print(cfg, "fractions of SQ_WAVE_CYCLES:", {k: round(v / w, 4) for k, v in sorted(d.items()) if k != "SQ_WAVE_CYCLES"})
PY
done
exit 0
