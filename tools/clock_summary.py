"""Per-library summary of tools/gpu_clock_ab.sh: HIP-event kernel ms from the bench line, and
from the PMC pass the median over the last 10 dispatches of VALU wave-instructions, kernel ms
and clock = GRBM_GUI_ACTIVE / 8 XCDs / duration (as tools/valu_update.py)."""
import collections
import csv
import glob
import json
import os
import statistics
import sys

root, tag = sys.argv[1], sys.argv[2]
cfg = sys.argv[3] if len(sys.argv) > 3 else "4k"
KERNEL = {"4k": "k_seal_uniform", "100b": "k_seal_uniform", "open4k": "k_open_uniform", "zipf": "k_seal_segments_lines"}[cfg]
line = json.loads(open(os.path.join(root, f"clk_{tag}.log")).read().strip().splitlines()[-1])
rows = collections.defaultdict(dict)
for f in glob.glob(os.path.join(root, f"clkpmc_{tag}", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if KERNEL not in r["Kernel_Name"]:
            continue
        d = rows[int(r["Dispatch_Id"])]
        d[r["Counter_Name"]] = float(r["Counter_Value"])
        d["t"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
last = [rows[k] for k in sorted(rows)][-10:]
if not last:
    print(tag, "no counter rows")
    sys.exit(0)
t = statistics.median(d["t"] for d in last)
clk = statistics.median(d.get("GRBM_GUI_ACTIVE", 0.0) / 8 / d["t"] / 1e9 for d in last)
valu = statistics.median(d.get("SQ_INSTS_VALU", 0.0) for d in last)
busy = valu * 4 / 1024 / (clk * 1e9) / t if clk else 0.0
print(f"{tag} {cfg} ({KERNEL}): bench kernel {line['roofline']['kernel_ms']:.4f} ms ({line['value']:.0f} GiB/s) | profiled "
      f"{t * 1e3:.4f} ms, clock {clk:.3f} GHz, VALU {valu:.4g}, VALU busy at that clock {busy:.3f}")
