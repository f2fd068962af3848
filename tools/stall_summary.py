"""Summary of tools/gpu_stall.sh: medians over the last 8 dispatches of the config's main
kernel, each SQ counter as a fraction of SQ_WAVE_CYCLES (wave-cycles the kernel's waves lived)."""
import collections
import csv
import glob
import os
import statistics
import sys

root, cfg = sys.argv[1], sys.argv[2]
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_key import file_safe, parse  # noqa: E402
KERNEL = {"4k": "k_seal_uniform", "4k_dense": "k_seal_uniform", "100b": "k_seal_uniform", "open4k": "k_open_uniform",
          "zipf": "k_seal_segments_lines"}[parse(cfg)[0]]
vals = collections.defaultdict(list)
for p in (1, 2):
    rows = collections.defaultdict(dict)
    for f in glob.glob(os.path.join(root, f"stall_{file_safe(cfg)}_{p}", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if KERNEL in r["Kernel_Name"]:
                rows[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    for d in [rows[k] for k in sorted(rows)][-8:]:
        for c, v in d.items():
            vals[c].append(v)
med = {c: statistics.median(v) for c, v in vals.items()}
wc = med.get("SQ_WAVE_CYCLES", 0.0)
print(f"{cfg} ({KERNEL}): SQ_WAVE_CYCLES {wc:.4g}")
for c in sorted(med):
    if c != "SQ_WAVE_CYCLES":
        print(f"  {c:32s} {med[c]:12.4g}  {med[c] / wc if wc else 0:8.4f} of wave-cycles")
