"""Summarise tools/gpu_pmc_pass.sh output: per directory, the dominant kernel's counters averaged
over its dispatches (and divided by SQ_WAVE_CYCLES when that counter was collected).
usage: python3 tools/pmc_pass_summary.py gpurun_out/pmc_NAME_*"""
import collections
import csv
import glob
import os
import sys

for d in sys.argv[1:]:
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    if not rows:
        print(d, "no counter csv")
        continue
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in rows:
        per[(r["Kernel_Name"][:60], r["Dispatch_Id"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    kern = collections.Counter(k for k, _ in per)
    top = kern.most_common(1)[0][0]
    acc = collections.defaultdict(list)
    for (k, _), ctrs in per.items():
        if k == top:
            for c, v in ctrs.items():
                acc[c].append(sum(v))
    wc = sum(acc["SQ_WAVE_CYCLES"]) / len(acc["SQ_WAVE_CYCLES"]) if "SQ_WAVE_CYCLES" in acc else None
    print(f"{os.path.basename(d)}: {top} ({len(acc[next(iter(acc))])} dispatches)")
    for c in sorted(acc):
        m = sum(acc[c]) / len(acc[c])
        print(f"  {c:32s} {m:12.4g}" + (f"   {m / wc:.4f} of wave-cycles" if wc and c != "SQ_WAVE_CYCLES" else ""))
