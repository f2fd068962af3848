"""Summarise rocprofv3 --pmc CSVs written by tools/gpu_pmc.sh: mean counter per dispatch + derived rates."""
import collections
import csv
import glob
import os
import sys

root, tag = sys.argv[1], sys.argv[2]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)


def short(name):
    return name.split("(")[-2].split("::")[-1] if "(" in name else name


for d in sorted(glob.glob(os.path.join(root, tag + "_[0-9]*"))):
    for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
if not dur:
    sys.exit("no counter rows")
# report the dominant kernel (largest total profiled time); list the others
totals = {k: sum(v) for k, v in dur.items()}
kern = max(totals, key=totals.get)
for k in sorted(totals, key=totals.get, reverse=True):
    print(f"{'*' if k == kern else ' '} {k}: {len(dur[k])} counter rows, median {sorted(dur[k])[len(dur[k]) // 2] * 1e3:.3f} ms")
m = {c: sum(v) / len(v) for c, v in vals[kern].items()}
t = sorted(dur[kern])[len(dur[kern]) // 2]
print(f"kernel {kern} (median profiled dispatch) {t*1e3:.3f} ms")
for k in sorted(m):
    print(f"  {k:28s} {m[k]:.4e}")
if "GRBM_GUI_ACTIVE" in m:
    print(f"  clock ~ GRBM_GUI_ACTIVE/8/t = {m['GRBM_GUI_ACTIVE'] / 8 / t / 1e9:.3f} GHz")
if "FETCH_SIZE" in m:
    print(f"  FETCH_SIZE bytes/dispatch = {m['FETCH_SIZE'] * 1024:.4e} (x2 gfx950 correction for wide streams: "
          f"{m['FETCH_SIZE'] * 2048:.4e})")
if "WRITE_SIZE" in m:
    print(f"  WRITE_SIZE bytes/dispatch = {m['WRITE_SIZE'] * 1024:.4e}")
if "SQ_WAVE_CYCLES" in m:
    w = m["SQ_WAVE_CYCLES"]
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
        if k in m:
            print(f"  {k}/SQ_WAVE_CYCLES = {m[k] / w:.3f}")
if "SQ_INSTS_VALU" in m and "GRBM_GUI_ACTIVE" in m:
    cyc = m["GRBM_GUI_ACTIVE"] / 8
    print(f"  VALU wave-instr per SIMD per cycle = {m['SQ_INSTS_VALU'] / 1024 / cyc:.3f} (1 per 2 cycles = 0.5)")
if "TA_BUSY_avr" in m and "GRBM_GUI_ACTIVE" in m:
    print(f"  TA_BUSY_avr / (GRBM_GUI_ACTIVE/8) = {m['TA_BUSY_avr'] / (m['GRBM_GUI_ACTIVE'] / 8):.3f}")
