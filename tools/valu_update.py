"""Fold the instruction-count passes of tools/gpu_valu.sh into profiles/pmc_traffic.json.

Per config: wave-instructions per launch (VALU, SALU, LDS) summed over the config's kernels
(medians over dispatches), and the profiled clock GRBM_GUI_ACTIVE / 8 XCDs / kernel time of the
dominant kernel.  bench.py turns valu_insts_per_launch into the VALU issue roofline: every
int32 VALU wave-instruction occupies a SIMD for 4 cycles (tools/diag/salsa_ub.hip,
profiles/r01/ubench_salsa_issue.log), so the chip issues at most 1024 SIMDs x 2.4 GHz / 4."""
import collections
import csv
import glob
import json
import os
import statistics
import sys

root, cfgs = sys.argv[1], sys.argv[2:]
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_key import file_safe, parse  # noqa: E402
KERNELS = {"4k": ("k_seal_uniform",), "100b": ("k_seal_uniform",), "open4k": ("k_open_uniform",),
           "zipf": ("k_seal_segments", "k_seal_combine"), "zipf_lane": ("k_seal_desc",),
           "zipf_open": ("k_open_segments", "k_open_combine"),
           "4k_dense": ("k_seal_uniform",)}
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from jeromq_amd.build import PRODUCT_LIB, kernel_code_sha256  # noqa: E402
LIB = os.environ.get("CZ_LIB", PRODUCT_LIB)   # the library the passes ran (A/B builds set CZ_LIB)
path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
data = json.load(open(path)) if os.path.exists(path) else {}


def short(n):
    return n.split("(")[-2].split("::")[-1] if "(" in n else n


for cfg in cfgs:
    keep = KERNELS.get(parse(cfg)[0], ("k_",))
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for f in glob.glob(os.path.join(root, f"valu_{file_safe(cfg)}", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            if not k.startswith(keep):
                continue
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    if not vals:
        print(cfg, "no counter rows")
        continue
    med = {k: {c: statistics.median(v) for c, v in cs.items()} for k, cs in vals.items()}
    tot = lambda c: sum(m.get(c, 0.0) for m in med.values())  # noqa: E731
    dom = max(dur, key=lambda k: sum(dur[k]))
    t = statistics.median(dur[dom])
    entry = data.setdefault(cfg, {})
    entry.update({"valu_insts_per_launch": round(tot("SQ_INSTS_VALU")), "salu_insts_per_launch": round(tot("SQ_INSTS_SALU")),
                  "lds_insts_per_launch": round(tot("SQ_INSTS_LDS")),
                  "profiled_clock_ghz": round(med[dom].get("GRBM_GUI_ACTIVE", 0.0) / 8 / t / 1e9, 3),
                  "profiled_kernel_ms": round(t * 1e3, 4),
                  "valu_source": f"tools/gpu_valu.sh {cfg} (rocprofv3 --pmc SQ_INSTS_VALU ... GRBM_GUI_ACTIVE)",
                  "valu_kernels": sorted(med), "valu_kernel_sha256": kernel_code_sha256(LIB, sorted(med))})
    print(cfg, {k: entry[k] for k in entry if k.startswith(("valu", "salu", "lds", "profiled"))})
json.dump(data, open(path, "w"), indent=1)
