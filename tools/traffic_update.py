"""Fold FETCH_SIZE/WRITE_SIZE passes (tools/gpu_traffic.sh) into profiles/pmc_traffic.json.

HBM bytes per launch = sum over the config's kernels of median(FETCH_SIZE)*1024*2 + median(WRITE_SIZE)*1024
(the MI355X guide's gfx950 correction: FETCH_SIZE reports half of a wide streaming read; WRITE_SIZE is
exact for 16-B-per-lane stores).  One launch of a config may be several kernels (segments + combine)."""
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
# the kernels that make up one timed launch of each config (setup kernels excluded)
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


def per_kernel(pmc, cfg):
    vals = collections.defaultdict(list)
    for f in glob.glob(os.path.join(root, f"traffic_{file_safe(cfg)}_{pmc}", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[-2].split("::")[-1] if "(" in r["Kernel_Name"] else r["Kernel_Name"]
            vals[name].append(float(r["Counter_Value"]))
    return {k: statistics.median(v) for k, v in vals.items()}


for cfg in cfgs:
    keep = KERNELS.get(parse(cfg)[0], ("k_",))
    fetch = {k: v for k, v in per_kernel("FETCH_SIZE", cfg).items() if k.startswith(keep)}
    write = {k: v for k, v in per_kernel("WRITE_SIZE", cfg).items() if k.startswith(keep)}
    if not fetch or not write:
        print(cfg, "no counter rows")
        continue
    fb = sum(v * 1024 * 2 for v in fetch.values())
    wb = sum(v * 1024 for v in write.values())
    entry = data.setdefault(cfg, {})
    entry.update({"hbm_bytes_per_launch": round(fb + wb), "fetch_bytes": round(fb), "write_bytes": round(wb),
                  "kernels": sorted(fetch), "source": f"tools/gpu_traffic.sh {cfg} (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE)",
                  # the machine code these counts belong to: bench.py marks them stale when the loaded
                  # library's code of these kernels differs
                  "traffic_kernel_sha256": kernel_code_sha256(LIB, sorted(fetch))})
    print(cfg, data[cfg])
json.dump(data, open(path, "w"), indent=1)
