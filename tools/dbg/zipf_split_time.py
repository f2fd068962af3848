"""Time the Zipf seal on sub-batches by frame length: how much of the kernel the short frames cost
against their share of the bytes.  usage: python tools/dbg/zipf_split_time.py [jmax ...]"""
import os, sys
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, ROOT)
import numpy as np, torch
import bench
from jeromq_amd import batch
dev = torch.device("cuda:0")
wl = bench.Workload("zipf", 1 << 20, 0, dev)
desc = wl.desc_np
sk = wl.subkey.view(1, 32)


def timeit(sub, reps=20):
    d_desc = torch.from_numpy(np.ascontiguousarray(sub).view(np.uint8).copy()).to(dev)
    plan = batch.SegmentPlan(sub, open_=False).to(dev)
    for _ in range(5):
        batch.seal_segments(d_desc, plan, wl.d_in, wl.d_out, sk)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    # ramp the clock
    for _ in range(30):
        batch.seal_segments(d_desc, plan, wl.d_in, wl.d_out, sk)
    e0.record()
    for _ in range(reps):
        batch.seal_segments(d_desc, plan, wl.d_in, wl.d_out, sk)
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps, plan.nseg


total_bytes = int(desc["len"].astype(np.uint64).sum())
ms, nseg = timeit(desc)
print(f"all: {len(desc)} frames {nseg} segs {ms:.3f} ms {total_bytes / ms / 1e6 / 1.073741824:.0f} GiB/s")
for jmax in [int(x) for x in sys.argv[1:]] or [2, 4, 8, 16, 64]:
    m = desc["len"] <= 64 * jmax
    for name, sub in ((f"len<={64*jmax}", desc[m]), (f"len>{64*jmax}", desc[~m])):
        b = int(sub["len"].astype(np.uint64).sum())
        t, ns = timeit(sub)
        print(f"{name:12s} frames {len(sub):8d} segs {ns:8d} bytes {b / total_bytes * 100:5.1f}% time {t:.3f} ms "
              f"({t / ms * 100:5.1f}% of all) {b / t / 1e6 / 1.073741824:7.0f} GiB/s")
