"""In-process A/B of the segment kernels' SHIFT16 rule (cz_tune "shift16": 16-byte aligned outputs not
on 128-byte lines through EmitShiftLines instead of EmitSegLines), seal and open of the Zipf batch.
usage: KNOB=shift16|open_ina python tools/dbg/seg_shift16_ab.py [out_align ...]"""
import os, sys
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, ROOT)
import numpy as np, torch
import bench
from jeromq_amd import batch, _lib
dev = torch.device("cuda:0")


def timed(fn, reps=20):
    for _ in range(30):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


for oa in [int(x) for x in sys.argv[1:]] or [16, 8, 128]:
    wl = bench.Workload("zipf", 1 << 20, 0, dev, out_align=oa, in_align=8 if oa == 8 else 64)
    desc = wl.desc_np
    pay = int(desc["len"].astype(np.uint64).sum()) / 2**30
    odesc = desc.copy()
    odesc["in_off"], odesc["out_off"] = desc["out_off"], desc["in_off"]
    odesc["len"] = desc["len"] + np.uint64(33)
    odesc["counter"] = desc["counter"] - np.uint64(1)
    odesc["flags"] = 0x100
    d_odesc = torch.from_numpy(odesc.view(np.uint8).copy()).to(dev)
    oplan = batch.SegmentPlan(odesc, open_=True).to(dev)
    plain = torch.empty_like(wl.d_in)
    status = torch.empty((wl.count,), dtype=torch.int16, device=dev)
    wl.step(); torch.cuda.synchronize()
    op = lambda: batch.open_segments(d_odesc, oplan, wl.d_out, plain, wl.subkey.view(1, 32), status)
    for rnd in (1, 2):
        for v in (0, 1):
            _lib.lib().cz_tune(os.environ.get("KNOB", "shift16").encode(), v)
            ts = timed(wl.step)
            to = timed(op)
            ok = bool(torch.equal(plain, wl.d_in)) and not bool((status & 0xff).any())
            print(f"out_align {oa:3d} {os.environ.get('KNOB', 'shift16')}={v} round {rnd}: seal {ts:.4f} ms {pay / ts * 1e3:7.1f} GiB/s | "
                  f"open {to:.4f} ms {pay / to * 1e3:7.1f} GiB/s, plaintext ok {ok}", flush=True)
    del wl, plain
    torch.cuda.empty_cache()
