"""In-process A/B of cz_tune("seal_ina") on a 2^20-frame Zipf batch whose payload lengths are not
64-byte multiples and are packed back to back (1-byte offsets) or at 8 bytes; bodies into 128-byte
slots.  usage: python tools/dbg/zipf_unaligned_seal.py [in_round ...]"""
import os, sys
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, ROOT)
import numpy as np, torch
from jeromq_amd import batch, _lib
import bench
dev = torch.device("cuda:0")
rng = np.random.default_rng(42)
j = np.empty(0, dtype=np.int64)
while len(j) < (1 << 20):
    z = rng.zipf(1.2, size=1 << 20)
    j = np.concatenate([j, z[z <= 1024]])
lens = (64 * j[:1 << 20] - rng.integers(0, 64, size=1 << 20)).astype(np.uint64)
sk = batch.subkeys(torch.tensor(list(bench.PRECOM), dtype=torch.uint8, device=dev).view(1, 32), 0)
for r in [int(x) for x in sys.argv[1:]] or [1, 8, 16]:
    ir = np.uint64(r)
    in_len = (lens + ir - np.uint64(1)) // ir * ir
    out_len = (lens + np.uint64(33 + 127)) // np.uint64(128) * np.uint64(128)
    desc = np.zeros(len(lens), dtype=batch.DESC_DTYPE)
    desc["in_off"][1:] = np.cumsum(in_len[:-1])
    desc["out_off"][1:] = np.cumsum(out_len[:-1])
    desc["len"] = lens
    desc["counter"] = 3 + np.arange(len(lens), dtype=np.uint64)
    desc["prev"] = -1
    d_in = torch.empty(int(in_len.sum()) + 64, dtype=torch.uint8, device=dev)
    batch.fill(d_in, 7)
    d_out = torch.empty(int(out_len.sum()) + 64, dtype=torch.uint8, device=dev)
    d_desc = torch.from_numpy(desc.view(np.uint8).copy()).to(dev)
    plan = batch.SegmentPlan(desc, open_=False).to(dev)
    pay = float(lens.sum()) / 2**30
    for rnd in (1, 2):
        res = {}
        for v in (0, 1):
            _lib.lib().cz_tune(b"seal_ina", v)
            for _ in range(20):
                batch.seal_segments(d_desc, plan, d_in, d_out, sk)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                batch.seal_segments(d_desc, plan, d_in, d_out, sk)
            e1.record(); torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 20
            res[v] = (ms, pay / ms * 1e3)
        print(f"in_round {r:2d} round {rnd}: seal_ina=0 {res[0][0]:.3f} ms {res[0][1]:.0f} GiB/s | "
              f"seal_ina=1 {res[1][0]:.3f} ms {res[1][1]:.0f} GiB/s", flush=True)
    del d_in, d_out
    torch.cuda.empty_cache()
