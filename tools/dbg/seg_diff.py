"""Map mismatches between segmented and lane-per-frame seal to frames/segments."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import numpy as np, torch
from cz_testlib import DESC_DTYPE, load_golden, splitmix_bytes
from jeromq_amd import batch, _lib
G = load_golden(); PRECOM = bytes.fromhex(G["keys"]["precom"])
dev = torch.device("cuda:0")
k = torch.tensor(list(PRECOM), dtype=torch.uint8, device=dev).view(1, 32)
sk = torch.cat([batch.subkeys(k, 0), batch.subkeys(k, 1)])
rng = np.random.default_rng(7)
j = np.clip(rng.zipf(1.2, size=4000), 1, 1024)
lens = [int(x) for x in (64 * j - rng.integers(0, 64, size=len(j)))]
desc = np.zeros(len(lens), dtype=DESC_DTYPE); io = oo = 0
for i, n in enumerate(lens):
    desc[i] = (io, oo, n, 0, 7 + 3 * i, i & 3, -1); io += (n + 15) // 16 * 16; oo += (n + 33 + 15) // 16 * 16
hin = np.zeros(io + 64, dtype=np.uint8)
for i, n in enumerate(lens):
    o = int(desc[i]["in_off"]); hin[o:o + n] = np.frombuffer(splitmix_bytes(n, 5 + 77 * i), dtype=np.uint8)
ob = oo + 64
d_desc = torch.from_numpy(desc.view(np.uint8).copy()).to(dev); d_in = torch.from_numpy(hin).to(dev)
ref = torch.zeros(ob, dtype=torch.uint8, device=dev)
batch.seal_batch(d_desc, len(desc), d_in, ref, sk)
for lines, pair in ((1, 1), (1, 0), (0, 1)):
    _lib.lib().cz_tune(b"seglines", lines); _lib.lib().cz_tune(b"pair", pair)
    plan = batch.SegmentPlan(desc, open_=False, seg_blocks=64).to(dev)
    out = torch.zeros(ob, dtype=torch.uint8, device=dev)
    batch.seal_segments(d_desc, plan, d_in, out, sk)
    torch.cuda.synchronize()
    a, b = out.cpu().numpy(), ref.cpu().numpy()
    bad = np.nonzero(a != b)[0]
    print(f"lines={lines} pair={pair}: {len(bad)} bad bytes")
    if len(bad):
        fr = np.searchsorted(desc["out_off"].astype(np.int64), bad, side="right") - 1
        for f in np.unique(fr)[:10]:
            offs = bad[fr == f] - int(desc[f]["out_off"])
            segs = [(int(s["first_block"]), int(s["nblocks"]), int(s["part"])) for s in plan.segments if s["frame"] == f]
            pos = [int(np.nonzero(plan.segments["frame"] == f)[0][0])]
            print(f"  frame {f} len {lens[f]} body {lens[f]+33} bad offs {offs.min()}..{offs.max()} n={len(offs)} segs {segs[:3]} seg-index {pos}")
