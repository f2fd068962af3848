"""Where a full-size Zipf seal differs from the oracle: frames, segments, bad 16-byte units.
usage: python tools/dbg/zipf_full_diff.py IN_ALIGN OUT_ALIGN [max_frames]"""
import os, sys
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np, torch
import bench
from cz_testlib import oracle
ia, oa = int(sys.argv[1]), int(sys.argv[2]); maxf = int(sys.argv[3]) if len(sys.argv) > 3 else 12
dev = torch.device("cuda:0")
wl = bench.Workload("zipf", 1 << 20, 0, dev, out_align=oa, in_align=ia)
wl.step(); torch.cuda.synchronize()
desc = wl.desc_np; n = len(desc)
segs = wl.plan.segments if hasattr(wl.plan, "segments") else None
blen = desc["len"].astype(np.uint64) + np.uint64(33)
pk = np.frombuffer(bench.PRECOM, dtype=np.uint8).copy()
a = 0; nbad = 0; chunk = 256 << 20
while a < n and nbad < maxf:
    o0 = int(desc["out_off"][a]); b = max(int(np.searchsorted(desc["out_off"], np.uint64(o0 + chunk), side="left")), a + 1)
    i0 = int(desc["in_off"][a]); i1 = int((desc["in_off"][a:b] + desc["len"][a:b].astype(np.uint64)).max())
    o1 = int((desc["out_off"][a:b] + blen[a:b]).max())
    hin = wl.d_in[i0:i1].cpu().numpy(); got = wl.d_out[o0:o1].cpu().numpy(); want = got.copy()
    cd = desc[a:b].copy(); cd["in_off"] -= np.uint64(i0); cd["out_off"] -= np.uint64(o0)
    oracle().or_seal_batch(cd.ctypes.data, b - a, hin.ctypes.data, want.ctypes.data, pk.ctypes.data, 0, 16)
    if not np.array_equal(got, want):
        for k in range(a, b):
            s0, s1 = int(cd["out_off"][k - a]), int(cd["out_off"][k - a] + blen[k])
            d = np.nonzero(got[s0:s1] != want[s0:s1])[0]
            if len(d) == 0: continue
            nbad += 1
            units = sorted(set((d // 16).tolist()))
            oo = int(desc["out_off"][k])
            sg = [(int(segs[i]["first_block"]), int(segs[i]["nblocks"]), int(i)) for i in np.nonzero(segs["frame"] == k)[0]] if segs is not None else []
            print(f"frame {k} len {int(desc['len'][k])} out_off%128={oo % 128} bad bytes {len(d)} units {units[:12]}{'...' if len(units) > 12 else ''} "
                  f"(byte {d.min()}..{d.max()}) segs {sg[:8]}")
            if nbad <= 3:
                gf, wf = got[s0:s1], want[s0:s1]
                starts = [u for u in units if u - 1 not in units][:6]
                for u in starts:
                    g16 = gf[16 * u + 8:16 * u + 24].tobytes()
                    hits = [h - (16 * u + 8) for h in range(0, len(wf) - 16) if wf[h:h + 16].tobytes() == g16][:4]
                    ghits = [h - (16 * u + 8) for h in range(0, len(gf) - 16) if gf[h:h + 16].tobytes() == g16 and h != 16 * u + 8][:4]
                    print(f"   unit {u}: got {g16.hex()[:24]} want {wf[16*u+8:16*u+24].tobytes().hex()[:24]} found in want at delta {hits} in got at {ghits}")
            if nbad >= maxf: break
    a = b
print("bad frames listed:", nbad)
