"""Diagnostic: which frames / bytes of the counter-high-word open case differ (CZ_LIB selects the build)."""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from jeromq_amd import batch, _lib  # noqa: E402
PRECOM = bytes.fromhex("0e8790cb0dc8703af2533cc8594eecfbf62ca560a66ebee1259cc0a30435c6f3")

dev = torch.device("cuda:0")
key = torch.tensor(list(PRECOM), dtype=torch.uint8, device=dev).view(1, 32)
sub = batch.subkeys(key, _lib.CZ_DIR_C2S)[0].contiguous()
n, ist, ost, count = 4096, 4096, 4224, 1088
for counter0 in (2**32 - 100, 2**32 + 7, 5):
    d_in = torch.empty(count * ist, dtype=torch.uint8, device=dev)
    batch.fill(d_in, 0x5EED1000 + n)
    flags = torch.zeros(count, dtype=torch.uint8, device=dev)
    flags[::8] = 1
    d_out = torch.full((count * ost,), 0xAB, dtype=torch.uint8, device=dev)
    batch.seal_uniform(d_in, ist, d_out, ost, count, n, sub, counter0, flags8=flags)
    for rep in range(2):
        d_plain = torch.zeros(count * ist, dtype=torch.uint8, device=dev)
        status = torch.full((count,), -1, dtype=torch.int16, device=dev)
        batch.open_uniform(d_out, ost, d_plain, ist, count, n + 33, sub, counter0 - 1, status)
        torch.cuda.synchronize()
        got = d_plain.cpu().numpy().reshape(count, ist)
        want = d_in.cpu().numpy().reshape(count, ist)
        diff = got != want
        bad = np.nonzero(diff.any(axis=1))[0]
        print(f"counter0={counter0:#x} rep {rep}: {len(bad)} bad frames {bad[:10]}...{bad[-3:] if len(bad) else ''}")
        if len(bad):
            f = bad[0]
            pos = np.nonzero(diff[f])[0]
            print("  frame", f, "bad bytes", len(pos), "first", pos[:8], "last", pos[-4:],
                  "64B blocks", np.unique(pos // 64)[:20])
            print("  got ", got[f, pos[0]:pos[0] + 16].tobytes().hex())
            print("  want", want[f, pos[0]:pos[0] + 16].tobytes().hex())
