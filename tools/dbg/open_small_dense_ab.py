"""In-process A/B of cz_tune("open_ina") on the uniform open of 2^20 small bodies packed back to back
(100-byte payloads: 133-byte bodies at a 133-byte stride) into 128-byte plaintext slots (region staging).
usage: python tools/dbg/open_small_dense_ab.py"""
import os, sys
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, ROOT)
import torch
import bench
from jeromq_amd import batch, _lib
dev = torch.device("cuda:0")
count, n, stride, pstride = 1 << 20, 100, 133, 128
sk = batch.subkeys(torch.tensor(list(bench.PRECOM), dtype=torch.uint8, device=dev).view(1, 32), 0)[0].contiguous()
d_in = torch.empty(count * 112, dtype=torch.uint8, device=dev)
batch.fill(d_in, 9)
d_body = torch.empty(count * stride + 64, dtype=torch.uint8, device=dev)
batch.seal_uniform(d_in, 112, d_body, stride, count, n, sk, 3)
d_plain = torch.empty(count * pstride, dtype=torch.uint8, device=dev)
status = torch.empty(count, dtype=torch.int16, device=dev)
torch.cuda.synchronize()
step = lambda: batch.open_uniform(d_body, stride, d_plain, pstride, count, n + 33, sk, 2, status)
for rnd in (1, 2):
    for v in (0, 1):
        _lib.lib().cz_tune(b"open_ina", v)
        for _ in range(50):
            step()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            step()
        e1.record(); torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 50
        ok = bool(torch.equal(d_plain.view(count, pstride)[:, :n], d_in.view(count, 112)[:, :n])) and not bool((status & 0xff).any())
        print(f"open_ina={v} round {rnd}: {ms:.4f} ms {count * n / ms / 1e6 / 1.073741824:.1f} GiB/s ok {ok}", flush=True)
