"""GPU parity for cz_seal_uniform_box: the uniform seal from input in the reference's own box layout.

CurveClientMechanism.encode (CurveClientMechanism.java:144-153) builds m = 0^32 || flags || payload
and hands it to Curve.afternm (Curve.java:134-137); cz_seal_uniform_box reads that buffer where it
lies.  Every body is compared with the oracle's MESSAGE encoding of (payload, box byte 32 as the
flags, counter), bit-exact; box bytes 0..31 are filled with garbage to pin that they are not read.
Cases: payloads around the block and line edges, partial and full waves, 128-byte output slots
(line staging) and 16-byte slots (direct stores), and the full 2^20 x 4 KiB batch as bench.py's
4k_box line builds it."""
import os
import sys

import numpy as np
import pytest

from cz_testlib import DESC_DTYPE, load_golden, oracle_check_full, or_curve_encode

pytestmark = pytest.mark.gpu
G = load_golden()
PRECOM = bytes.fromhex(G["keys"]["precom"])
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def dev_subkey():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from jeromq_amd import _lib, batch
    dev = torch.device("cuda:0")
    k = torch.tensor(list(PRECOM), dtype=torch.uint8, device=dev).view(1, 32)
    return torch, dev, batch.subkeys(k, _lib.CZ_DIR_C2S)[0].contiguous()


@pytest.mark.parametrize("n", [0, 1, 30, 31, 63, 94, 95, 96, 127, 200, 1000, 4096, 5000])
@pytest.mark.parametrize("count,lines", [(1, True), (63, True), (64, True), (300, True), (130, False)])
def test_seal_uniform_box_vs_oracle(dev_subkey, n, count, lines):
    torch, dev, sub = dev_subkey
    from jeromq_amd import batch
    rng = np.random.default_rng(n * 1000 + count)
    box_stride = (n + 33 + 15) // 16 * 16 + (16 if count % 2 else 0)
    out_stride = (n + 33 + 127) // 128 * 128 if lines else (n + 33 + 15) // 16 * 16
    hbox = rng.integers(0, 256, size=count * box_stride, dtype=np.uint8)  # bytes 0..31: garbage
    flags = rng.integers(0, 4, size=count, dtype=np.uint8)
    hbox.reshape(count, box_stride)[:, 32] = flags
    d_box = torch.from_numpy(hbox).to(dev)
    d_out = torch.full((count * out_stride,), 0xA5, dtype=torch.uint8, device=dev)
    counter0 = 3 if count != 300 else (1 << 32) - 100  # 300: the high nonce word changes inside a wave
    batch.seal_uniform_box(d_box, box_stride, d_out, out_stride, count, n, sub, counter0)
    torch.cuda.synchronize()
    out = d_out.cpu().numpy()
    for i in range(count):
        o = i * box_stride
        want = or_curve_encode(hbox[o + 33:o + 33 + n].tobytes(), int(flags[i]), counter0 + i, 0, PRECOM)
        got = out[i * out_stride:i * out_stride + n + 33].tobytes()
        assert got == want, f"frame {i} of {count} (n={n}) differs from the oracle"


def test_full_box_layout_4k(dev_subkey):
    """bench.py's 4k_box line exactly as timed: every one of 2^20 bodies against the oracle."""
    torch, dev, _ = dev_subkey
    sys.path.insert(0, ROOT)
    import bench
    wl = bench.Workload("4k_box", 1 << 20, 0, dev)
    wl.step()
    torch.cuda.synchronize()
    desc = np.zeros(wl.count, dtype=DESC_DTYPE)
    desc["in_off"] = np.arange(wl.count, dtype=np.uint64) * np.uint64(wl.in_stride) + np.uint64(33)
    desc["out_off"] = np.arange(wl.count, dtype=np.uint64) * np.uint64(wl.out_stride)
    desc["len"] = wl.n
    desc["counter"] = wl.counter0 + np.arange(wl.count, dtype=np.uint64)
    desc["flags"] = (np.arange(wl.count) % 8 == 0).astype(np.uint32)
    desc["prev"] = -1
    assert oracle_check_full(wl.d_in, wl.d_out, desc, bench.PRECOM) == wl.count
    assert not wl.d_out.view(wl.count, wl.out_stride)[:, wl.n + 33:].any()
    del wl
    torch.cuda.empty_cache()
