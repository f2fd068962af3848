"""Full-size (2^20-frame) oracle parity for every benchmarked layout, built exactly as bench.py
builds it (bench.Workload), so the batches the bench lines time are the batches checked here.

The wire layouts run the EmitShiftLines emitter (bodies at any byte offset: class-permuted
waves, ds_bpermute'd bases, clipped edge units), which the other suites check only on a few
hundred frames; round 2 showed that emitter bugs can live in a single wave.  Cases:
  - the headline, configs[1]: 2^20 x 4 KiB into 4224-byte slots with MORE on every 8th frame
    (CurveClientMechanism.java:126-163 encode; the flags byte is box byte 32);
  - the dense wire layout: bodies back to back at a 4129-byte stride (V2Encoder.java:23-56
    writes them that way), seal and the open of the same dense bodies;
  - the Zipf batch, configs[3], at SURVEY.md 8(d) row 4's 8-byte offset table (input and
    output) and with bodies at 1-byte output offsets, seal and open.
Every body is compared with the multi-threaded oracle (cz_testlib.oracle_check_full); every
opened payload with the input and every status (CZ_STATUS_OK | flags << 8) with the sealed flags."""
import os
import sys

import numpy as np
import pytest

from cz_testlib import DESC_DTYPE, oracle_check_full

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FRAMES = 1 << 20


@pytest.fixture(scope="module")
def bench_mod():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    sys.path.insert(0, ROOT)
    import bench
    return bench


def _uniform_desc(wl):
    desc = np.zeros(wl.count, dtype=DESC_DTYPE)
    desc["in_off"] = np.arange(wl.count, dtype=np.uint64) * np.uint64(wl.in_stride)
    desc["out_off"] = np.arange(wl.count, dtype=np.uint64) * np.uint64(wl.out_stride)
    desc["len"] = wl.n
    desc["counter"] = wl.counter0 + np.arange(wl.count, dtype=np.uint64)
    desc["flags"] = (np.arange(wl.count) % 8 == 0).astype(np.uint32)  # bench.py: flags[::8] = 1
    desc["prev"] = -1
    return desc


def test_full_headline_4k_more_every_8th(bench_mod):
    """configs[1] exactly as timed: every frame against the oracle, slot padding zero."""
    import torch
    wl = bench_mod.Workload("4k", FRAMES, 0, torch.device("cuda:0"))
    assert wl.flags.cpu().numpy()[:16].tolist() == [1, 0, 0, 0, 0, 0, 0, 0] * 2
    wl.step()
    torch.cuda.synchronize()
    desc = _uniform_desc(wl)
    assert oracle_check_full(wl.d_in, wl.d_out, desc, bench_mod.PRECOM) == FRAMES
    assert not wl.d_out.view(wl.count, wl.out_stride)[:, wl.n + 33:].any()
    del wl
    torch.cuda.empty_cache()


def test_full_dense_4k_seal_and_open(bench_mod):
    """Bodies back to back (stride 4129 = 33 + 4096): every body against the oracle, then the
    open of the dense bodies (input at any byte offset) back to the payloads."""
    import torch
    from jeromq_amd import batch
    dev = torch.device("cuda:0")
    wl = bench_mod.Workload("4k_dense", FRAMES, 0, dev)
    assert wl.out_stride == 4129
    wl.step()
    torch.cuda.synchronize()
    desc = _uniform_desc(wl)
    assert oracle_check_full(wl.d_in, wl.d_out, desc, bench_mod.PRECOM) == FRAMES
    plain = torch.empty_like(wl.d_in)
    status = torch.full((wl.count,), -1, dtype=torch.int16, device=dev)
    batch.open_uniform(wl.d_out, wl.out_stride, plain, wl.in_stride, wl.count, wl.n + 33, wl.subkey,
                       wl.counter0 - 1, status)
    torch.cuda.synchronize()
    st = status.cpu().numpy().view(np.uint16)
    assert not np.any(st & 0xff)
    assert np.array_equal(st >> 8, desc["flags"].astype(np.uint16))
    assert torch.equal(plain, wl.d_in)
    del wl, plain
    torch.cuda.empty_cache()


@pytest.mark.parametrize("in_align,out_align", [(8, 8), (64, 1)])
def test_full_zipf_offset_tables_seal_and_open(bench_mod, in_align, out_align):
    """configs[3] with the 8-byte offset table of SURVEY.md 8(d) row 4 and with 1-byte output
    offsets: every body against the oracle; the segmented open of those bodies restores every
    payload with its flags."""
    import torch
    from jeromq_amd import batch
    dev = torch.device("cuda:0")
    wl = bench_mod.Workload("zipf", FRAMES, 0, dev, out_align=out_align, in_align=in_align)
    wl.step()
    torch.cuda.synchronize()
    desc = wl.desc_np
    if out_align == 1:  # bodies back to back: no slot padding anywhere
        assert np.array_equal(desc["out_off"][1:], desc["out_off"][:-1] + desc["len"][:-1] + np.uint64(33))
    assert oracle_check_full(wl.d_in, wl.d_out, desc, bench_mod.PRECOM) == FRAMES
    odesc = desc.copy()
    odesc["in_off"], odesc["out_off"] = desc["out_off"], desc["in_off"]
    odesc["len"] = desc["len"] + np.uint64(33)
    odesc["counter"] = desc["counter"] - np.uint64(1)  # replay floor = nonce - 1
    odesc["flags"] = 0x100                             # CZ_DESC_CHECK_NONCE
    d_odesc = torch.from_numpy(odesc.view(np.uint8).copy()).to(dev)
    oplan = batch.SegmentPlan(odesc, open_=True).to(dev)
    plain = torch.full_like(wl.d_in, 0x55)
    status = torch.full((wl.count,), -1, dtype=torch.int16, device=dev)
    batch.open_segments(d_odesc, oplan, wl.d_out, plain, wl.subkey.view(1, 32), status)
    torch.cuda.synchronize()
    st = status.cpu().numpy().view(np.uint16)
    assert not np.any(st & 0xff)
    assert np.array_equal(st >> 8, desc["flags"].astype(np.uint16))
    # payload lengths are 64-byte multiples, so the input slots hold no padding at these alignments
    assert int((desc["len"]).sum()) == wl.d_in.numel()
    assert torch.equal(plain, wl.d_in)
    del wl, plain
    torch.cuda.empty_cache()
