"""GPU parity for bodies at ANY byte offset: the shifted line emitter (EmitSegLines).

Dense output is what the wire needs (bodies back to back, or behind V2 headers,
V2Encoder.java:23-56): a 4 KiB body slot of 4129 bytes puts every frame at a
different byte phase of the 128-byte line.  Cases:
  * cz_seal_uniform at strides 4129 (dense), 4130, 4131, 4136, 4144 and 4226, and bodies back to
    back of 320 / 352 / 4033 / 333 / 1041 bytes (the round-5 whole-unit edges), at output
    bases shifted by 0..15 bytes, with a partial last wave: every body bit-exact against
    the oracle (CurveClientMechanism.encode -> Curve.afternm, Curve.java:129-137), and
    every byte between bodies left as the caller wrote it;
  * cz_seal_segments with ragged frames packed densely (byte offsets) and on the 8-byte
    offset table of SURVEY.md 8(d) row 4, short and long segments;
  * cz_open_segments writing plaintext densely (CurveClientMechanism.decode).
"""
import numpy as np
import pytest

from cz_testlib import DESC_DTYPE, load_golden, oracle, oracle_check_full, or_curve_encode, splitmix_bytes

pytestmark = pytest.mark.gpu

G = load_golden()
PRECOM = bytes.fromhex(G["keys"]["precom"])
SENTINEL = 0xA5


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch, torch.device("cuda:0")


@pytest.fixture(scope="module")
def subkeys(torch_dev):
    torch, dev = torch_dev
    from jeromq_amd import _lib, batch
    k = torch.tensor(list(PRECOM), dtype=torch.uint8, device=dev).view(1, 32)
    return torch.cat([batch.subkeys(k, _lib.CZ_DIR_C2S), batch.subkeys(k, _lib.CZ_DIR_S2C)])


def _gaps_untouched(out, spans, lo, hi):
    """bytes of out[lo:hi] outside every [s, e) span still hold the sentinel"""
    mask = np.ones(hi - lo, dtype=bool)
    for s, e in spans:
        mask[s - lo:e - lo] = False
    bad = np.nonzero(out[lo:hi][mask] != SENTINEL)[0]
    assert bad.size == 0, f"{bad.size} bytes outside the bodies were written (first at {lo + int(np.nonzero(mask)[0][bad[0]])})"


@pytest.mark.parametrize("n,stride", [(4096, 4129), (4096, 4130), (4096, 4131), (4096, 4136), (4096, 4144),
                                      (4096, 4226), (223, 256 + 5), (300, 333), (1000, 1041),
                                      # bodies back to back whose length is a 64-byte multiple (no edge
                                      # unit shared with the next body's header) or a 16-byte one
                                      (287, 320), (319, 352), (4000, 4033)])
@pytest.mark.parametrize("base", [0, 1, 8, 13])
def test_seal_uniform_any_offset(torch_dev, subkeys, n, stride, base):
    torch, dev = torch_dev
    from jeromq_amd import batch
    count = 64 * 5 + 17  # five full waves and a partial one
    in_stride = (n + 15) // 16 * 16
    hin = np.frombuffer(splitmix_bytes(count * in_stride, 1000 + n + stride), dtype=np.uint8).copy()
    d_in = torch.from_numpy(hin).to(dev)
    size = base + count * stride + 64
    d_buf = torch.full((size,), SENTINEL, dtype=torch.uint8, device=dev)
    d_out = d_buf[base:]
    flags = torch.tensor([(i % 3 == 0) | (2 if i % 5 == 0 else 0) for i in range(count)], dtype=torch.uint8, device=dev)
    c0 = 0xFFFFFFF0 - 100  # the high nonce word changes inside a wave
    batch.seal_uniform(d_in, in_stride, d_out, stride, count, n, subkeys[0], c0, flags8=flags)
    torch.cuda.synchronize()
    out = d_buf.cpu().numpy()
    fl = flags.cpu().numpy()
    spans = []
    for i in range(count):
        o = base + i * stride
        want = or_curve_encode(hin[i * in_stride:i * in_stride + n].tobytes(), int(fl[i]), c0 + i, 0, PRECOM)
        got = out[o:o + n + 33].tobytes()
        assert got == want, f"frame {i} (stride {stride}, base {base}) differs from the oracle"
        spans.append((o, o + n + 33))
    _gaps_untouched(out, spans, 0, size)


def _ragged(lens, out_round, in_align=64):
    """payloads on in_align boundaries, bodies packed at out_round-byte granularity (1 = dense)"""
    desc = np.zeros(len(lens), dtype=DESC_DTYPE)
    io = oo = 0
    for i, n in enumerate(lens):
        desc[i] = (io, oo, n, 0, 3 + i, 1 if i % 8 == 0 else 0, -1)
        io += (n + in_align - 1) // in_align * in_align
        oo += (n + 33 + out_round - 1) // out_round * out_round
    hin = np.zeros(io + 64, dtype=np.uint8)
    for i, n in enumerate(lens):
        o = int(desc[i]["in_off"])
        hin[o:o + n] = np.frombuffer(splitmix_bytes(n, 5 + 31 * i), dtype=np.uint8)
    return desc, hin, oo + 64


def _zipf_lens(count, seed):
    rng = np.random.default_rng(seed)
    j = rng.zipf(1.2, size=4 * count)
    j = j[j <= 1024][:count]
    return [int(64 * x) for x in j]


@pytest.mark.parametrize("out_round", [1, 8])
@pytest.mark.parametrize("seg_blocks", [3, 64])
def test_seal_segments_dense_outputs(torch_dev, subkeys, out_round, seg_blocks):
    torch, dev = torch_dev
    from jeromq_amd import batch
    lens = _zipf_lens(3000, 42) + [0, 1, 31, 65536, 4096, 4095, 100, 223]
    desc, hin, ob = _ragged(lens, out_round)
    plan = batch.SegmentPlan(desc, open_=False, seg_blocks=seg_blocks).to(dev)
    d_in = torch.from_numpy(hin).to(dev)
    d_out = torch.full((ob,), SENTINEL, dtype=torch.uint8, device=dev)
    d_desc = torch.from_numpy(desc.view(np.uint8).copy()).to(dev)
    batch.seal_segments(d_desc, plan, d_in, d_out, subkeys, desc_np=desc)
    torch.cuda.synchronize()
    assert oracle_check_full(d_in, d_out, desc, PRECOM) == len(desc)
    out = d_out.cpu().numpy()
    spans = [(int(d["out_off"]), int(d["out_off"]) + int(d["len"]) + 33) for d in desc]
    _gaps_untouched(out, spans, 0, ob)


@pytest.mark.parametrize("out_round", [1, 8])
def test_open_segments_dense_plaintext(torch_dev, subkeys, out_round):
    """bodies on 16-byte boundaries, plaintext packed densely: every payload recovered, gaps kept"""
    torch, dev = torch_dev
    from jeromq_amd import batch
    lens = _zipf_lens(2000, 7) + [0, 1, 65536, 4096]
    count = len(lens)
    desc = np.zeros(count, dtype=DESC_DTYPE)
    bodies, io = [], 0
    for i, n in enumerate(lens):
        p = splitmix_bytes(n, 900 + i)
        b = or_curve_encode(p, i & 1, 10 + i, 0, PRECOM)
        bodies.append((io, p, b))
        io += (len(b) + 15) // 16 * 16
    hin = np.zeros(io + 64, dtype=np.uint8)
    oo = 0
    for i, (o, p, b) in enumerate(bodies):
        hin[o:o + len(b)] = np.frombuffer(b, dtype=np.uint8)
        # the server opens client bodies: nonce floor 9 for the first, chained through prev
        desc[i] = (o, oo, len(b), 0, 9, 0, i - 1 if i else -1)
        oo += (len(p) + out_round - 1) // out_round * out_round if p else out_round
    desc["flags"] |= np.uint32(1 << 8)  # CZ_DESC_CHECK_NONCE
    ob = oo + 64
    plan = batch.SegmentPlan(desc, open_=True, seg_blocks=64).to(dev)
    d_out = torch.full((ob,), SENTINEL, dtype=torch.uint8, device=dev)
    status = torch.full((count,), -1, dtype=torch.int16, device=dev)
    batch.open_segments(torch.from_numpy(desc.view(np.uint8).copy()).to(dev), plan, torch.from_numpy(hin).to(dev),
                        d_out, subkeys, status, desc_np=desc)
    torch.cuda.synchronize()
    st = status.cpu().numpy().view(np.uint16)
    out = d_out.cpu().numpy()
    spans = []
    for i, (o, p, b) in enumerate(bodies):
        assert st[i] & 0xff == 0, f"frame {i}: status {st[i]:#x}"
        assert (st[i] >> 8) == (i & 1)
        s = int(desc[i]["out_off"])
        assert out[s:s + len(p)].tobytes() == p, f"frame {i} (len {len(p)}) plaintext differs"
        spans.append((s, s + len(p)))
    _gaps_untouched(out, spans, 0, ob)


@pytest.mark.parametrize("n,stride", [(4096, 4129), (4096, 4130), (4096, 4131), (4096, 4136), (4096, 4144),
                                      (300, 333), (1000, 1041), (100, 133), (100, 136)])
@pytest.mark.parametrize("base", [0, 1, 8, 13])
@pytest.mark.parametrize("layout", ["line", "shift"])
def test_open_uniform_any_offset(torch_dev, subkeys, n, stride, base, layout):
    """cz_open_uniform of bodies back to back at any byte phase (the receive side of the dense wire
    layout: V2Decoder.java:67-105 leaves bodies back to back; CurveClientMechanism.decode,
    :165-224) into line-aligned plaintext slots: the line path with dword-aligned loads.  Tampered
    frames report CZ_STATUS_CRYPTO and leave zeros; every other payload and flags byte comes back.
    layout="shift": plaintext slots that are not 128-byte multiples, 5 bytes off the buffer's line
    (byte-shifted line staging); the bytes between slots stay as the caller wrote them."""
    torch, dev = torch_dev
    from jeromq_amd import _lib, batch
    count = 64 * 5 + 17
    in_stride = (n + 15) // 16 * 16
    hin = np.frombuffer(splitmix_bytes(count * in_stride, 2000 + n + stride), dtype=np.uint8).copy()
    d_in = torch.from_numpy(hin).to(dev)
    size = base + count * stride + 64
    d_buf = torch.full((size,), SENTINEL, dtype=torch.uint8, device=dev)
    d_bodies = d_buf[base:]
    flags = torch.tensor([(i % 3 == 0) | (2 if i % 5 == 0 else 0) for i in range(count)], dtype=torch.uint8, device=dev)
    c0 = 0xFFFFFFF0 - 100  # the high nonce word changes inside a wave
    batch.seal_uniform(d_in, in_stride, d_bodies, stride, count, n, subkeys[0], c0, flags8=flags)
    torch.cuda.synchronize()
    bodies = d_buf.cpu().numpy()
    rng = np.random.default_rng(n + stride + base)
    bad = sorted(int(x) for x in rng.choice(count, size=9, replace=False))
    for j, i in enumerate(bad):  # tag, first / middle / last ciphertext byte
        where = [16 + j % 16, 33, (n + 33) // 2, n + 32][j % 4]
        bodies[base + i * stride + where] ^= 1 << (j % 8)
    d_buf.copy_(torch.from_numpy(bodies))
    if layout == "line":
        plain_stride, pbase = (n + 127) // 128 * 128, 0
    else:
        plain_stride, pbase = (n + 16 if n % 128 == 0 else n), 5
    d_pbuf = torch.full((pbase + count * plain_stride + 64,), SENTINEL, dtype=torch.uint8, device=dev)
    d_plain = d_pbuf[pbase:]
    status = torch.full((count,), -1, dtype=torch.int16, device=dev)
    batch.open_uniform(d_bodies, stride, d_plain, plain_stride, count, n + 33, subkeys[0], c0 - 1, status)
    torch.cuda.synchronize()
    st = status.cpu().numpy().view(np.uint16)
    pall = d_pbuf.cpu().numpy()
    plain = pall[pbase:]
    if layout == "shift":
        spans = [(pbase + i * plain_stride, pbase + i * plain_stride + n) for i in range(count)]
        _gaps_untouched(pall, spans, 0, len(pall))
    fl = flags.cpu().numpy()
    for i in range(count):
        p = plain[i * plain_stride:i * plain_stride + n]
        if i in bad:
            assert st[i] & 0xff == _lib.CZ_STATUS_CRYPTO, f"frame {i}"
            assert not p.any(), f"frame {i} leaked plaintext"
        else:
            assert st[i] & 0xff == _lib.CZ_STATUS_OK and st[i] >> 8 == fl[i], f"frame {i} status {st[i]:#x}"
            assert p.tobytes() == hin[i * in_stride:i * in_stride + n].tobytes(), f"frame {i} (stride {stride}, base {base})"


@pytest.mark.parametrize("n,in_stride,out_stride", [(4096, 4097, 4224), (4096, 4100, 4224), (4096, 4104, 4224),
                                                    (4096, 4097, 4129), (4096, 4104, 4136), (100, 100, 144),
                                                    (100, 101, 144), (1000, 1003, 1041), (64, 65, 112)])
@pytest.mark.parametrize("ibase", [0, 1, 3, 8])
def test_seal_uniform_unaligned_payloads(torch_dev, subkeys, n, in_stride, out_stride, ibase):
    """cz_seal_uniform of payloads packed at any byte offset (messages back to back in the caller's
    buffer): the staged kernels with dword-aligned loads and a per-frame funnel shift, every body
    against the oracle (CurveClientMechanism.encode), flags on some frames, the high nonce word
    changing inside a wave, and a partial last wave."""
    torch, dev = torch_dev
    from jeromq_amd import batch
    count = 64 * 5 + 17
    hbuf = np.frombuffer(splitmix_bytes(ibase + count * in_stride + 64, 3000 + n + in_stride + ibase),
                         dtype=np.uint8).copy()
    d_buf = torch.from_numpy(hbuf).to(dev)
    d_in = d_buf[ibase:]
    d_out = torch.full((count * out_stride + 64,), SENTINEL, dtype=torch.uint8, device=dev)
    flags = torch.tensor([(i % 3 == 0) | (2 if i % 7 == 0 else 0) for i in range(count)], dtype=torch.uint8, device=dev)
    c0 = 0xFFFFFFF0 - 200
    batch.seal_uniform(d_in, in_stride, d_out, out_stride, count, n, subkeys[0], c0, flags8=flags)
    torch.cuda.synchronize()
    out = d_out.cpu().numpy()
    fl = flags.cpu().numpy()
    for i in range(count):
        p = hbuf[ibase + i * in_stride:ibase + i * in_stride + n].tobytes()
        want = or_curve_encode(p, int(fl[i]), c0 + i, 0, PRECOM)
        assert out[i * out_stride:i * out_stride + n + 33].tobytes() == want, \
            f"frame {i} (in_stride {in_stride}, out_stride {out_stride}, ibase {ibase})"


@pytest.mark.parametrize("n,stride,base,tail", [(4096, 4129, 0, 37), (4096, 4129, 3, 0), (1024, 1064, 8, 21),
                                                (4096, 4136, 8, 5), (512, 545, 1, 64 * 3 + 1), (2048, 2082, 2, 9)])
@pytest.mark.parametrize("carry", [1, 2, 0])
def test_open_uniform_phase_sorted_carry(torch_dev, subkeys, n, stride, base, tail, carry):
    """The phase-sorted open of 8-byte aligned bodies (k_open_uniform_carry, cz_tune "open_carry"):
    whole blocks of 64 P frames, P = the period of the bodies' line phase (16 for a 4136 or 1064-byte
    stride), every wave one phase with the aligned lines carried; the frames after the last whole
    block go to k_open_uniform, whose first frame takes its replay floor from the body before it.
    Bodies at odd byte offsets (strides 4129, 545, 2082: P = 128 / 128 / 64) keep the straddling
    loads unless the knob is 2 (carried lines for INA 1, an A/B option), so they check both paths
    and the partial-wave slot contract.  Tampered frames inside carry waves and in the tail report
    CRYPTO with zeros; a replayed nonce on the first tail frame reports SEQUENCE; every other payload
    and flags byte comes back, with carry on and off."""
    torch, dev = torch_dev
    from jeromq_amd import _lib, batch
    g = np.gcd(stride % 128, 128) if stride % 128 else 128
    P = 128 // g
    count = 64 * P + tail
    in_stride = (n + 15) // 16 * 16
    hin = np.frombuffer(splitmix_bytes(count * in_stride, 3000 + n + stride), dtype=np.uint8).copy()
    d_in = torch.from_numpy(hin).to(dev)
    d_buf = torch.full((base + count * stride + 64,), SENTINEL, dtype=torch.uint8, device=dev)
    d_bodies = d_buf[base:]
    flags = torch.tensor([(i % 3 == 0) for i in range(count)], dtype=torch.uint8, device=dev)
    c0 = 0xFFFFFFF0 - 1000  # the high nonce word changes inside the batch
    batch.seal_uniform(d_in, in_stride, d_bodies, stride, count, n, subkeys[0], c0, flags8=flags)
    torch.cuda.synchronize()
    bodies = d_buf.cpu().numpy()
    rng = np.random.default_rng(n + stride + base)
    bad = sorted(set(int(x) for x in rng.choice(64 * P, size=7, replace=False)) | ({64 * P + tail // 2} if tail > 2 else set()))
    for j, i in enumerate(bad):  # tag, first / middle / last ciphertext byte
        where = [16 + j % 16, 33, (n + 33) // 2, n + 32][j % 4]
        bodies[base + i * stride + where] ^= 1 << (j % 8)
    replay = 64 * P if tail else None
    if replay is not None:   # the first tail frame repeats the nonce of the last carry frame
        o, p = base + replay * stride, base + (replay - 1) * stride
        bodies[o + 8:o + 16] = bodies[p + 8:p + 16]
    d_buf.copy_(torch.from_numpy(bodies))
    plain_stride = (n + 127) // 128 * 128
    d_plain = torch.full((count * plain_stride + 64,), SENTINEL, dtype=torch.uint8, device=dev)
    status = torch.full((count,), -1, dtype=torch.int16, device=dev)
    lib = _lib.lib()
    old = lib.cz_tune(b"open_carry", carry)
    try:
        batch.open_uniform(d_bodies, stride, d_plain, plain_stride, count, n + 33, subkeys[0], c0 - 1, status)
        torch.cuda.synchronize()
    finally:
        lib.cz_tune(b"open_carry", old)
    st = status.cpu().numpy().view(np.uint16)
    plain = d_plain.cpu().numpy()
    fl = flags.cpu().numpy()
    for i in range(count):
        p = plain[i * plain_stride:i * plain_stride + n]
        if i in bad:
            assert st[i] & 0xff == _lib.CZ_STATUS_CRYPTO, f"frame {i} status {st[i]:#x}"
            assert not p.any(), f"frame {i} leaked plaintext"
        elif i == replay:
            assert st[i] & 0xff == _lib.CZ_STATUS_SEQUENCE, f"replayed frame {i} status {st[i]:#x}"
            assert not p.any(), f"frame {i} leaked plaintext"
        else:
            assert st[i] & 0xff == _lib.CZ_STATUS_OK and st[i] >> 8 == fl[i], f"frame {i} status {st[i]:#x}"
            assert p.tobytes() == hin[i * in_stride:i * in_stride + n].tobytes(), f"frame {i}"
        assert not plain[i * plain_stride + n:(i + 1) * plain_stride].any(), f"slot {i} padding"


# EmitShiftLinesT keeps flag bits 28..31 above an output's end d + total, so the
# launchers send one frame to the byte-shifted emitter only while d + total < 2^28
# (SHIFT_TOTAL_MAX = 2^28 - 128 in cz_kernels.hip).  One frame at the bound (shifted emitter, its
# end field at 2^28 - 1 with d = 127) and one just above it (lane-wise stores), output 127 bytes
# into a line, 16-byte aligned payload: the whole body against the oracle, the bytes around it kept.
SHIFT_TOTAL_MAX = (1 << 28) - 128


@pytest.mark.parametrize("total", [SHIFT_TOTAL_MAX, SHIFT_TOTAL_MAX + 1])
def test_seal_uniform_single_frame_at_shift_bound(torch_dev, subkeys, total):
    torch, dev = torch_dev
    from jeromq_amd import batch
    n = total - 33
    base = 127
    hin = np.frombuffer(splitmix_bytes(n, 4242), dtype=np.uint8)
    d_in = torch.from_numpy(hin.copy()).to(dev)
    d_buf = torch.full((base + total + 64,), SENTINEL, dtype=torch.uint8, device=dev)
    flags = torch.tensor([1], dtype=torch.uint8, device=dev)
    batch.seal_uniform(d_in, (n + 15) // 16 * 16, d_buf[base:], total, 1, n, subkeys[0], 77, flags8=flags)
    torch.cuda.synchronize()
    out = d_buf.cpu().numpy()
    want = or_curve_encode(hin.tobytes(), 1, 77, 0, PRECOM)
    assert out[base:base + total].tobytes() == want, f"single {n}-byte frame differs from the oracle"
    _gaps_untouched(out, [(base, base + total)], 0, len(out))


@pytest.mark.parametrize("nout", [SHIFT_TOTAL_MAX, SHIFT_TOTAL_MAX + 1])
def test_open_uniform_single_frame_at_shift_bound(torch_dev, subkeys, nout):
    torch, dev = torch_dev
    from jeromq_amd import _lib, batch
    p = np.frombuffer(splitmix_bytes(nout, 4343), dtype=np.uint8)
    body = or_curve_encode(p.tobytes(), 0, 90, 0, PRECOM)
    d_body = torch.from_numpy(np.frombuffer(body, dtype=np.uint8).copy()).to(dev)
    base = 127
    d_buf = torch.full((base + nout + 64,), SENTINEL, dtype=torch.uint8, device=dev)
    status = torch.full((1,), -1, dtype=torch.int16, device=dev)
    batch.open_uniform(d_body, len(body), d_buf[base:], nout, 1, len(body), subkeys[0], 89, status)
    torch.cuda.synchronize()
    assert int(status.cpu().numpy().view(np.uint16)[0]) & 0xff == _lib.CZ_STATUS_OK
    out = d_buf.cpu().numpy()
    assert out[base:base + nout].tobytes() == p.tobytes(), f"single {nout}-byte plaintext differs"
    _gaps_untouched(out, [(base, base + nout)], 0, len(out))
