"""GPU parity for segmented ragged batches (cz_seal_segments / cz_open_segments).

Long frames are split across lanes and their Poly1305 partials joined by the
combine kernels; the output contract is cz_seal_batch's / cz_open_batch's, so
every case is checked bit-exact against the CPU oracle (seal: or_seal_batch;
open: or_curve_decode semantics via the golden statuses) and against the
one-lane-per-frame kernels.  Small seg_blocks values put segment boundaries
inside short frames, so every boundary/tail position is reached cheaply.
"""
import numpy as np
import pytest

from cz_testlib import DESC_DTYPE, load_golden, oracle, oracle_check_full, or_curve_encode, splitmix_bytes

pytestmark = pytest.mark.gpu

G = load_golden()
PRECOM = bytes.fromhex(G["keys"]["precom"])


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch, torch.device("cuda:0")


@pytest.fixture(scope="module")
def L():
    from jeromq_amd import _lib
    return _lib


@pytest.fixture(scope="module")
def subkeys(torch_dev, L):
    torch, dev = torch_dev
    from jeromq_amd import batch
    k = torch.tensor(list(PRECOM), dtype=torch.uint8, device=dev).view(1, 32)
    return torch.cat([batch.subkeys(k, L.CZ_DIR_C2S), batch.subkeys(k, L.CZ_DIR_S2C)])


def _boundary_lengths(seg_blocks):
    """Payload lengths whose box (n + 33 bytes) ends at every interesting offset
    around segment boundaries, plus short frames that are never split."""
    lens = [0, 1, 31, 64, 100, 4096]
    for nblk in sorted({seg_blocks + seg_blocks // 2, seg_blocks + seg_blocks // 2 + 1, 2 * seg_blocks,
                        2 * seg_blocks + 1, 3 * seg_blocks - 1, 5 * seg_blocks + 2, 1025}):
        for r in (0, 1, 15, 16, 17, 31, 32, 33, 48, 63):
            mlen = 64 * (nblk - 1) + (r if r else 64)
            if mlen >= 33:
                lens.append(mlen - 33)
    lens.append(65536)
    return lens


def _pack(lens, shift=0, seed=0):
    desc = np.zeros(len(lens), dtype=DESC_DTYPE)
    io, oo = shift, 2 * shift + 1 if shift else 0
    for i, n in enumerate(lens):
        desc[i] = (io, oo, n, 0, 7 + 3 * i, i & 3, -1)   # or_seal_batch seals C2S
        io += (n + 15) // 16 * 16
        oo += (n + 33 + 15) // 16 * 16
    hin = np.zeros(io + 64, dtype=np.uint8)
    for i, n in enumerate(lens):
        o = int(desc[i]["in_off"])
        hin[o:o + n] = np.frombuffer(splitmix_bytes(n, seed + 77 * i), dtype=np.uint8)
    return desc, hin, oo + 64


def _oracle_seal(desc, hin, out_bytes):
    out = np.zeros(out_bytes, dtype=np.uint8)
    precom = np.frombuffer(PRECOM * 2, dtype=np.uint8)
    oracle().or_seal_batch(desc.ctypes.data, len(desc), hin.ctypes.data, out.ctypes.data, precom.ctypes.data, 0, 8)
    return out


def _dev(torch_dev, a):
    torch, dev = torch_dev
    return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).copy()).to(dev)


def _seal_seg(torch_dev, subkeys, desc, hin, ob, seg_blocks):
    torch, dev = torch_dev
    from jeromq_amd import batch
    plan = batch.SegmentPlan(desc, open_=False, seg_blocks=seg_blocks).to(dev)
    d_out = torch.zeros(ob, dtype=torch.uint8, device=dev)
    batch.seal_segments(_dev(torch_dev, desc), plan, _dev(torch_dev, hin), d_out, subkeys, desc_np=desc)
    torch.cuda.synchronize()
    return d_out.cpu().numpy(), plan


def _open_seg(torch_dev, subkeys, desc, hin, ob, seg_blocks):
    torch, dev = torch_dev
    from jeromq_amd import batch
    plan = batch.SegmentPlan(desc, open_=True, seg_blocks=seg_blocks).to(dev)
    d_out = torch.full((ob,), 0xA5, dtype=torch.uint8, device=dev)
    status = torch.full((len(desc),), -1, dtype=torch.int16, device=dev)
    nonces = torch.zeros(len(desc), dtype=torch.int64, device=dev)
    batch.open_segments(_dev(torch_dev, desc), plan, _dev(torch_dev, hin), d_out, subkeys, status, nonces=nonces,
                        desc_np=desc)
    torch.cuda.synchronize()
    return (status.cpu().numpy().view(np.uint16), d_out.cpu().numpy(), nonces.cpu().numpy().view(np.uint64), plan)


@pytest.mark.parametrize("seg_blocks", [2, 3, 5, 64])
@pytest.mark.parametrize("shift", [0, 3])
def test_seal_segments_vs_oracle(torch_dev, subkeys, seg_blocks, shift):
    lens = _boundary_lengths(seg_blocks)
    desc, hin, ob = _pack(lens, shift=shift, seed=seg_blocks)
    out, plan = _seal_seg(torch_dev, subkeys, desc, hin, ob, seg_blocks)
    assert plan.ncomb > 0
    want = _oracle_seal(desc, hin, ob)
    assert np.array_equal(out, want)


def _bodies(lens, seed):
    bodies, meta = [], []
    for i, n in enumerate(lens):
        p = splitmix_bytes(n, seed + 31 * i)
        ctr, fl, k = 11 + 2 * i, i & 3, i & 1
        bodies.append(bytearray(or_curve_encode(p, fl, ctr, k, PRECOM)))
        meta.append((p, fl, ctr, k))
    return bodies, meta


def _bodies_desc(bodies, meta, shift=0, pack=16):
    """pack: body slot granularity (8 with shift 0 = SURVEY.md 8(d) row 4's 8-byte offset table)"""
    desc = np.zeros(len(bodies), dtype=DESC_DTYPE)
    io, oo = shift, 3 if shift else 0
    for i, b in enumerate(bodies):
        desc[i] = (io, oo, len(b), meta[i][3], meta[i][2] - 1, 0x100, -1)
        io += (len(b) + pack - 1) // pack * pack
        oo += (max(len(b) - 33, 0) + 15) // 16 * 16
    hin = np.zeros(io + 64, dtype=np.uint8)
    for i, b in enumerate(bodies):
        o = int(desc[i]["in_off"])
        hin[o:o + len(b)] = np.frombuffer(bytes(b), dtype=np.uint8)
    return desc, hin, oo + 64


@pytest.mark.parametrize("seg_blocks", [2, 5, 64])
@pytest.mark.parametrize("shift", [0, 5])
def test_open_segments_roundtrip_and_tamper(torch_dev, subkeys, L, seg_blocks, shift):
    lens = _boundary_lengths(seg_blocks)
    bodies, meta = _bodies(lens, seed=1000 + seg_blocks)
    want = [L.CZ_STATUS_OK] * len(bodies)
    rng = np.random.default_rng(seg_blocks)
    # tamper some split frames (tag, first/middle/last ciphertext byte) and reject others early
    big = [i for i, b in enumerate(bodies) if len(b) > 64 * (seg_blocks + seg_blocks // 2)]
    for j, i in enumerate(big[::3]):
        b = bodies[i]
        where = [16 + (j % 16), 33, 64 * seg_blocks + 7 if len(b) > 64 * seg_blocks + 7 else 40, len(b) - 1][j % 4]
        b[where] ^= 1 << int(rng.integers(0, 8))
        want[i] = L.CZ_STATUS_CRYPTO
    for i in big[1::7]:
        bodies[i][3] ^= 0x20          # header byte: COMMAND
        want[i] = L.CZ_STATUS_COMMAND
    desc, hin, ob = _bodies_desc(bodies, meta, shift=shift)
    for i in big[2::11]:
        if want[i] == L.CZ_STATUS_OK:
            desc[i]["counter"] = meta[i][2]   # floor == nonce: replay
            want[i] = L.CZ_STATUS_SEQUENCE
    st, out, nn, plan = _open_seg(torch_dev, subkeys, desc, hin, ob, seg_blocks)
    assert plan.ncomb > 0
    assert list(st & 0xff) == want
    for i, (p, fl, ctr, k) in enumerate(meta):
        o = int(desc[i]["out_off"])
        if want[i] == L.CZ_STATUS_OK:
            assert st[i] >> 8 == fl, f"frame {i}"
            assert out[o:o + len(p)].tobytes() == p, f"frame {i} len {len(p)}"
        elif want[i] == L.CZ_STATUS_CRYPTO:
            assert not out[o:o + len(p)].any(), f"frame {i} leaked plaintext"
        if want[i] != L.CZ_STATUS_COMMAND:
            assert nn[i] == ctr


def test_segments_match_unsplit_kernels(torch_dev, subkeys):
    """Zipf batch (the bench's ragged workload, up to 64 KiB): segmented == one lane per frame."""
    torch, dev = torch_dev
    from jeromq_amd import batch
    rng = np.random.default_rng(7)
    j = np.clip(rng.zipf(1.2, size=4000), 1, 1024)
    lens = list((64 * j - rng.integers(0, 64, size=len(j))).astype(np.uint32))
    desc, hin, ob = _pack([int(x) for x in lens], seed=5)
    out_seg, _ = _seal_seg(torch_dev, subkeys, desc, hin, ob, 64)
    d_out = torch.zeros(ob, dtype=torch.uint8, device=dev)
    batch.seal_batch(_dev(torch_dev, desc), len(desc), _dev(torch_dev, hin), d_out, subkeys, desc_np=desc)
    torch.cuda.synchronize()
    assert np.array_equal(out_seg, d_out.cpu().numpy())


@pytest.mark.parametrize("seglines,pair", [(1, 1), (1, 0), (0, 1), (0, 0)])
def test_zipf_seal_open_line_and_direct_stores(torch_dev, subkeys, L, seglines, pair):
    """Every load/store variant of the segment kernels (cz_tune "seglines", "pair"): a Zipf
    batch sealed vs the oracle, then opened with tampered and replayed frames mixed in."""
    lib = L.lib()
    old = lib.cz_tune(b"seglines", seglines)
    old_pair = lib.cz_tune(b"pair", pair)
    try:
        rng = np.random.default_rng(11 + seglines)
        j = np.clip(rng.zipf(1.2, size=3000), 1, 1024)
        lens = [int(x) for x in (64 * j - rng.integers(0, 64, size=len(j)))]
        desc, hin, ob = _pack(lens, seed=17)
        out, _ = _seal_seg(torch_dev, subkeys, desc, hin, ob, 64)
        assert np.array_equal(out, _oracle_seal(desc, hin, ob))
        # open the sealed bodies in place of the oracle's (identical, checked above)
        bodies, meta = [], []
        for i, n in enumerate(lens):
            o = int(desc[i]["out_off"])
            bodies.append(bytearray(out[o:o + n + 33].tobytes()))
            o_in = int(desc[i]["in_off"])
            meta.append((hin[o_in:o_in + n].tobytes(), int(desc[i]["flags"]), int(desc[i]["counter"]), 0))
        want = [L.CZ_STATUS_OK] * len(bodies)
        for i in rng.choice(len(bodies), size=40, replace=False):
            b = bodies[i]
            b[int(rng.integers(16, len(b)))] ^= 0x10
            want[i] = L.CZ_STATUS_CRYPTO
        odesc, ohin, oob = _bodies_desc(bodies, meta)
        for i in rng.choice(len(bodies), size=10, replace=False):
            if want[i] == L.CZ_STATUS_OK:
                odesc[i]["counter"] = meta[i][2] + 1
                want[i] = L.CZ_STATUS_SEQUENCE
        st, pout, nn, plan = _open_seg(torch_dev, subkeys, odesc, ohin, oob, 64)
        assert list(st & 0xff) == want
        for i, (p, fl, ctr, k) in enumerate(meta):
            o = int(odesc[i]["out_off"])
            if want[i] == L.CZ_STATUS_OK:
                assert st[i] >> 8 == fl
                assert pout[o:o + len(p)].tobytes() == p, f"frame {i} len {len(p)}"
            elif want[i] == L.CZ_STATUS_CRYPTO:
                assert not pout[o:o + len(p)].any()
            assert nn[i] == ctr
    finally:
        lib.cz_tune(b"seglines", old)
        lib.cz_tune(b"pair", old_pair)


@pytest.mark.parametrize("shift16,pack", [(1, 8), (0, 8), (1, 1)])
def test_zipf_open_8byte_bodies_and_16byte_outputs(torch_dev, subkeys, L, shift16, pack):
    """Line-emitter paths by alignment (cz_tune "shift16": 16-byte aligned outputs off the 128-byte
    lines through EmitShiftLines): a Zipf batch sealed into 16-byte slots vs the oracle, then its
    bodies repacked at 8-byte offsets (the open's 8-byte-load lines path) or back to back (pack 1:
    funnelled loads from any byte offset) and opened with tampered and replayed frames mixed in;
    rejected frames leave zeros."""
    lib = L.lib()
    old = lib.cz_tune(b"shift16", shift16)
    try:
        rng = np.random.default_rng(23 + shift16)
        j = np.clip(rng.zipf(1.2, size=3000), 1, 1024)
        lens = [int(x) for x in (64 * j - rng.integers(0, 64, size=len(j)))]
        desc, hin, ob = _pack(lens, seed=29)
        assert (desc["out_off"] % 16 == 0).all() and (desc["out_off"] % 128 != 0).any()
        out, _ = _seal_seg(torch_dev, subkeys, desc, hin, ob, 64)
        assert np.array_equal(out, _oracle_seal(desc, hin, ob))
        bodies, meta = [], []
        for i, n in enumerate(lens):
            o = int(desc[i]["out_off"])
            bodies.append(bytearray(out[o:o + n + 33].tobytes()))
            o_in = int(desc[i]["in_off"])
            meta.append((hin[o_in:o_in + n].tobytes(), int(desc[i]["flags"]), int(desc[i]["counter"]), 0))
        want = [L.CZ_STATUS_OK] * len(bodies)
        for i in rng.choice(len(bodies), size=40, replace=False):
            b = bodies[i]
            b[int(rng.integers(16, len(b)))] ^= 0x04
            want[i] = L.CZ_STATUS_CRYPTO
        odesc, ohin, oob = _bodies_desc(bodies, meta, pack=pack)
        assert (odesc["in_off"] % 16 == 8).any() if pack == 8 else (odesc["in_off"] % 4 == 3).any()
        for i in rng.choice(len(bodies), size=10, replace=False):
            if want[i] == L.CZ_STATUS_OK:
                odesc[i]["counter"] = meta[i][2] + 1
                want[i] = L.CZ_STATUS_SEQUENCE
        st, pout, nn, plan = _open_seg(torch_dev, subkeys, odesc, ohin, oob, 64)
        assert list(st & 0xff) == want
        for i, (p, fl, ctr, k) in enumerate(meta):
            o = int(odesc[i]["out_off"])
            if want[i] == L.CZ_STATUS_OK:
                assert st[i] >> 8 == fl
                assert pout[o:o + len(p)].tobytes() == p, f"frame {i} len {len(p)}"
            elif want[i] == L.CZ_STATUS_CRYPTO:
                assert not pout[o:o + len(p)].any()
            assert nn[i] == ctr
    finally:
        lib.cz_tune(b"shift16", old)


def test_full_size_zipf_roundtrip(torch_dev, subkeys, L):
    """BASELINE configs[3] at full size (2^20 Zipf frames, 64 B..64 KiB, 128-byte slots): segmented
    seal -> segmented open is the identity with every status OK; sampled frames across the length
    range equal the oracle; a tampered 64 KiB frame is rejected and its plaintext zeroed."""
    torch, dev = torch_dev
    from jeromq_amd import batch
    rng = np.random.default_rng(42)
    n = 1 << 20
    j = np.empty(0, dtype=np.int64)
    while len(j) < n:
        z = rng.zipf(1.2, size=n)
        j = np.concatenate([j, z[z <= 1024]])
    lens = (64 * j[:n]).astype(np.uint64)
    slot_in = lens
    slot_out = (lens + np.uint64(33 + 127)) // np.uint64(128) * np.uint64(128)
    desc = np.zeros(n, dtype=DESC_DTYPE)
    desc["in_off"][1:] = np.cumsum(slot_in[:-1])
    desc["out_off"][1:] = np.cumsum(slot_out[:-1])
    desc["len"] = lens
    desc["counter"] = 3 + np.arange(n, dtype=np.uint64)
    desc["flags"] = (np.arange(n) % 8 == 0).astype(np.uint32)
    desc["prev"] = -1
    in_bytes, out_bytes = int(slot_in.sum()), int(slot_out.sum())
    d_in = torch.empty(in_bytes, dtype=torch.uint8, device=dev)
    batch.fill(d_in, 0x5EED0003)
    d_out = torch.zeros(out_bytes, dtype=torch.uint8, device=dev)
    d_desc = _dev(torch_dev, desc)
    plan = batch.SegmentPlan(desc, open_=False).to(dev)
    batch.seal_segments(d_desc, plan, d_in, d_out, subkeys[0:1])
    # open: bodies in place, payloads into a fresh buffer laid out like the input
    odesc = desc.copy()
    odesc["in_off"], odesc["out_off"] = desc["out_off"], desc["in_off"]
    odesc["len"] = lens + np.uint64(33)
    odesc["counter"] = 2 + np.arange(n, dtype=np.uint64)        # floor = nonce - 1
    odesc["flags"] = 0x100
    big = int(np.argmax(lens))
    d_out[int(desc["out_off"][big]) + 40000] ^= 1              # tamper inside a 64 KiB frame
    d_odesc = _dev(torch_dev, odesc)
    oplan = batch.SegmentPlan(odesc, open_=True).to(dev)
    d_plain = torch.full((in_bytes,), 0x55, dtype=torch.uint8, device=dev)
    status = torch.full((n,), -1, dtype=torch.int16, device=dev)
    batch.open_segments(d_odesc, oplan, d_out, d_plain, subkeys[0:1], status)
    torch.cuda.synchronize()
    st = status.cpu().numpy().view(np.uint16)
    assert st[big] & 0xff == L.CZ_STATUS_CRYPTO
    ok = np.ones(n, dtype=bool)
    ok[big] = False
    assert not np.any(st[ok] & 0xff)
    assert np.array_equal(st[ok] >> 8, desc["flags"][ok].astype(np.uint16))
    b0, b1 = int(desc["in_off"][big]), int(desc["in_off"][big] + lens[big])
    assert not d_plain[b0:b1].any()
    assert torch.equal(d_plain[:b0], d_in[:b0]) and torch.equal(d_plain[b1:], d_in[b1:])
    d_out[int(desc["out_off"][big]) + 40000] ^= 1
    # EVERY frame against the multi-threaded oracle
    assert oracle_check_full(d_in, d_out, desc, PRECOM) == n
    del d_in, d_out, d_plain
    torch.cuda.empty_cache()


@pytest.mark.parametrize("in_round,out_round", [(1, 16), (8, 8), (1, 1)])
def test_zipf_seal_payloads_at_any_offset(torch_dev, subkeys, L, in_round, out_round):
    """Ragged payloads packed at 1- or 8-byte granularity (messages back to back in the caller's
    buffer): full waves take the line-staged path with dword-aligned loads and the per-frame funnel
    (cz_tune "seal_ina"); every body against the oracle, with both settings of the knob."""
    torch, dev = torch_dev
    rng = np.random.default_rng(31 + in_round + out_round)
    j = np.clip(rng.zipf(1.2, size=3000), 1, 1024)
    lens = [int(x) for x in (64 * j - rng.integers(0, 64, size=len(j)))]
    desc = np.zeros(len(lens), dtype=DESC_DTYPE)
    io = oo = 0
    for i, n in enumerate(lens):
        desc[i] = (io, oo, n, 0, 7 + 3 * i, i & 3, -1)
        io += (n + in_round - 1) // in_round * in_round
        oo += (n + 33 + out_round - 1) // out_round * out_round
    assert (desc["in_off"] % 16 != 0).sum() > len(lens) // 3
    hin = np.frombuffer(splitmix_bytes(io + 64, 41 + in_round), dtype=np.uint8).copy()
    ob = oo + 64
    want = _oracle_seal(desc, hin, ob)
    lib = L.lib()
    old = lib.cz_tune(b"seal_ina", 1)
    try:
        for v in (1, 0):
            lib.cz_tune(b"seal_ina", v)
            out, plan = _seal_seg(torch_dev, subkeys, desc, hin, ob, 64)
            assert plan.ncomb > 0
            bad = np.nonzero(out != want)[0]
            assert bad.size == 0, f"seal_ina={v}: {bad.size} bytes differ, first at {int(bad[0])}"
    finally:
        lib.cz_tune(b"seal_ina", old)


@pytest.mark.parametrize("seal_ina", [1, 0])
def test_seal_segments_tiny_payloads_at_odd_offsets_end_of_buffer(torch_dev, subkeys, L, seal_ina):
    """0..2-byte payloads at byte offsets 1..3 mod 4 are shorter than the distance d to
    their first dword boundary; the any-offset segment seal must read nothing past them (its byte
    count from the dword boundary is clamped to 0, the payload lives in P[-1]).  Full waves of such
    frames, packed back to back, the last payload ending exactly at the end of the input buffer and
    the last body at the end of the output buffer; every body against the oracle."""
    torch, dev = torch_dev
    rng = np.random.default_rng(5)
    lens = [int(x) for x in rng.choice([0, 1, 2, 0, 1, 2, 3, 5], size=256)]
    desc = np.zeros(len(lens), dtype=DESC_DTYPE)
    io, oo = 1, 3          # odd starts: every payload at some byte offset mod 4
    for i, n in enumerate(lens):
        desc[i] = (io, oo, n, 0, 7 + 3 * i, i & 3, -1)
        io += n
        oo += n + 33
    assert (desc["in_off"] % 4 != 0).sum() > len(lens) // 2
    hin = np.frombuffer(splitmix_bytes(io, 99), dtype=np.uint8).copy()   # no slack past the last payload
    want = _oracle_seal(desc, hin, oo)
    lib = L.lib()
    old = lib.cz_tune(b"seal_ina", seal_ina)
    try:
        out, plan = _seal_seg(torch_dev, subkeys, desc, hin, oo, 64)
    finally:
        lib.cz_tune(b"seal_ina", old)
    bad = np.nonzero(out != want)[0]
    assert bad.size == 0, f"{bad.size} bytes differ, first at {int(bad[0])}"


def test_open_segments_8byte_packed_equal_lengths(torch_dev, subkeys, L):
    """Open segments of 8-byte packed bodies in all 16 line phases: equal-length frames (full
    waves of one chunk count on the line paths), long frames split into segments, and ragged ones,
    sealed into 8-byte packed body slots (checked against the oracle), then opened from there with
    tampered (early, middle and last block) and replayed frames mixed in; payloads equal the sealed
    plaintext, rejected frames leave zeros."""
    rng = np.random.default_rng(57)
    lens = [167] * 2048 + [967] * 2048 + [4096] * 1024 + [8967] * 512 + [65536] * 64 + \
        [int(x) for x in rng.integers(0, 3000, size=500)]
    order = rng.permutation(len(lens))
    lens = [lens[k] for k in order]
    desc = np.zeros(len(lens), dtype=DESC_DTYPE)
    io, oo = 0, 8
    for i, n in enumerate(lens):
        desc[i] = (io, oo, n, 0, 7 + 3 * i, i & 3, -1)
        io += (n + 15) // 16 * 16
        oo += (n + 33 + 7) // 8 * 8
    assert (desc["out_off"] % 16 == 8).sum() > len(lens) // 3
    hin = np.frombuffer(splitmix_bytes(io + 64, 61), dtype=np.uint8).copy()
    ob = oo + 64
    sealed, _ = _seal_seg(torch_dev, subkeys, desc, hin, ob, 64)
    assert np.array_equal(sealed, _oracle_seal(desc, hin, ob))
    odesc = np.zeros(len(lens), dtype=DESC_DTYPE)
    po = 0
    for i, n in enumerate(lens):
        odesc[i] = (int(desc[i]["out_off"]), po, n + 33, 0, int(desc[i]["counter"]) - 1, 0x100, -1)
        po += (n + 15) // 16 * 16
    want = [L.CZ_STATUS_OK] * len(lens)
    body = sealed.copy()
    big = [i for i, n in enumerate(lens) if n >= 900]
    for j, i in enumerate(rng.choice(big, size=60, replace=False)):
        n = lens[i] + 33
        where = [40, 64 + int(rng.integers(0, 64)), n // 2, n - 1][j % 4]
        body[int(odesc[i]["in_off"]) + where] ^= 0x08
        want[i] = L.CZ_STATUS_CRYPTO
    for i in rng.choice(len(lens), size=20, replace=False):
        if want[i] == L.CZ_STATUS_OK:
            odesc[i]["counter"] += 1
            want[i] = L.CZ_STATUS_SEQUENCE
    st, pout, nn, plan = _open_seg(torch_dev, subkeys, odesc, body, po + 64, 64)
    assert plan.ncomb > 0
    assert list(st & 0xff) == want
    for i, n in enumerate(lens):
        o, oi = int(odesc[i]["out_off"]), int(desc[i]["in_off"])
        if want[i] == L.CZ_STATUS_OK:
            assert st[i] >> 8 == int(desc[i]["flags"]) & 0xff
            assert pout[o:o + n].tobytes() == hin[oi:oi + n].tobytes(), f"frame {i} len {n}"
        elif want[i] == L.CZ_STATUS_CRYPTO:
            assert not pout[o:o + n].any(), f"frame {i} leaked plaintext"
        assert nn[i] == int(desc[i]["counter"])


def _uneven_plan(plan, rng, open_, min_b0):
    """Re-split every split frame of `plan` at random cuts (2..6 segments of unequal length, the
    first at block 0, every other at or above `min_b0`), renumbering the partial records: the
    kernels take any partition, and the combine then joins unequal middle segments (its general
    per-segment power of r) as well as unequal last ones."""
    segs = plan.segments
    parts = {}
    for sg in segs:
        if sg["part"] != 0xFFFFFFFF:
            parts.setdefault(int(sg["frame"]), []).append(sg)
    keep = [sg for sg in segs if sg["part"] == 0xFFFFFFFF]
    new_segs, combs, npart = [], [], 0
    for c in plan.combines:
        f = int(c["frame"])
        nblk = max(int(s["first_block"]) + int(s["nblocks"]) for s in parts[f])
        lo = min_b0
        if nblk - lo < 2:
            cuts = []
        else:
            k = int(rng.integers(1, min(5, nblk - lo) + 1))
            cuts = sorted(int(x) for x in rng.choice(np.arange(lo, nblk), size=k, replace=False))
        edges = [0] + cuts + [nblk]
        combs.append((f, npart, len(edges) - 1, 0))
        for s in range(len(edges) - 1):
            new_segs.append((f, edges[s], edges[s + 1] - edges[s], npart + s))
        npart += len(edges) - 1
    from jeromq_amd import batch
    out = np.zeros(len(keep) + len(new_segs), dtype=batch.SEGMENT_DTYPE)
    out[:len(keep)] = keep
    out[len(keep):] = new_segs
    plan.segments = out
    plan.combines = np.array(combs, dtype=batch.COMBINE_DTYPE)
    plan.nseg, plan.ncomb, plan.npart = len(out), len(combs), npart
    return plan


@pytest.mark.parametrize("seed", [1, 2])
def test_seal_open_segments_uneven_custom_plans(torch_dev, subkeys, L, seed):
    """Segment plans that cut long frames at random, unequal points (not the planner's equal
    segments): seal against the oracle, then open (with tampered frames) through uneven plans."""
    torch, dev = torch_dev
    from jeromq_amd import batch
    rng = np.random.default_rng(seed)
    lens = _boundary_lengths(6) + [int(x) for x in rng.integers(500, 20000, size=300)]
    desc, hin, ob = _pack(lens, shift=0, seed=90 + seed)
    plan = _uneven_plan(batch.SegmentPlan(desc, open_=False, seg_blocks=6), rng, False, 1).to(dev)
    assert plan.ncomb > 50
    d_out = torch.zeros(ob, dtype=torch.uint8, device=dev)
    batch.seal_segments(_dev(torch_dev, desc), plan, _dev(torch_dev, hin), d_out, subkeys, desc_np=desc)
    torch.cuda.synchronize()
    sealed = d_out.cpu().numpy()
    assert np.array_equal(sealed, _oracle_seal(desc, hin, ob))
    # open the sealed bodies through another uneven plan (open segments s >= 1 start at block >= 2)
    odesc = np.zeros(len(lens), dtype=DESC_DTYPE)
    po = 0
    for i, n in enumerate(lens):
        odesc[i] = (int(desc[i]["out_off"]), po, n + 33, int(desc[i]["key_idx"]), int(desc[i]["counter"]) - 1,
                    0x100, -1)
        po += (n + 15) // 16 * 16
    body = sealed.copy()
    want = [L.CZ_STATUS_OK] * len(lens)
    big = [i for i, n in enumerate(lens) if n > 64 * 9]
    for j, i in enumerate(rng.choice(big, size=24, replace=False)):
        n = lens[i] + 33
        body[int(odesc[i]["in_off"]) + [20, 70, n // 2, n - 1][j % 4]] ^= 0x10
        want[i] = L.CZ_STATUS_CRYPTO
    oplan = _uneven_plan(batch.SegmentPlan(odesc, open_=True, seg_blocks=6), rng, True, 2).to(dev)
    d_plain = torch.full((po + 64,), 0xA5, dtype=torch.uint8, device=dev)
    status = torch.full((len(lens),), -1, dtype=torch.int16, device=dev)
    batch.open_segments(_dev(torch_dev, odesc), oplan, _dev(torch_dev, body), d_plain, subkeys, status,
                        desc_np=odesc)
    torch.cuda.synchronize()
    st = status.cpu().numpy().view(np.uint16)
    pout = d_plain.cpu().numpy()
    assert list(st & 0xff) == want
    for i, n in enumerate(lens):
        o, oi = int(odesc[i]["out_off"]), int(desc[i]["in_off"])
        if want[i] == L.CZ_STATUS_OK:
            assert pout[o:o + n].tobytes() == hin[oi:oi + n].tobytes(), f"frame {i} len {n}"
        else:
            assert not pout[o:o + n].any(), f"frame {i} leaked plaintext"
