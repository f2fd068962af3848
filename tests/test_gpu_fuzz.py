"""GPU: randomized parity over every batched seal/open path, against the CPU oracle.

Each seed draws a ragged batch -- payload lengths biased to the block and chunk edges
(0, 1, 15..17, 31..33, 63..65, ...), frames packed at random byte offsets (so every output
alignment class and emitter is reached), three connection keys, random MORE/COMMAND flags and
nonce counters next to the 2^32 and 2^63 boundaries -- and runs it through:
  * cz_seal_batch (one lane per frame) and cz_seal_segments at a random segment length,
    both compared byte for byte with or_seal_batch (CurveClientMechanism.encode,
    CurveClientMechanism.java:126-163);
  * cz_open_batch and cz_open_segments of the oracle's bodies with tampered tags / ciphertext,
    COMMAND headers, short bodies and replays mixed in: statuses as decode raises them
    (CurveClientMechanism.java:165-224), payloads and flags of the good frames, zeroed
    plaintext for the bad tags;
  * cz_seal_uniform / cz_open_uniform at a random length, stride and counter.
"""
import numpy as np
import pytest

from cz_testlib import DESC_DTYPE, load_golden, oracle, or_curve_encode, splitmix_bytes

pytestmark = pytest.mark.gpu

G = load_golden()
PRECOMS = [bytes.fromhex(G["keys"]["precom"]), splitmix_bytes(32, 901), splitmix_bytes(32, 902)]
EDGES = [0, 1, 15, 16, 17, 30, 31, 32, 33, 34, 63, 64, 65, 95, 96, 97, 127, 128, 129, 191, 223, 224, 4063, 4064,
         4095, 4096, 4097]


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
    k = torch.tensor([list(p) for p in PRECOMS], dtype=torch.uint8, device=dev)
    return batch.subkeys(k, L.CZ_DIR_C2S)


def _lengths(rng, count):
    pick = rng.random(count)
    edge = rng.choice(EDGES, size=count)
    block = 64 * rng.integers(1, 200, size=count) + rng.choice([-33, -32, -17, -16, -1, 0, 1, 15], size=count)
    wide = rng.integers(0, 20000, size=count)
    lens = np.where(pick < 0.4, edge, np.where(pick < 0.8, block, wide))
    return [int(max(0, x)) for x in lens]


def _counters(rng, count, signed_edge=True):
    bases = [3, (1 << 32) - 40, (1 << 33) + 5, int(rng.integers(1, 1 << 40))] + ([(1 << 63) - 500] if signed_edge else [])
    base = int(rng.choice(bases))
    return [base + 2 * i + int(rng.integers(0, 2)) for i in range(count)]


def _signed(x):
    """a nonce as Java's long (the replay check compares signed, CurveClientMechanism.java:186-193)"""
    return x - (1 << 64) if x >= 1 << 63 else x


def _pack(rng, sizes, dense):
    """Random byte offsets: slots of size + gap, gap 0 (dense) or random."""
    offs, o = [], int(rng.integers(0, 64))
    for n in sizes:
        offs.append(o)
        o += n + (0 if dense else int(rng.integers(0, 40)))
    return offs, o + 64


def _dev(torch_dev, a):
    torch, dev = torch_dev
    return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).copy()).to(dev)


@pytest.mark.parametrize("seed", range(6))
def test_fuzz_seal_paths_vs_oracle(torch_dev, subkeys, seed):
    torch, dev = torch_dev
    from jeromq_amd import batch
    rng = np.random.default_rng(1000 + seed)
    count = int(rng.integers(64, 400))
    lens = _lengths(rng, count)
    ctrs = _counters(rng, count)
    dense = seed % 2 == 0
    in_offs, in_bytes = _pack(rng, lens, dense)
    out_offs, out_bytes = _pack(rng, [n + 33 for n in lens], dense)
    desc = np.zeros(count, dtype=DESC_DTYPE)
    for i in range(count):
        desc[i] = (in_offs[i], out_offs[i], lens[i], int(rng.integers(0, 3)), ctrs[i], int(rng.integers(0, 4)), -1)
    hin = np.frombuffer(splitmix_bytes(in_bytes, 5000 + seed), dtype=np.uint8).copy()
    want = np.zeros(out_bytes, dtype=np.uint8)
    table = np.frombuffer(b"".join(PRECOMS), dtype=np.uint8).copy()
    oracle().or_seal_batch(desc.ctypes.data, count, hin.ctypes.data, want.ctypes.data, table.ctypes.data, 0, 8)
    mask = np.zeros(out_bytes, dtype=bool)
    for i in range(count):
        mask[out_offs[i]:out_offs[i] + lens[i] + 33] = True
    d_desc, d_in = _dev(torch_dev, desc), _dev(torch_dev, hin)
    seg = int(rng.choice([2, 3, 4, 7, 16, 64, 128]))
    for path in ("batch", "segments"):
        d_out = torch.zeros(out_bytes, dtype=torch.uint8, device=dev)
        if path == "batch":
            batch.seal_batch(d_desc, count, d_in, d_out, subkeys, desc_np=desc)
        else:
            plan = batch.SegmentPlan(desc, open_=False, seg_blocks=seg).to(dev)
            batch.seal_segments(d_desc, plan, d_in, d_out, subkeys, desc_np=desc)
        torch.cuda.synchronize()
        got = d_out.cpu().numpy()
        bad = np.nonzero((got != want) & mask)[0]
        if len(bad):
            i = int(np.searchsorted(out_offs, bad[0], side="right")) - 1
            raise AssertionError(f"{path} (seg {seg}): frame {i} len {lens[i]} at out offset {out_offs[i]} "
                                 f"differs from the oracle")


@pytest.mark.parametrize("seed", range(6))
def test_fuzz_open_paths_vs_oracle(torch_dev, subkeys, L, seed):
    torch, dev = torch_dev
    from jeromq_amd import batch
    rng = np.random.default_rng(2000 + seed)
    count = int(rng.integers(64, 300))
    lens = _lengths(rng, count)
    ctrs = _counters(rng, count)
    keys = [int(rng.integers(0, 3)) for _ in range(count)]
    flags = [int(rng.integers(0, 4)) for _ in range(count)]
    payloads = [splitmix_bytes(n, 7000 + 13 * i + seed) for i, n in enumerate(lens)]
    bodies = [bytearray(or_curve_encode(payloads[i], flags[i], ctrs[i], 0, PRECOMS[keys[i]])) for i in range(count)]
    floors = [c - 1 for c in ctrs]
    want = [L.CZ_STATUS_OK] * count
    for i in range(count):
        r = rng.random()
        if r < 0.08:        # tag or ciphertext byte
            j = int(rng.integers(16, len(bodies[i])))
            bodies[i][j] ^= 1 << int(rng.integers(0, 8))
            want[i] = L.CZ_STATUS_CRYPTO
        elif r < 0.11:      # replay: floor == nonce
            floors[i] = ctrs[i]
            want[i] = L.CZ_STATUS_SEQUENCE
        elif r < 0.13:      # not a MESSAGE command
            bodies[i][1] ^= 0x20
            want[i] = L.CZ_STATUS_COMMAND
        elif r < 0.15:      # shorter than the 33-byte overhead
            bodies[i] = bodies[i][:int(rng.integers(8, 33))]
            want[i] = L.CZ_STATUS_MALFORMED
    for i in range(count):  # a counter that crosses 2^63 is a replay as a signed long
        if want[i] == L.CZ_STATUS_OK and _signed(ctrs[i]) <= _signed(floors[i]):
            want[i] = L.CZ_STATUS_SEQUENCE
    sizes = [len(b) for b in bodies]
    dense = seed % 2 == 1
    in_offs, in_bytes = _pack(rng, sizes, dense)
    out_offs, out_bytes = _pack(rng, [max(n - 33, 0) for n in sizes], dense)
    desc = np.zeros(count, dtype=DESC_DTYPE)
    hin = np.zeros(in_bytes, dtype=np.uint8)
    for i in range(count):
        desc[i] = (in_offs[i], out_offs[i], sizes[i], keys[i], floors[i] & ((1 << 64) - 1), L.CZ_DESC_CHECK_NONCE, -1)
        hin[in_offs[i]:in_offs[i] + sizes[i]] = np.frombuffer(bytes(bodies[i]), dtype=np.uint8)
    d_desc, d_in = _dev(torch_dev, desc), _dev(torch_dev, hin)
    seg = int(rng.choice([2, 3, 5, 16, 64, 128]))
    for path in ("batch", "segments"):
        d_out = torch.full((out_bytes,), 0xA5, dtype=torch.uint8, device=dev)
        status = torch.full((count,), -1, dtype=torch.int16, device=dev)
        if path == "batch":
            batch.open_batch(d_desc, count, d_in, d_out, subkeys, status, desc_np=desc)
        else:
            plan = batch.SegmentPlan(desc, open_=True, seg_blocks=seg).to(dev)
            batch.open_segments(d_desc, plan, d_in, d_out, subkeys, status, desc_np=desc)
        torch.cuda.synchronize()
        st = status.cpu().numpy().view(np.uint16)
        out = d_out.cpu().numpy()
        for i in range(count):
            where = f"{path} (seg {seg}) frame {i} len {lens[i]} at {in_offs[i]}"
            assert st[i] & 0xff == want[i], where
            o, n = out_offs[i], sizes[i] - 33
            if want[i] == L.CZ_STATUS_OK:
                assert st[i] >> 8 == flags[i], where
                assert out[o:o + n].tobytes() == payloads[i], where
            elif want[i] == L.CZ_STATUS_CRYPTO:
                assert not out[o:o + n].any(), where + ": plaintext of a bad tag left in the output"


@pytest.mark.parametrize("seed", range(4))
def test_fuzz_uniform_vs_oracle(torch_dev, subkeys, L, seed):
    torch, dev = torch_dev
    from jeromq_amd import batch
    rng = np.random.default_rng(3000 + seed)
    n = int(rng.choice(EDGES + [int(rng.integers(0, 9000))]))
    count = int(rng.integers(1, 700))
    in_stride = n + int(rng.integers(0, 50))
    out_stride = n + 33 + int(rng.integers(0, 50))
    c0 = _counters(rng, 1, signed_edge=False)[0]
    hin = np.frombuffer(splitmix_bytes(max(in_stride * count, 16), 9000 + seed), dtype=np.uint8).copy()
    flags = rng.integers(0, 4, size=count).astype(np.uint8)
    d_in = torch.from_numpy(hin).to(dev)
    d_out = torch.zeros(out_stride * count, dtype=torch.uint8, device=dev)
    batch.seal_uniform(d_in, in_stride, d_out, out_stride, count, n, subkeys[0], c0,
                       flags8=torch.from_numpy(flags).to(dev))
    torch.cuda.synchronize()
    out = d_out.cpu().numpy()
    for i in list(range(min(count, 40))) + list(rng.integers(0, count, size=20)):
        i = int(i)
        p = hin[i * in_stride:i * in_stride + n].tobytes()
        body = out[i * out_stride:i * out_stride + n + 33].tobytes()
        assert body == or_curve_encode(p, int(flags[i]), c0 + i, 0, PRECOMS[0]), f"seal frame {i} (n {n})"
    plain = torch.full((in_stride * count + 16,), 0xA5, dtype=torch.uint8, device=dev)
    status = torch.full((count,), -1, dtype=torch.int16, device=dev)
    batch.open_uniform(d_out, out_stride, plain, in_stride, count, n + 33, subkeys[0], c0 - 1, status)
    torch.cuda.synchronize()
    st = status.cpu().numpy().view(np.uint16)
    assert np.all(st & 0xff == L.CZ_STATUS_OK)
    assert np.array_equal(st >> 8, flags)
    back = plain.cpu().numpy()
    for i in range(count):
        assert back[i * in_stride:i * in_stride + n].tobytes() == hin[i * in_stride:i * in_stride + n].tobytes()


@pytest.mark.parametrize("seed", range(6))
def test_fuzz_uniform_back_to_back_bodies(torch_dev, subkeys, seed):
    """cz_seal_uniform with bodies back to back (out_stride == n + 33, the V2 wire layout) at a
    random output base: the class-static, whole-unit emitter, whose edge
    units carry the next body's header.  Body lengths near every residue that matters mod 64 and
    mod 16, batches with partial workgroups and partial waves, counters crossing 2^32 inside a
    wave; every body against the oracle and every byte around the batch untouched."""
    torch, dev = torch_dev
    from jeromq_amd import batch
    rng = np.random.default_rng(7000 + seed)
    mlen = 64 * int(rng.integers(4, 80)) + int(rng.choice([1, 15, 16, 17, 31, 32, 33, 47, 63]))
    n = mlen - 33
    count = int(rng.integers(300, 1300))
    base = int(rng.integers(0, 16))
    in_stride = (n + 15) // 16 * 16
    c0 = [3, (1 << 32) - int(rng.integers(1, 600)), int(rng.integers(1, 1 << 40))][seed % 3]
    hin = np.frombuffer(splitmix_bytes(in_stride * count, 7100 + seed), dtype=np.uint8).copy()
    flags = rng.integers(0, 4, size=count).astype(np.uint8)
    d_in = torch.from_numpy(hin).to(dev)
    size = base + count * mlen + 64
    d_buf = torch.full((size,), 0xA5, dtype=torch.uint8, device=dev)
    batch.seal_uniform(d_in, in_stride, d_buf[base:], mlen, count, n, subkeys[0], c0,
                       flags8=torch.from_numpy(flags).to(dev))
    torch.cuda.synchronize()
    out = d_buf.cpu().numpy()
    for i in range(count):
        o = base + i * mlen
        want = or_curve_encode(hin[i * in_stride:i * in_stride + n].tobytes(), int(flags[i]), c0 + i, 0, PRECOMS[0])
        assert out[o:o + mlen].tobytes() == want, f"frame {i} of {count} (body {mlen} B, base {base}, c0 {c0})"
    assert not (out[:base] != 0xA5).any(), "bytes before the first body were written"
    assert not (out[base + count * mlen:] != 0xA5).any(), "bytes past the last body were written"
