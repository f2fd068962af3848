"""GPU parity: the gfx950 kernels (through the C-ABI) against the golden fixtures and the
CPU oracle, bit-exact.  Runs on the MI355X box: `pytest -m gpu`.

Cases follow SURVEY.md 8(c): payload sizes {0..65536}, flags 0..3, both directions,
counters {2, 3, 2^32-1, 2^32, 2^63-1}, tampered tag / ciphertext / header, replay,
unaligned offsets, ragged batches, and full-size round trips.
"""
import ctypes
import hashlib

import numpy as np
import pytest

from cz_testlib import (DESC_DTYPE, load_golden, oracle, oracle_check_full, or_curve_encode, splitmix_bytes,
                        splitmix_words)

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


def _pack(frames, align=16, base_in=0, base_out=0, overhead=33):
    """frames: list of (payload bytes, flags, counter, key_idx) -> desc, host input"""
    desc = np.zeros(len(frames), dtype=DESC_DTYPE)
    io, oo = base_in, base_out
    for i, (p, fl, ctr, kidx) in enumerate(frames):
        desc[i] = (io, oo, len(p), kidx, ctr, fl, -1)
        io += (len(p) + align - 1) // align * align
        oo += (len(p) + overhead + align - 1) // align * align
    hin = np.zeros(max(io + 64, 64), dtype=np.uint8)
    for i, (p, *_rest) in enumerate(frames):
        o = int(desc[i]["in_off"])
        hin[o:o + len(p)] = np.frombuffer(p, dtype=np.uint8)
    return desc, hin, max(oo + 64, 64)


def _seal(torch_dev, subkeys, desc, hin, out_bytes, order=None):
    torch, dev = torch_dev
    from jeromq_amd import batch
    d_in = torch.from_numpy(hin).to(dev)
    d_out = torch.zeros(out_bytes, dtype=torch.uint8, device=dev)
    d_desc = torch.from_numpy(desc.view(np.uint8).copy()).to(dev)
    d_order = None if order is None else torch.from_numpy(order.view(np.int32)).to(dev)
    batch.seal_batch(d_desc, len(desc), d_in, d_out, subkeys, order=d_order, desc_np=desc)
    torch.cuda.synchronize()
    return d_out.cpu().numpy()


def test_subkeys_match_golden(subkeys):
    sk = subkeys.cpu().numpy()
    assert sk[0].tobytes().hex() == G["keys"]["subkey_c2s"]
    assert sk[1].tobytes().hex() == G["keys"]["subkey_s2c"]


def test_host_subkey(L, torch_dev):
    from jeromq_amd.curve import subkey
    assert subkey(PRECOM, L.CZ_DIR_C2S).hex() == G["keys"]["subkey_c2s"]
    assert subkey(PRECOM, L.CZ_DIR_S2C).hex() == G["keys"]["subkey_s2c"]


def test_golden_messages_seal(torch_dev, subkeys):
    msgs = G["messages"]
    frames = [(splitmix_bytes(v["n"], v["seed"]), v["flags"], v["counter"], v["from_server"]) for v in msgs]
    desc, hin, ob = _pack(frames)
    out = _seal(torch_dev, subkeys, desc, hin, ob)
    for i, v in enumerate(msgs):
        o = int(desc[i]["out_off"])
        body = out[o:o + v["n"] + 33].tobytes()
        assert hashlib.sha256(body).hexdigest() == v["sha256"], f"vector {i}: {v['n']} B"
        if "body" in v:
            assert body.hex() == v["body"]


def test_survey_kat(torch_dev, subkeys):
    kat = G["survey_kat"]
    desc, hin, ob = _pack([(bytes.fromhex(kat["payload_hex"]), 0, 3, 0)])
    out = _seal(torch_dev, subkeys, desc, hin, ob)
    assert out[:133].tobytes().hex() == kat["body"]


def _open(torch_dev, subkeys, odesc, hin, out_bytes, nonces=False):
    torch, dev = torch_dev
    from jeromq_amd import batch
    d_in = torch.from_numpy(hin).to(dev)
    d_out = torch.zeros(out_bytes, dtype=torch.uint8, device=dev)
    d_desc = torch.from_numpy(odesc.view(np.uint8).copy()).to(dev)
    status = torch.full((len(odesc),), -1, dtype=torch.int16, device=dev)
    d_non = torch.zeros(len(odesc), dtype=torch.int64, device=dev) if nonces else None
    batch.open_batch(d_desc, len(odesc), d_in, d_out, subkeys, status, nonces=d_non, desc_np=odesc)
    torch.cuda.synchronize()
    st = status.cpu().numpy().view(np.uint16)
    return st, d_out.cpu().numpy(), (d_non.cpu().numpy().view(np.uint64) if nonces else None)


def _bodies_desc(bodies, key_idx, floors, check=True, align=16):
    desc = np.zeros(len(bodies), dtype=DESC_DTYPE)
    io, oo = 0, 0
    for i, b in enumerate(bodies):
        desc[i] = (io, oo, len(b), key_idx[i], floors[i], 0x100 if check else 0, -1)
        io += (len(b) + align - 1) // align * align
        oo += (max(len(b) - 33, 0) + align - 1) // align * align
    hin = np.zeros(io + 64, dtype=np.uint8)
    for i, b in enumerate(bodies):
        o = int(desc[i]["in_off"])
        hin[o:o + len(b)] = np.frombuffer(b, dtype=np.uint8)
    return desc, hin, oo + 64


def test_golden_messages_open(torch_dev, subkeys, L):
    msgs = [v for v in G["messages"] if "body" in v]
    bodies = [bytes.fromhex(v["body"]) for v in msgs]
    desc, hin, ob = _bodies_desc(bodies, [v["from_server"] for v in msgs], [v["counter"] - 1 for v in msgs])
    st, out, nn = _open(torch_dev, subkeys, desc, hin, ob, nonces=True)
    for i, v in enumerate(msgs):
        assert st[i] & 0xff == L.CZ_STATUS_OK, f"vector {i}"
        assert st[i] >> 8 == v["flags"]
        assert nn[i] == v["counter"]
        o = int(desc[i]["out_off"])
        assert out[o:o + v["n"]].tobytes() == splitmix_bytes(v["n"], v["seed"])


def test_open_rejections(torch_dev, subkeys, L):
    v = next(x for x in G["messages"] if x["n"] == 100 and x["from_server"] == 0 and "body" in x)
    good = bytes.fromhex(v["body"])
    tag_bad = bytearray(good); tag_bad[20] ^= 1
    ct_bad = bytearray(good); ct_bad[-1] ^= 0x80
    flag_bad = bytearray(good); flag_bad[32] ^= 2
    cmd_bad = b"\x07MESSAXE" + good[8:]
    quirk = b"\x07MESSAGx" + good[8:]   # Msgs.startsWith never compares byte 7
    short = good[:32]
    tiny = good[:7]
    wrong_dir = good
    bodies = [good, bytes(tag_bad), bytes(ct_bad), bytes(flag_bad), cmd_bad, quirk, short, tiny, wrong_dir, good, good]
    keys = [0] * 8 + [1, 0, 0]
    floors = [v["counter"] - 1] * 9 + [v["counter"], v["counter"] + 5]
    desc, hin, ob = _bodies_desc(bodies, keys, floors)
    st, out, _ = _open(torch_dev, subkeys, desc, hin, ob)
    want = [L.CZ_STATUS_OK, L.CZ_STATUS_CRYPTO, L.CZ_STATUS_CRYPTO, L.CZ_STATUS_CRYPTO, L.CZ_STATUS_COMMAND,
            L.CZ_STATUS_OK, L.CZ_STATUS_MALFORMED, L.CZ_STATUS_COMMAND, L.CZ_STATUS_CRYPTO, L.CZ_STATUS_SEQUENCE,
            L.CZ_STATUS_SEQUENCE]
    assert list(st & 0xff) == want
    # rejected frames never expose plaintext
    for i in (1, 2, 3, 8):
        o = int(desc[i]["out_off"])
        assert not out[o:o + 100].any()
    o = int(desc[5]["out_off"])
    assert out[o:o + 100].tobytes() == splitmix_bytes(100, v["seed"])


def test_open_signed_nonce_compare(torch_dev, subkeys, L):
    # Java compares `long` values: a nonce >= 2^63 is negative and fails against floor 5
    p = b"x" * 10
    b1 = or_curve_encode(p, 0, 1 << 63, 0, PRECOM)
    b2 = or_curve_encode(p, 0, (1 << 63) - 1, 0, PRECOM)
    desc, hin, ob = _bodies_desc([b1, b2], [0, 0], [5, 5])
    st, _, _ = _open(torch_dev, subkeys, desc, hin, ob)
    assert list(st & 0xff) == [L.CZ_STATUS_SEQUENCE, L.CZ_STATUS_OK]


def test_open_prev_chain(torch_dev, subkeys, L):
    bodies = [or_curve_encode(b"abc" * i, 0, c, 0, PRECOM) for i, c in enumerate([3, 4, 9, 9, 10])]
    desc, hin, ob = _bodies_desc(bodies, [0] * 5, [2] * 5)
    desc["prev"] = [-1, 0, 1, 2, 3]
    st, _, _ = _open(torch_dev, subkeys, desc, hin, ob)
    assert list(st & 0xff) == [0, 0, 0, L.CZ_STATUS_SEQUENCE, 0]


@pytest.mark.parametrize("shift", [1, 3, 8])
def test_unaligned_offsets(torch_dev, subkeys, shift):
    frames = [(splitmix_bytes(n, 500 + n), n & 3, 1000 + n, n & 1) for n in [0, 5, 31, 32, 33, 64, 100, 257, 4096]]
    desc, hin, ob = _pack(frames, align=16)
    desc["in_off"] += shift
    desc["out_off"] += 2 * shift + 1
    hin = np.concatenate([np.zeros(shift, dtype=np.uint8), hin])
    out = _seal(torch_dev, subkeys, desc, hin, ob + 64)
    for i, (p, fl, ctr, k) in enumerate(frames):
        o = int(desc[i]["out_off"])
        assert out[o:o + len(p) + 33].tobytes() == or_curve_encode(p, fl, ctr, k, PRECOM)
    # and open from unaligned bodies
    bodies = [or_curve_encode(p, fl, ctr, k, PRECOM) for (p, fl, ctr, k) in frames]
    odesc, ohin, oob = _bodies_desc(bodies, [f[3] for f in frames], [f[2] - 1 for f in frames])
    odesc["in_off"] += shift
    odesc["out_off"] += 3
    ohin = np.concatenate([np.zeros(shift, dtype=np.uint8), ohin])
    st, pout, _ = _open(torch_dev, subkeys, odesc, ohin, oob + 16)
    assert not np.any(st & 0xff)
    for i, (p, *_r) in enumerate(frames):
        o = int(odesc[i]["out_off"])
        assert pout[o:o + len(p)].tobytes() == p


def _oracle_seal(desc, hin, out_bytes, from_server=0):
    out = np.zeros(out_bytes, dtype=np.uint8)
    precom = np.frombuffer(PRECOM * 2, dtype=np.uint8)
    oracle().or_seal_batch(desc.ctypes.data, len(desc), hin.ctypes.data, out.ctypes.data, precom.ctypes.data,
                           from_server, 8)
    return out


def test_ragged_zipf_vs_oracle(torch_dev, subkeys):
    rng = np.random.default_rng(42)
    n = 3000
    j = rng.zipf(1.2, size=n)
    j = np.clip(j, 1, 1024)
    lens = (64 * j - rng.integers(0, 64, size=n)).astype(np.uint32)  # ragged, not multiples of 64
    frames = [(splitmix_bytes(int(l), 9000 + i), i & 3, 3 + i, 0) for i, l in enumerate(lens)]
    desc, hin, ob = _pack(frames)
    from jeromq_amd.batch import plan_order
    order = plan_order(desc)
    out = _seal(torch_dev, subkeys, desc, hin, ob, order=order)
    want = _oracle_seal(desc, hin, ob)
    assert np.array_equal(out, want)


def _oracle_uniform(hin, in_stride, count, n, flags, counter0):
    desc = np.zeros(count, dtype=DESC_DTYPE)
    desc["in_off"] = np.arange(count, dtype=np.uint64) * in_stride
    desc["out_off"] = np.arange(count, dtype=np.uint64) * (n + 33)
    desc["len"] = n
    desc["counter"] = counter0 + np.arange(count, dtype=np.uint64)
    desc["flags"] = flags
    return _oracle_seal(desc, hin, count * (n + 33)).reshape(count, n + 33)


# (payload length, in_stride, out_stride, count): exercises every output stager --
# LINES (out_stride % 128 == 0), REGION (64 slots <= 16 KiB), DIRECT -- and partial waves
UNIFORM_CASES = [
    (4096, 4096, 4224, 4096),        # LINES, the benchmark layout
    (4096, 4096, 4224, 4096 + 37),   # LINES + a partial last wave (direct)
    (4096, 4096, 4144, 1000),        # DIRECT (stride not a line multiple)
    (100, 112, 144, 4096 + 5),       # REGION, the 100 B benchmark layout
    (100, 112, 256, 640),            # REGION with 256-byte slots
    (1000, 1008, 1152, 777),         # LINES, mid-size
    (223, 224, 256, 300),            # body 256 B exactly: LINES
    (300, 304, 384, 200),            # LINES, 6 blocks, 13-byte last block, 3 lines
    (4000, 4000, 4096, 130),         # LINES, last line 33 bytes short of the slot
    (0, 16, 48, 200),                # empty payloads: REGION
    (31, 32, 128, 130),              # body = 64 B (block-0 only): REGION
]


@pytest.mark.parametrize("n,in_stride,out_stride,count", UNIFORM_CASES)
def test_uniform_seal_open_vs_oracle(torch_dev, subkeys, n, in_stride, out_stride, count):
    torch, dev = torch_dev
    from jeromq_amd import batch
    d_in = torch.empty(max(count * in_stride, 16), dtype=torch.uint8, device=dev)
    batch.fill(d_in, 0x5EED0002 + n)
    flags = torch.zeros(count, dtype=torch.uint8, device=dev)
    flags[::8] = 1
    flags[3::8] = 2
    d_out = torch.full((count * out_stride,), 0xAB, dtype=torch.uint8, device=dev)
    batch.seal_uniform(d_in, in_stride, d_out, out_stride, count, n, subkeys[0], 3, flags8=flags)
    torch.cuda.synchronize()
    hin = d_in.cpu().numpy()
    fl = flags.cpu().numpy()
    want = _oracle_uniform(hin, in_stride, count, n, fl, 3)
    got = d_out.cpu().numpy().reshape(count, out_stride)
    bad = np.nonzero(np.any(got[:, :n + 33] != want, axis=1))[0]
    assert len(bad) == 0, f"{len(bad)} frames differ, first {bad[:5]}"
    # slot padding: written as zero by the staged paths, untouched (0xAB) by the direct path
    pad = got[:, n + 33:]
    assert np.all((pad == 0) | (pad == 0xAB))
    # open back, in order, replay-checked, into payload slots of in_stride bytes
    d_plain = torch.full((count * in_stride,), 0xCD, dtype=torch.uint8, device=dev)
    status = torch.full((count,), -1, dtype=torch.int16, device=dev)
    batch.open_uniform(d_out, out_stride, d_plain, in_stride, count, n + 33, subkeys[0], 2, status)
    torch.cuda.synchronize()
    st = status.cpu().numpy().view(np.uint16)
    assert np.all(st & 0xff == 0)
    assert np.array_equal(st >> 8, fl)
    plain = d_plain.cpu().numpy().reshape(count, in_stride)[:, :n]
    assert np.array_equal(plain, hin[:count * in_stride].reshape(count, in_stride)[:, :n])


# Nonce counters whose high 32-bit word changes inside a wave (2^32 - 100: waves straddle the
# boundary and take the per-lane path) or is uniform but nonzero (2^32 + 7, 2^48 + 3).  The
# uniform kernels move wave-uniform Salsa20 work to the scalar unit only when the high word
# is the same in every lane (cz_device.h rounds12_uniform), so both paths are compared here.
@pytest.mark.parametrize("counter0", [2**32 - 100, 2**32 + 7, 2**48 + 3])
@pytest.mark.parametrize("n,in_stride,out_stride,count", [(4096, 4096, 4224, 1024 + 64), (100, 112, 144, 2048)])
def test_uniform_counter_high_word(torch_dev, subkeys, n, in_stride, out_stride, count, counter0):
    torch, dev = torch_dev
    from jeromq_amd import batch
    d_in = torch.empty(count * in_stride, dtype=torch.uint8, device=dev)
    batch.fill(d_in, 0x5EED1000 + n)
    flags = torch.zeros(count, dtype=torch.uint8, device=dev)
    flags[::8] = 1
    d_out = torch.full((count * out_stride,), 0xAB, dtype=torch.uint8, device=dev)
    batch.seal_uniform(d_in, in_stride, d_out, out_stride, count, n, subkeys[0], counter0, flags8=flags)
    torch.cuda.synchronize()
    hin = d_in.cpu().numpy()
    fl = flags.cpu().numpy()
    want = _oracle_uniform(hin, in_stride, count, n, fl, counter0)
    got = d_out.cpu().numpy().reshape(count, out_stride)[:, :n + 33]
    bad = np.nonzero(np.any(got != want, axis=1))[0]
    assert len(bad) == 0, f"{len(bad)} frames differ, first {bad[:5]}"
    d_plain = torch.zeros(count * in_stride, dtype=torch.uint8, device=dev)
    status = torch.full((count,), -1, dtype=torch.int16, device=dev)
    batch.open_uniform(d_out, out_stride, d_plain, in_stride, count, n + 33, subkeys[0], counter0 - 1, status)
    torch.cuda.synchronize()
    st = status.cpu().numpy().view(np.uint16)
    assert np.all(st & 0xff == 0)
    plain = d_plain.cpu().numpy().reshape(count, in_stride)[:, :n]
    assert np.array_equal(plain, hin.reshape(count, in_stride)[:, :n])


@pytest.mark.parametrize("n,body_stride,pay_stride", [(4096, 4224, 4096), (100, 144, 112), (1000, 1040, 1008)])
def test_uniform_open_rejections_in_a_full_wave(torch_dev, subkeys, L, n, body_stride, pay_stride):
    """Rejected frames inside a cooperative (LDS-staged) wave: statuses per frame, the
    other frames intact, rejected slots zeroed."""
    torch, dev = torch_dev
    from jeromq_amd import batch
    count = 256
    d_in = torch.empty(count * pay_stride, dtype=torch.uint8, device=dev)
    batch.fill(d_in, 99 + n)
    d_body = torch.zeros(count * body_stride, dtype=torch.uint8, device=dev)
    batch.seal_uniform(d_in, pay_stride, d_body, body_stride, count, n, subkeys[0], 10)
    torch.cuda.synchronize()
    bodies = d_body.cpu().numpy().reshape(count, body_stride).copy()
    bodies[5, 40] ^= 1                       # ciphertext -> CRYPTO
    bodies[17, 3] ^= 0x20                    # "\x07MESsAGE" -> COMMAND
    bodies[40, 8:16] = bodies[39, 8:16]      # nonce == previous -> SEQUENCE
    bodies[63, 20] ^= 4                      # tag -> CRYPTO (last lane of wave 0)
    bodies[64, 7] ^= 0x55                    # byte 7 is never compared (Msgs.java:31) -> OK
    d_body = torch.from_numpy(bodies.reshape(-1)).to(dev)
    d_plain = torch.full((count * pay_stride,), 0xEE, dtype=torch.uint8, device=dev)
    status = torch.full((count,), -1, dtype=torch.int16, device=dev)
    batch.open_uniform(d_body, body_stride, d_plain, pay_stride, count, n + 33, subkeys[0], 9, status)
    torch.cuda.synchronize()
    st = status.cpu().numpy().view(np.uint16) & 0xff
    want = np.zeros(count, dtype=np.uint16)
    want[[5, 63]] = L.CZ_STATUS_CRYPTO
    want[17] = L.CZ_STATUS_COMMAND
    want[40] = L.CZ_STATUS_SEQUENCE
    assert np.array_equal(st, want), np.nonzero(st != want)
    plain = d_plain.cpu().numpy().reshape(count, pay_stride)[:, :n]
    ref = d_in.cpu().numpy().reshape(count, pay_stride)[:, :n]
    ok = want == 0
    assert np.array_equal(plain[ok], ref[ok])
    rej = plain[~ok]
    assert np.all((rej == 0) | (rej == 0xEE))  # never the plaintext
    assert not np.array_equal(rej, ref[~ok])


def test_nacl_box_afternm_golden(L, torch_dev):
    from jeromq_amd.curve import Curve
    cv = Curve()
    for v in G["box_afternm"]:
        key, n24 = bytes.fromhex(v["key"]), bytes.fromhex(v["nonce"])
        m = bytes(32) + splitmix_bytes(v["n"], v["m_seed"])
        c = bytearray(len(m))
        assert cv.afternm(c, m, len(m), n24, key) == 0
        assert c.hex() == v["c"]
        m2 = bytearray(len(m))
        assert cv.openAfternm(m2, bytes(c), len(c), n24, key) == 0
        assert bytes(m2) == m
        c[-1] ^= 1
        m3 = bytearray(len(m))
        assert cv.openAfternm(m3, bytes(c), len(c), n24, key) == -1
        assert not any(m3)
    assert cv.afternm(bytearray(31), bytes(31), 31, bytes(24), bytes(32)) == -1


def test_nacl_one_launch_contract_and_subkey_cache(L, torch_dev):
    """The one-launch drop-in (k_nacl_one): the per-thread subkey cache -- 12 keys cycled through the
    8-entry cache, the same key under two nonce prefixes (client / server direction),
    cz_nacl_forget in between -- never serves a stale subkey: every box against the oracle."""
    from cz_testlib import or_box_afternm
    lib = L.lib()
    rng = np.random.default_rng(5)
    keys = [rng.integers(0, 256, 32, dtype=np.uint8).tobytes() for _ in range(12)]
    for rnd in range(3):
        for i, key in enumerate(keys):
            for prefix in (b"CurveZMQMESSAGEC", b"CurveZMQMESSAGES"):
                n24 = prefix + (1000 * rnd + i).to_bytes(8, "big")
                mlen = 32 + 1 + int(rng.integers(0, 6000))
                mm = bytes(32) + rng.integers(0, 256, mlen - 32, dtype=np.uint8).tobytes()
                rc, want = or_box_afternm(mm, n24, key)
                assert rc == 0
                cc = ctypes.create_string_buffer(mlen)
                assert lib.cz_box_afternm(cc, mm, mlen, n24, key) == 0 and cc.raw == want, (rnd, i, mlen)
                back = ctypes.create_string_buffer(mlen)
                assert lib.cz_box_open_afternm(back, want, mlen, n24, key) == 0 and back.raw == mm
        if rnd == 1:
            assert lib.cz_nacl_forget() == 0


@pytest.mark.parametrize("v", G["box_afternm_prefix"], ids=lambda v: f"mlen{v['mlen']}")
def test_nacl_box_nonzero_prefix_golden(L, torch_dev, v):
    """NaCl's crypto_box_afternm for EVERY m (Curve.box, Curve.java:184-193, hands jnacl any m): an m
    whose first 32 bytes are not zero seals with rc 0, the ciphertext of its zero-prefixed twin and
    the tag of a MAC keyed with c[0:32] = keystream ^ m[0:32] -- libsodium's box, byte for byte,
    through cz_box_afternm and cz_secretbox (81953 bytes: past the one-pass 80 KiB, several passes of
    k_nacl_one).  The open of such a box fails as in NaCl (its MAC key is the keystream alone), and
    leaves the output untouched."""
    import hashlib
    lib = L.lib()
    key, n24 = bytes.fromhex(v["key"]), bytes.fromhex(v["nonce"])
    m = splitmix_bytes(v["mlen"], v["m_seed"])
    for fn in (lib.cz_box_afternm, lib.cz_secretbox):
        c = ctypes.create_string_buffer(b"\x5a" * len(m), len(m))
        assert fn(c, m, len(m), n24, key) == 0
        assert c.raw[:16] == bytes(16) and c.raw[16:32].hex() == v["tag"]
        assert hashlib.sha256(c.raw).hexdigest() == v["sha256"]
        if "c" in v:
            assert c.raw.hex() == v["c"]
    out = ctypes.create_string_buffer(b"\x33" * len(m), len(m))
    assert lib.cz_box_open_afternm(out, c.raw, len(m), n24, key) == -1
    assert out.raw == b"\x33" * len(m)


@pytest.mark.parametrize("one_max", [80 << 10, 1 << 22])
def test_nacl_one_multi_pass_against_oracle(L, torch_dev, one_max):
    """k_nacl_one past one pass (boxes > 80 KiB walk several passes of 5 blocks per thread, the MAC
    joined as G r^(n_L) + A_L): random m (zero and non-zero m[0:32]) at sizes around the pass and
    thread edges, against the oracle; with cz_tune("nacl_one_max") at 4 MiB the zero-prefix seals
    and every open take it too, otherwise the segment kernels -- both must agree with NaCl."""
    from cz_testlib import or_box_afternm, or_box_open_afternm
    lib = L.lib()
    old = lib.cz_tune(b"nacl_one_max", one_max)
    try:
        rng = np.random.default_rng(one_max & 0xffff)
        key = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
        sizes = [81920, 81921, 81953, 81920 + 64 * 256, 163840, 163841 + 15, 409600 + 7, 1 << 20, 3 * (1 << 20) + 33]
        for j, mlen in enumerate(sizes):
            n24 = rng.integers(0, 256, 24, dtype=np.uint8).tobytes()
            body = rng.integers(0, 256, mlen - 32, dtype=np.uint8).tobytes()
            for m in (bytes(32) + body, rng.integers(0, 256, 32, dtype=np.uint8).tobytes() + body):
                rc, want = or_box_afternm(m, n24, key)
                assert rc == 0
                c = ctypes.create_string_buffer(mlen)
                assert lib.cz_box_afternm(c, m, mlen, n24, key) == 0, (mlen, L.last_error())
                assert c.raw == want, (mlen, m[:32] == bytes(32))
            # open the zero-prefix box; tamper the last byte
            _, want = or_box_afternm(bytes(32) + body, n24, key)
            back = ctypes.create_string_buffer(mlen)
            assert lib.cz_box_open_afternm(back, want, mlen, n24, key) == 0
            assert back.raw == bytes(32) + body
            bad = bytearray(want)
            bad[-1] ^= 1
            assert or_box_open_afternm(bytes(bad), n24, key)[0] == -1
            back2 = ctypes.create_string_buffer(b"\x11" * mlen, mlen)
            assert lib.cz_box_open_afternm(back2, bytes(bad), mlen, n24, key) == -1
            assert back2.raw == b"\x11" * mlen
    finally:
        lib.cz_tune(b"nacl_one_max", old)


def test_nacl_single_shot_multi_lane(L, torch_dev):
    """The jnacl drop-ins (Curve.java:129-147) for one message of any size: large boxes run through the
    segment kernels (many lanes); every byte and tag against the oracle (NaCl secretbox), m[32] any
    byte value, tampering anywhere -> -1 with the output buffer untouched."""
    from cz_testlib import or_box_afternm
    lib = L.lib()
    rng = np.random.default_rng(77)
    for mlen in (32, 33, 34, 63, 64, 95, 96, 97, 160, 1000, 4128, 4129, 16416, 65568, 65568 + 33 + 64 * 7, 200003):
        key = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
        n24 = rng.integers(0, 256, 24, dtype=np.uint8).tobytes()
        m = bytes(32) + rng.integers(0, 256, mlen - 32, dtype=np.uint8).tobytes()
        rc, want = or_box_afternm(m, n24, key)
        assert rc == 0
        c = ctypes.create_string_buffer(mlen)
        assert lib.cz_box_afternm(c, m, mlen, n24, key) == 0, mlen
        assert c.raw == want, f"box mismatch at mlen={mlen}"
        c2 = ctypes.create_string_buffer(mlen)
        assert lib.cz_secretbox(c2, m, mlen, n24, key) == 0 and c2.raw == want
        out = ctypes.create_string_buffer(mlen)
        assert lib.cz_box_open_afternm(out, want, mlen, n24, key) == 0 and out.raw == m, mlen
        for pos in sorted({16, 31, 32, mlen - 1, (mlen + 32) // 2}):
            if pos >= mlen:
                continue
            bad = bytearray(want)
            bad[pos] ^= 0x40
            sentinel = ctypes.create_string_buffer(b"\xaa" * mlen, mlen)
            assert lib.cz_secretbox_open(sentinel, bytes(bad), mlen, n24, key) == -1, (mlen, pos)
            assert sentinel.raw == b"\xaa" * mlen
        # bytes 0..15 of c are not authenticated (NaCl ignores them)
        junk = bytearray(want)
        junk[:16] = b"\x55" * 16
        assert lib.cz_box_open_afternm(out, bytes(junk), mlen, n24, key) == 0 and out.raw == m


def test_mechanism_client_server(L, torch_dev):
    from jeromq_amd.mechanism import CurveClientMechanism, CurveServerMechanism, Msg
    cli = CurveClientMechanism(PRECOM)
    srv = CurveServerMechanism(PRECOM)
    payloads = [splitmix_bytes(n, 40 + n) for n in (0, 1, 32, 100, 4096, 70000)]
    for i, p in enumerate(payloads):
        enc = cli.encode(Msg(p, i & 3))
        assert enc.data == or_curve_encode(p, i & 3, 3 + i, 0, PRECOM)
        dec = srv.decode(enc)
        assert dec is not None and dec.data == p and dec.flags == i & 3
    assert cli.cnNonce == 3 + len(payloads) and srv.cnPeerNonce == 2 + len(payloads)
    # replay: the same body again is an INVALID_SEQUENCE on the server ...
    again = cli.encode(Msg(b"hello"))
    assert srv.decode(again) is not None
    assert srv.decode(again) is None and srv.last_event == L.CZ_ZMTP_INVALID_SEQUENCE
    # ... and CRYPTOGRAPHIC on the client (CurveClientMechanism.java:188-191)
    back = srv.encode(Msg(b"pong", Msg.MORE))
    assert cli.decode(back).data == b"pong"
    assert cli.decode(back) is None and cli.last_event == L.CZ_ZMTP_CRYPTOGRAPHIC
    bad = bytearray(srv.encode(Msg(b"tamper")).data)
    bad[-1] ^= 1
    assert cli.decode(Msg(bytes(bad))) is None and cli.last_event == L.CZ_ZMTP_CRYPTOGRAPHIC
    assert cli.decode(Msg(b"\x07MESSAGE" + bytes(10))) is None
    assert cli.last_event == L.CZ_ZMTP_MALFORMED_COMMAND_MESSAGE
    assert cli.decode(Msg(b"\x05READY" + bytes(40))) is None and cli.last_event == L.CZ_ZMTP_UNEXPECTED_COMMAND


def test_mechanism_limits_and_flags(L, torch_dev):
    """oversized payloads are refused before any device work (a u32 mlen would wrap), and
    decode / decodeBatch map the decrypted flags byte to MORE | COMMAND only, as the reference does
    (CurveClientMechanism.java:207-213) -- a 0xff flags byte gives MORE | COMMAND, not 0xff."""
    import ctypes
    from jeromq_amd import _lib
    from jeromq_amd.mechanism import CurveClientMechanism, CurveServerMechanism, Msg
    cli = CurveClientMechanism(PRECOM)
    srv = CurveServerMechanism(PRECOM)
    buf = ctypes.create_string_buffer(64)
    assert _lib.lib().cz_mech_encode(cli._h, buf, L.CZ_MESSAGE_MAX + 1, 0, buf) == L.CZ_EMSGSIZE
    assert _lib.lib().cz_mech_encode(cli._h, buf, 1 << 32, 0, buf) == L.CZ_EMSGSIZE
    lens = (ctypes.c_uint32 * 2)(3, 0xffffffff)
    offs = (ctypes.c_uint64 * 2)(0, 0)
    assert _lib.lib().cz_mech_encode_batch(cli._h, 2, buf, offs, lens, None, buf, offs) == L.CZ_EMSGSIZE
    assert cli.cnNonce == 3                                   # nothing was sealed
    body = or_curve_encode(b"payload", 0xff, 3, 0, PRECOM)    # flags byte 0xff from a foreign peer
    got = srv.decode(Msg(body))
    assert got.data == b"payload" and got.flags == Msg.MORE | Msg.COMMAND
    srv2 = CurveServerMechanism(PRECOM)
    got = srv2.decodeBatch([Msg(body), Msg(or_curve_encode(b"x", 0xfc, 4, 0, PRECOM))])
    assert [g.flags for g in got] == [Msg.MORE | Msg.COMMAND, 0]


def test_mechanism_batches(L, torch_dev):
    from jeromq_amd.mechanism import CurveClientMechanism, CurveServerMechanism, Msg
    cli = CurveClientMechanism(PRECOM)
    srv = CurveServerMechanism(PRECOM)
    msgs = [Msg(splitmix_bytes(n, n), n & 1) for n in range(0, 300, 7)]
    enc = cli.encodeBatch(msgs)
    for i, (m, e) in enumerate(zip(msgs, enc)):
        assert e.data == or_curve_encode(m.data, m.flags, 3 + i, 0, PRECOM)
    enc[20] = Msg(enc[20].data[:-1] + bytes([enc[20].data[-1] ^ 1]))
    dec = srv.decodeBatch(enc)
    assert len(dec) == 20 and all(d.data == m.data and d.flags == m.flags for d, m in zip(dec, msgs))
    assert srv.last_event == L.CZ_ZMTP_CRYPTOGRAPHIC


def test_mechanism_one_launch_and_segmented_paths(L, torch_dev):
    """encode / decode of one MESSAGE up to 2 MiB (cz_tune "nacl_one_max") run in one launch
    (k_nacl_one, one pass up to 80 KiB, several above) with the mechanism's own subkeys; longer ones
    and batches run the segment kernels with the segment length scaled to the batch.  Bodies against
    the oracle on both sides of the one-pass 80 KiB edge and of the one-launch edge (the default and
    one moved to 80 KiB), a ragged batch of long and short frames, and the header rejections of the
    one-launch path (short body, wrong command, replay) against the reference's events."""
    from jeromq_amd.mechanism import CurveClientMechanism, CurveServerMechanism, Msg
    cli = CurveClientMechanism(PRECOM)
    srv = CurveServerMechanism(PRECOM)
    nonce = 3
    lib = L.lib()
    for knob in (2 << 20, 80 << 10):
        old = lib.cz_tune(b"nacl_one_max", knob)
        try:
            for n in (81919 - 33, 81920 - 33, 81921 - 33, 200000, (2 << 20) - 33, (2 << 20) - 32):
                p = splitmix_bytes(n, n)
                enc = cli.encode(Msg(p, 1))
                assert enc.data == or_curve_encode(p, 1, nonce, 0, PRECOM), (knob, n)
                dec = srv.decode(enc)
                assert dec is not None and dec.data == p and dec.flags == 1, (knob, n)
                nonce += 1
        finally:
            lib.cz_tune(b"nacl_one_max", old)
    msgs = [Msg(splitmix_bytes(n, 7 * n + 1), n & 3) for n in (100000, 1, 5000, 0, 300000, 64)]
    enc = cli.encodeBatch(msgs)
    for i, (m, e) in enumerate(zip(msgs, enc)):
        assert e.data == or_curve_encode(m.data, m.flags, nonce + i, 0, PRECOM), i
    dec = srv.decodeBatch(enc)
    assert [d.data for d in dec] == [m.data for m in msgs] and [d.flags for d in dec] == [m.flags for m in msgs]
    assert srv.cnPeerNonce == nonce + len(msgs) - 1
    # one-launch decode rejections: nothing changes but the event (and cnPeerNonce on a bad tag)
    before = srv.cnPeerNonce
    assert srv.decode(Msg(b"\x07MESS")) is None and srv.last_event == L.CZ_ZMTP_UNEXPECTED_COMMAND
    assert srv.decode(enc[-1]) is None and srv.last_event == L.CZ_ZMTP_INVALID_SEQUENCE
    assert srv.cnPeerNonce == before
    fresh = bytearray(cli.encode(Msg(b"tampered")).data)
    fresh[20] ^= 0x40                                        # the tag
    assert srv.decode(Msg(bytes(fresh))) is None and srv.last_event == L.CZ_ZMTP_CRYPTOGRAPHIC
    assert srv.cnPeerNonce == before + 1                     # set before the tag check (:193)
    # byte 7 of the command name is not compared (Msgs.java:31), as the kernels do
    odd = bytearray(cli.encode(Msg(b"ok", 2)).data)
    odd[7] ^= 0x55
    got = srv.decode(Msg(bytes(odd)))
    assert got is not None and got.data == b"ok" and got.flags == 2


def test_ctx_host_staged(L, torch_dev):
    lib = L.lib()
    ctx = ctypes.c_void_p()
    L.check(lib.cz_ctx_create(ctypes.byref(ctx), 0))
    try:
        L.check(lib.cz_ctx_set_keys(ctx, PRECOM, 1, L.CZ_DIR_S2C))
        sizes = [0, 10, 100, 1000, 5000, 200000, 70000, 64]
        frames = [(splitmix_bytes(n, 3 * n), 1, 2 + i, 0) for i, n in enumerate(sizes)]
        desc, hin, ob = _pack(frames)
        hout = np.zeros(ob, dtype=np.uint8)
        L.check(lib.cz_ctx_seal(ctx, desc.ctypes.data, len(desc), hin.ctypes.data, hin.nbytes, hout.ctypes.data,
                                hout.nbytes))
        for i, (p, fl, ctr, k) in enumerate(frames):
            o = int(desc[i]["out_off"])
            assert hout[o:o + len(p) + 33].tobytes() == or_curve_encode(p, fl, ctr, 1, PRECOM)
        # cz_ctx_open of the same bodies: nonce floors chained through prev, a bad tag in frame 5
        # (200 KB: several segments, the combine kernel's reject) and a replay in frame 7
        bodies = [hout[int(d["out_off"]):int(d["out_off"]) + int(d["len"]) + 33].tobytes() for d in desc]
        bodies[5] = bodies[5][:100] + bytes([bodies[5][100] ^ 1]) + bodies[5][101:]
        bodies[7] = bodies[7][:8] + bodies[6][8:16] + bodies[7][16:]
        odesc, obody, pb = _pack([(b, 0, 0, 0) for b in bodies], overhead=-33)
        odesc["counter"] = 1
        odesc["flags"] = L.CZ_DESC_CHECK_NONCE
        odesc["prev"] = np.arange(len(bodies)) - 1
        plain = np.full(pb, 0xEE, dtype=np.uint8)
        st = np.full(len(bodies), 0xFFFF, dtype=np.uint16)
        L.check(lib.cz_ctx_open(ctx, odesc.ctypes.data, len(odesc), obody.ctypes.data, obody.nbytes,
                                plain.ctypes.data, plain.nbytes, st.ctypes.data))
        want = [L.CZ_STATUS_OK] * len(bodies)
        want[5], want[7] = L.CZ_STATUS_CRYPTO, L.CZ_STATUS_SEQUENCE
        assert list(st & 0xff) == want
        for i, (p, fl, _c, _k) in enumerate(frames):
            o = int(odesc[i]["out_off"])
            if want[i] == L.CZ_STATUS_OK:
                assert plain[o:o + len(p)].tobytes() == p and st[i] >> 8 == fl, i
            else:
                assert not plain[o:o + len(p)].any(), i
        # out-of-bounds descriptor is rejected before any launch
        bad = desc.copy()
        bad["in_off"][0] = hin.nbytes
        bad["len"][0] = 1
        assert lib.cz_ctx_seal(ctx, bad.ctypes.data, len(bad), hin.ctypes.data, hin.nbytes, hout.ctypes.data,
                               hout.nbytes) == L.CZ_EINVAL
    finally:
        lib.cz_ctx_destroy(ctx)


@pytest.mark.parametrize("chunk", [96, 0])
def test_ctx_pipelined_uniform(L, torch_dev, chunk):
    """Host-staged pipelined seal/open (3 streams, chunks of 96 frames) vs the oracle; chunk
    boundaries carry the replay floor across chunks.  chunk=0: the default chunk holds the whole
    688 KB batch, which runs on one stream (SMALL_BATCH_BYTES)."""
    lib = L.lib()
    ctx = ctypes.c_void_p()
    L.check(lib.cz_ctx_create(ctypes.byref(ctx), 0))
    try:
        L.check(lib.cz_ctx_set_keys(ctx, PRECOM, 1, L.CZ_DIR_C2S))
        count, n, ist, ost = 1000, 300, 304, 384
        hin = np.frombuffer(splitmix_bytes(count * ist, 1234), dtype=np.uint8).copy()
        flags = (np.arange(count) % 3).astype(np.uint8)
        hout = np.zeros(count * ost, dtype=np.uint8)
        L.check(lib.cz_ctx_seal_uniform(ctx, count, n, hin.ctypes.data, ist, hout.ctypes.data, ost, 7,
                                        flags.ctypes.data, chunk))
        for i in (0, 95, 96, 500, count - 1):
            body = hout[i * ost:i * ost + n + 33].tobytes()
            assert body == or_curve_encode(hin[i * ist:i * ist + n].tobytes(), int(flags[i]), 7 + i, 0, PRECOM)
        back = np.zeros(count * ist, dtype=np.uint8)
        st = np.zeros(count, dtype=np.uint16)
        L.check(lib.cz_ctx_set_keys(ctx, PRECOM, 1, L.CZ_DIR_C2S))
        L.check(lib.cz_ctx_open_uniform(ctx, count, n + 33, hout.ctypes.data, ost, back.ctypes.data, ist, 6, 1,
                                        st.ctypes.data, chunk))
        assert not np.any(st & 0xff)
        assert np.array_equal(st >> 8, flags)
        assert np.array_equal(back.reshape(count, ist)[:, :n], hin.reshape(count, ist)[:, :n])
        # a replayed frame at a chunk boundary is caught with the floor carried across chunks
        hout2 = hout.copy()
        hout2[96 * ost + 8:96 * ost + 16] = hout2[95 * ost + 8:95 * ost + 16]
        L.check(lib.cz_ctx_open_uniform(ctx, count, n + 33, hout2.ctypes.data, ost, back.ctypes.data, ist, 6, 1,
                                        st.ctypes.data, chunk))
        assert (st[96] & 0xff) == L.CZ_STATUS_SEQUENCE and not np.any(st[:96] & 0xff)
    finally:
        lib.cz_ctx_destroy(ctx)


def test_ctx_uniform_default_chunks(L, torch_dev):
    """chunk_frames = 0 on a batch of frames too short for the segment path: 20000 x 100 B in
    the default chunks of 16384 frames, three streams; frames around the chunk boundary against
    the oracle and the whole open round trip, with the replay floor carried across chunks."""
    lib = L.lib()
    ctx = ctypes.c_void_p()
    L.check(lib.cz_ctx_create(ctypes.byref(ctx), 0))
    try:
        L.check(lib.cz_ctx_set_keys(ctx, PRECOM, 1, L.CZ_DIR_C2S))
        count, n, ist, ost = 20000, 100, 112, 144
        hin = np.frombuffer(splitmix_bytes(count * ist, 4321), dtype=np.uint8).copy()
        hout = np.zeros(count * ost, dtype=np.uint8)
        L.check(lib.cz_ctx_seal_uniform(ctx, count, n, hin.ctypes.data, ist, hout.ctypes.data, ost, 5, None, 0))
        for i in (0, 1, 16383, 16384, 16385, count - 1):
            body = hout[i * ost:i * ost + n + 33].tobytes()
            assert body == or_curve_encode(hin[i * ist:i * ist + n].tobytes(), 0, 5 + i, 0, PRECOM), i
        back = np.zeros(count * ist, dtype=np.uint8)
        st = np.full(count, 0xFFFF, dtype=np.uint16)
        L.check(lib.cz_ctx_open_uniform(ctx, count, n + 33, hout.ctypes.data, ost, back.ctypes.data, ist, 4, 1,
                                        st.ctypes.data, 0))
        assert not np.any(st)
        assert np.array_equal(back.reshape(count, ist)[:, :n], hin.reshape(count, ist)[:, :n])
        bad = hout.copy()
        e = 16384  # replay at the chunk edge
        bad[e * ost + 8:e * ost + 16] = bad[(e - 1) * ost + 8:(e - 1) * ost + 16]
        L.check(lib.cz_ctx_open_uniform(ctx, count, n + 33, bad.ctypes.data, ost, back.ctypes.data, ist, 4, 1,
                                        st.ctypes.data, 0))
        assert (st[e] & 0xff) == L.CZ_STATUS_SEQUENCE and np.count_nonzero(st) == 1
        assert not back[e * ist:e * ist + n].any()
    finally:
        lib.cz_ctx_destroy(ctx)


@pytest.mark.parametrize("count,n,ist,ost", [(300, 4096, 4096, 4224), (1, 4096, 0, 0), (64, 1000, 1000, 1033),
                                             (7, 20000, 20000, 20040)])
def test_ctx_uniform_small_segmented(L, torch_dev, count, n, ist, ost):
    """Small host-staged uniform batches of multi-block frames (one chunk, <= 4 MiB) run the
    segment kernels, segment-major: every body against the oracle, zeros in the slot padding
    (whole slots, as the pipelined path writes them), the open round trip, and rejected frames (bad tag, replay, wrong command) with zeros in
    their payload slots."""
    lib = L.lib()
    ctx = ctypes.c_void_p()
    L.check(lib.cz_ctx_create(ctypes.byref(ctx), 0))
    try:
        L.check(lib.cz_ctx_set_keys(ctx, PRECOM, 1, L.CZ_DIR_C2S))
        si, so = max(ist, n), max(ost, n + 33)
        hin = np.frombuffer(splitmix_bytes(count * si, 77 + n), dtype=np.uint8).copy()
        flags = (np.arange(count) % 3).astype(np.uint8)
        hout = np.full(count * so, 0xCD, dtype=np.uint8)
        L.check(lib.cz_ctx_seal_uniform(ctx, count, n, hin.ctypes.data, ist, hout.ctypes.data, ost, 11,
                                        flags.ctypes.data, 0))
        for i in range(count):
            body = hout[i * so:i * so + n + 33].tobytes()
            assert body == or_curve_encode(hin[i * si:i * si + n].tobytes(), int(flags[i]), 11 + i, 0, PRECOM), i
            assert not hout[i * so + n + 33:(i + 1) * so].any(), i
        back = np.full(count * si, 0xEE, dtype=np.uint8)
        st = np.full(count, 0xFFFF, dtype=np.uint16)
        L.check(lib.cz_ctx_open_uniform(ctx, count, n + 33, hout.ctypes.data, ost, back.ctypes.data, ist, 10, 1,
                                        st.ctypes.data, 0))
        assert not np.any(st & 0xff)
        assert np.array_equal(st >> 8, flags)
        for i in range(count):
            assert np.array_equal(back[i * si:i * si + n], hin[i * si:i * si + n]), i
        if count < 64:
            return
        bad = hout.copy()
        bad[5 * so + 100] ^= 1                                   # ciphertext -> CRYPTO
        bad[17 * so + 8:17 * so + 16] = bad[16 * so + 8:16 * so + 16]  # replay -> SEQUENCE
        bad[40 * so + 2] ^= 0x20                                 # "\x07MEsSAGE" -> COMMAND
        back[:] = 0xEE
        L.check(lib.cz_ctx_open_uniform(ctx, count, n + 33, bad.ctypes.data, ost, back.ctypes.data, ist, 10, 1,
                                        st.ctypes.data, 0))
        want = np.zeros(count, dtype=np.uint16)
        want[5], want[17], want[40] = L.CZ_STATUS_CRYPTO, L.CZ_STATUS_SEQUENCE, L.CZ_STATUS_COMMAND
        assert np.array_equal(st & 0xff, want), np.nonzero((st & 0xff) != want)
        for i in (5, 17, 40):
            assert not back[i * si:i * si + n].any(), i
        for i in (4, 18, 41, count - 1):
            assert np.array_equal(back[i * si:i * si + n], hin[i * si:i * si + n]), i
    finally:
        lib.cz_ctx_destroy(ctx)


@pytest.mark.parametrize("n,ist,ost", [(4096, 4096, 4224), (1000, 1003, 1100)])
def test_ctx_uniform_paths_write_identical_whole_slots(L, torch_dev, n, ist, ost):
    """the one-chunk segment path (chunk_frames 0) and the pipelined path (chunks of 64
    frames) return byte-identical output buffers for the same frames -- bodies, zero slot padding,
    and for the open zeros in a rejected frame's slot -- into host buffers pre-filled with garbage."""
    lib = L.lib()
    ctx = ctypes.c_void_p()
    L.check(lib.cz_ctx_create(ctypes.byref(ctx), 0))
    try:
        L.check(lib.cz_ctx_set_keys(ctx, PRECOM, 1, L.CZ_DIR_C2S))
        count = 300
        hin = np.frombuffer(splitmix_bytes(count * ist, 5 + n), dtype=np.uint8).copy()
        outs, backs = [], []
        for chunk, fill in ((0, 0xCD), (64, 0x5A)):
            hout = np.full(count * ost, fill, dtype=np.uint8)
            L.check(lib.cz_ctx_seal_uniform(ctx, count, n, hin.ctypes.data, ist, hout.ctypes.data, ost, 9, None,
                                            chunk))
            outs.append(hout)
        assert np.array_equal(outs[0], outs[1])
        slots = outs[0].reshape(count, ost)
        assert not slots[:, n + 33:].any()
        assert slots[7, :n + 33].tobytes() == or_curve_encode(hin[7 * ist:7 * ist + n].tobytes(), 0, 16, 0, PRECOM)
        bad = outs[0].copy()
        bad[3 * ost + 60] ^= 1
        for chunk, fill in ((0, 0xEE), (64, 0x11)):
            back = np.full(count * ist, fill, dtype=np.uint8)
            st = np.zeros(count, dtype=np.uint16)
            L.check(lib.cz_ctx_open_uniform(ctx, count, n + 33, bad.ctypes.data, ost, back.ctypes.data, ist, 8, 1,
                                            st.ctypes.data, chunk))
            assert (st[3] & 0xff) == L.CZ_STATUS_CRYPTO and np.count_nonzero(st & 0xff) == 1
            backs.append(back)
        assert np.array_equal(backs[0], backs[1])
        plain = backs[0].reshape(count, ist)
        assert not plain[3].any() and not plain[:, n:].any()
        assert np.array_equal(plain[4, :n], hin[4 * ist:4 * ist + n])
    finally:
        lib.cz_ctx_destroy(ctx)


@pytest.mark.parametrize("count,n", [(1 << 20, 100), (1 << 20, 4096)])
def test_full_size_roundtrip(torch_dev, subkeys, count, n):
    """BASELINE configs 2 and 3 at full size: seal -> open round trip; every sealed body against the
    multi-threaded oracle, every opened payload against the input."""
    torch, dev = torch_dev
    from jeromq_amd import batch
    in_stride = (n + 15) // 16 * 16
    out_stride = (n + 33 + 127) // 128 * 128 if n >= 1024 else (n + 33 + 15) // 16 * 16
    d_in = torch.empty(count * in_stride, dtype=torch.uint8, device=dev)
    batch.fill(d_in, 0x5EED0000 + n)
    d_out = torch.empty(count * out_stride, dtype=torch.uint8, device=dev)
    batch.seal_uniform(d_in, in_stride, d_out, out_stride, count, n, subkeys[0], 3)
    d_plain = torch.zeros_like(d_in)
    status = torch.full((count,), -1, dtype=torch.int16, device=dev)
    batch.open_uniform(d_out, out_stride, d_plain, in_stride, count, n + 33, subkeys[0], 2, status)
    torch.cuda.synchronize()
    assert int((status != 0).sum()) == 0
    if in_stride == n:
        assert torch.equal(d_plain, d_in)
    else:
        assert torch.equal(d_plain.view(count, in_stride)[:, :n], d_in.view(count, in_stride)[:, :n])
    # EVERY frame against the oracle, and the slot padding is zero
    desc = np.zeros(count, dtype=DESC_DTYPE)
    desc["in_off"] = np.arange(count, dtype=np.uint64) * np.uint64(in_stride)
    desc["out_off"] = np.arange(count, dtype=np.uint64) * np.uint64(out_stride)
    desc["len"] = n
    desc["counter"] = 3 + np.arange(count, dtype=np.uint64)
    desc["prev"] = -1
    assert oracle_check_full(d_in, d_out, desc, PRECOM) == count
    if out_stride > n + 33:
        assert not d_out.view(count, out_stride)[:, n + 33:].any()
    del d_in, d_out, d_plain
    torch.cuda.empty_cache()
