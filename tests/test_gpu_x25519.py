"""GPU: X25519 / crypto_box_beforenm / crypto_box on gfx950 against the libsodium fixtures
(tests/golden/x25519_vectors.json) and the oracle, bit-exact."""
import numpy as np
import pytest

from cz_testlib import load_x25519_golden, or_beforenm, or_x25519, splitmix_bytes

pytestmark = pytest.mark.gpu
X = load_x25519_golden()


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch, torch.device("cuda:0")


def _batch(torch_dev, fn, a, b):
    torch, dev = torch_dev
    from jeromq_amd import _lib
    n = len(a)
    da = torch.from_numpy(np.frombuffer(b"".join(a), dtype=np.uint8).copy()).to(dev)
    db = None if b is None else torch.from_numpy(np.frombuffer(b"".join(b), dtype=np.uint8).copy()).to(dev)
    out = torch.zeros(32 * n, dtype=torch.uint8, device=dev)
    L = _lib.lib()
    if fn == "x25519":
        rc = L.cz_x25519_batch(da.data_ptr(), None if db is None else db.data_ptr(), out.data_ptr(), n, None)
    else:   # beforenm(pk=a, sk=b)
        rc = L.cz_beforenm_batch(da.data_ptr(), db.data_ptr(), out.data_ptr(), n, None)
    _lib.check(rc, fn)
    torch.cuda.synchronize()
    o = out.cpu().numpy().tobytes()
    return [o[32 * i:32 * i + 32] for i in range(n)]


def test_x25519_batch_golden(torch_dev):
    vs = X["x25519"]
    got = _batch(torch_dev, "x25519", [bytes.fromhex(v["k"]) for v in vs], [bytes.fromhex(v["u"]) for v in vs])
    for v, g in zip(vs, got):
        assert g.hex() == v["out"], v["case"]


def test_base_point_batch_gives_reference_publics(torch_dev):
    sks = [bytes.fromhex(v["k"]) for v in X["x25519"] if "keypair" in v["case"]]
    pks = [bytes.fromhex(v["out"]) for v in X["x25519"] if "keypair" in v["case"]]
    assert _batch(torch_dev, "x25519", sks, None) == pks


def test_beforenm_batch_and_single_golden(torch_dev):
    from jeromq_amd.curve import Curve
    vs = X["beforenm"]
    got = _batch(torch_dev, "beforenm", [bytes.fromhex(v["pk"]) for v in vs], [bytes.fromhex(v["sk"]) for v in vs])
    for v, g in zip(vs, got):
        assert g.hex() == v["k"], v["case"]
    c = Curve()
    for v in vs[:4]:
        k = bytearray(32)
        assert c.beforenm(k, bytes.fromhex(v["pk"]), bytes.fromhex(v["sk"])) == 0
        assert bytes(k).hex() == v["k"]


def test_iterated_single_calls(torch_dev):
    from jeromq_amd.curve import scalarmult
    k = u = (9).to_bytes(32, "little")
    k, u = scalarmult(k, u), k
    assert k.hex() == X["iterated_1"]
    for _ in range(999):
        k, u = scalarmult(k, u), k
    assert k.hex() == X["iterated_1000"]


def test_random_batch_vs_oracle(torch_dev):
    rng = np.random.default_rng(25519)
    n = 2048
    ks = [rng.integers(0, 256, 32, dtype=np.uint8).tobytes() for _ in range(n)]
    us = [rng.integers(0, 256, 32, dtype=np.uint8).tobytes() for _ in range(n)]   # incl. non-canonical u
    got = _batch(torch_dev, "x25519", ks, us)
    for i in range(0, n, 7):
        assert got[i] == or_x25519(ks[i], us[i]), i
    assert _batch(torch_dev, "x25519", [bytes(range(32))], [bytes(32)]) == [bytes(32)]   # order-2 point -> 0


def test_box_open_and_keypair(torch_dev):
    from jeromq_amd.curve import Curve, scalarmult
    c = Curve()
    for v in X["box"]:
        m = bytes(32) + splitmix_bytes(v["n"], v["m_seed"])
        ct = bytearray(len(m))
        assert c.box(ct, m, len(m), bytes.fromhex(v["nonce"]), bytes.fromhex(v["pk"]), bytes.fromhex(v["sk"])) == 0
        assert bytes(ct).hex() == v["c"]
    # box between two fresh key pairs, opened by the peer; tampering fails with -1
    a_pk, a_sk = c.keypair()
    b_pk, b_sk = c.keypair()
    assert a_pk == scalarmult(a_sk, (9).to_bytes(32, "little")) and a_sk != b_sk
    assert or_beforenm(b_pk, a_sk) == or_beforenm(a_pk, b_sk)
    nonce = bytes(range(24))
    m = bytes(32) + b"HELLO from the client"
    ct = bytearray(len(m))
    assert c.box(ct, m, len(m), nonce, b_pk, a_sk) == 0
    pt = bytearray(len(m))
    assert c.open(pt, bytes(ct), len(ct), nonce, a_pk, b_sk) == 0 and bytes(pt[32:]) == m[32:]
    ct[40] ^= 1
    assert c.open(pt, bytes(ct), len(ct), nonce, a_pk, b_sk) == -1
