"""Oracle X25519 / crypto_box_beforenm / crypto_box (oracle/curve_oracle.c) against the
libsodium fixtures of tests/golden/make_golden_x25519.py (RFC 7748 inputs, the reference's
published CurveZMQ key pairs, random pairs, non-canonical u).  CPU only."""
import pytest

from cz_testlib import load_x25519_golden, or_beforenm, or_box, or_x25519, splitmix_bytes

X = load_x25519_golden()


@pytest.mark.parametrize("v", X["x25519"], ids=lambda v: v["case"])
def test_x25519(v):
    assert or_x25519(bytes.fromhex(v["k"]), bytes.fromhex(v["u"])).hex() == v["out"]


def test_iterated():
    k = u = (9).to_bytes(32, "little")
    k, u = or_x25519(k, u), k
    assert k.hex() == X["iterated_1"]
    for _ in range(999):
        k, u = or_x25519(k, u), k
    assert k.hex() == X["iterated_1000"]


@pytest.mark.parametrize("v", X["beforenm"], ids=lambda v: v["case"])
def test_beforenm(v):
    assert or_beforenm(bytes.fromhex(v["pk"]), bytes.fromhex(v["sk"])).hex() == v["k"]


@pytest.mark.parametrize("v", X["box"], ids=lambda v: str(v["n"]))
def test_box(v):
    m = splitmix_bytes(v["n"], v["m_seed"])
    assert or_box(m, bytes.fromhex(v["nonce"]), bytes.fromhex(v["pk"]), bytes.fromhex(v["sk"])).hex() == v["c"]


def test_order_two_point_gives_zero():
    # u = 0 is the point of order 2: every clamped multiple encodes as 0 (jnacl does not reject it)
    assert or_x25519(bytes(range(32)), bytes(32)) == bytes(32)
