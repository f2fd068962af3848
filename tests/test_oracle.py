"""Pin the CPU oracle (oracle/curve_oracle.c) to the golden vectors.

The fixtures come from libsodium 1.0.18 (tests/golden/make_golden.py) because
the reference's NaCl (jnacl, eu.neilalexander:jnacl:1.0.0, jeromq-core/pom.xml:18-22)
is not vendored and no JDK exists in this image.  The reference's own tests hold
no crypto known-answer vectors; the RFC test keys they use
(org/zeromq/ZMQ.java:4603-4624) drive the MESSAGE vectors here.
"""
import numpy as np
import pytest

from cz_testlib import (load_golden, or_box_afternm, or_box_open_afternm, or_curve_decode, or_curve_encode,
                        or_hsalsa20, or_poly1305, or_salsa20_stream, splitmix_bytes)

G = load_golden()
K = bytes.fromhex(G["keys"]["precom"])


def test_subkeys_hoist():
    # the per-direction HSalsa20 subkey is constant per connection
    assert or_hsalsa20(b"CurveZMQMESSAGEC", K).hex() == G["keys"]["subkey_c2s"]
    assert or_hsalsa20(b"CurveZMQMESSAGES", K).hex() == G["keys"]["subkey_s2c"]


@pytest.mark.parametrize("v", G["hsalsa20"])
def test_hsalsa20(v):
    assert or_hsalsa20(bytes.fromhex(v["in"]), bytes.fromhex(v["key"])).hex() == v["out"]


@pytest.mark.parametrize("v", G["salsa20"])
def test_salsa20_stream(v):
    s = or_salsa20_stream(v["len"], bytes.fromhex(v["nonce"]), v["ic"], bytes.fromhex(v["key"]))
    assert s.hex() == v["stream"]


@pytest.mark.parametrize("v", G["poly1305"])
def test_poly1305(v):
    msg = bytes.fromhex(v["msg_hex"]) if "msg_hex" in v else splitmix_bytes(v["len"], v["msg_seed"])
    assert or_poly1305(msg, bytes.fromhex(v["key"])).hex() == v["tag"]


@pytest.mark.parametrize("v", G["box_afternm"])
def test_box_afternm_roundtrip(v):
    key, n24 = bytes.fromhex(v["key"]), bytes.fromhex(v["nonce"])
    m = bytes(32) + splitmix_bytes(v["n"], v["m_seed"])
    rc, c = or_box_afternm(m, n24, key)
    assert rc == 0 and c.hex() == v["c"]
    rc, m2 = or_box_open_afternm(c, n24, key)
    assert rc == 0 and m2 == m
    bad = bytearray(c)
    bad[-1] ^= 0x80
    assert or_box_open_afternm(bytes(bad), n24, key)[0] == -1


@pytest.mark.parametrize("v", G["box_afternm_prefix"])
def test_box_afternm_nonzero_prefix(v):
    """NaCl keys the MAC with c[0:32] = keystream ^ m[0:32]: an m whose first 32 bytes are not zero is
    sealed (rc 0) with the same ciphertext and a different tag (libsodium fixtures)."""
    import hashlib
    key, n24 = bytes.fromhex(v["key"]), bytes.fromhex(v["nonce"])
    m = splitmix_bytes(v["mlen"], v["m_seed"])
    rc, c = or_box_afternm(m, n24, key)
    assert rc == 0 and c[:16] == bytes(16) and c[16:32].hex() == v["tag"]
    assert hashlib.sha256(c).hexdigest() == v["sha256"]
    if "c" in v:
        assert c.hex() == v["c"]
    rc0, c0 = or_box_afternm(bytes(32) + m[32:], n24, key)
    assert rc0 == 0 and c0[32:] == c[32:]
    assert or_box_open_afternm(c, n24, key)[0] == -1  # the open keys the MAC with the keystream


def test_box_short_inputs_rejected():
    key, n24 = bytes(32), bytes(24)
    assert or_box_afternm(bytes(31), n24, key)[0] == -1
    assert or_box_open_afternm(bytes(31), n24, key)[0] == -1


@pytest.mark.parametrize("v", G["messages"], ids=lambda v: f"n{v['n']}-s{v['from_server']}-f{v['flags']}-c{v['counter']}")
def test_curve_message(v):
    import hashlib
    payload = splitmix_bytes(v["n"], v["seed"])
    body = or_curve_encode(payload, v["flags"], v["counter"], v["from_server"], K)
    assert hashlib.sha256(body).hexdigest() == v["sha256"]
    assert body[16:32].hex() == v["tag"]
    if "body" in v:
        assert body.hex() == v["body"]
    rc, p2, flags, nonce = or_curve_decode(body, v["from_server"], K)
    assert rc == 0 and p2 == payload and flags == v["flags"] and nonce == v["counter"]
    # wrong direction prefix -> cryptographic failure
    assert or_curve_decode(body, 1 - v["from_server"], K)[0] == 1


def test_survey_kat():
    kat = G["survey_kat"]
    body = or_curve_encode(bytes.fromhex(kat["payload_hex"]), 0, 3, 0, K)
    assert body.hex() == kat["body"]
    assert body[16:32].hex() == "860e3835aa998b0a5b3a9829a03a1189"
    assert body[32:40].hex() == "a479188bab220f90"


def test_decode_rejects_malformed():
    body = or_curve_encode(b"hello", 0, 3, 0, K)
    assert or_curve_decode(body[:32], 0, K)[0] == 2          # MALFORMED_COMMAND_MESSAGE
    assert or_curve_decode(body[:7], 0, K)[0] == 3           # too short to be a command
    assert or_curve_decode(b"\x07MESSAXE" + body[8:], 0, K)[0] == 3   # UNEXPECTED_COMMAND
    assert or_curve_decode(b"\x08MESSAGE" + body[8:], 0, K)[0] == 3
    # Msgs.startsWith never compares the 7th character (zmq/io/Msgs.java:31): accepted
    rc, payload, _, _ = or_curve_decode(b"\x07MESSAGx" + body[8:], 0, K)
    assert rc == 0 and payload == b"hello"
    bad = bytearray(body)
    bad[20] ^= 1
    assert or_curve_decode(bytes(bad), 0, K)[0] == 1


def test_oracle_check_full_helper():
    """The full-batch checker the GPU parity tests use (cz_testlib.oracle_check_full), exercised on
    CPU tensors: it accepts an oracle-sealed batch in several chunks and names a corrupted frame."""
    import torch
    from cz_testlib import DESC_DTYPE, oracle_check_full, or_curve_encode, splitmix_bytes
    key = bytes(range(32))
    lens = [0, 1, 100, 4096, 5000, 31, 64]
    desc = np.zeros(len(lens), dtype=DESC_DTYPE)
    io = oo = 0
    hin, hout = bytearray(), bytearray()
    for i, n in enumerate(lens):
        p = splitmix_bytes(n, 300 + i)
        desc[i] = (io, oo, n, 0, 3 + i, i & 3, -1)
        hin += p + bytes((-n) % 16)
        body = or_curve_encode(p, i & 3, 3 + i, 0, key)
        hout += body + bytes((-len(body)) % 128)
        io, oo = len(hin), len(hout)
    d_in = torch.frombuffer(bytearray(hin + bytes(16)), dtype=torch.uint8)
    d_out = torch.frombuffer(bytearray(hout), dtype=torch.uint8)
    assert oracle_check_full(d_in, d_out, desc, key, chunk_bytes=300) == len(lens)
    d_out[int(desc["out_off"][4]) + 2000] ^= 1
    with pytest.raises(AssertionError, match="frame 4"):
        oracle_check_full(d_in, d_out, desc, key, chunk_bytes=300)
