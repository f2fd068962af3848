#!/usr/bin/env python3
"""Generate the golden fixtures for the CURVE MESSAGE path.

Run in the build container (NOT on the GPU box): it needs libsodium 1.0.18 at
/opt/conda/lib/libsodium.so, an independent implementation of the NaCl
construction that JeroMQ reaches through jnacl (Curve.java:5-6, 129-147).
jnacl itself is not vendored in /root/reference and no JDK exists here, so the
fixtures are produced by libsodium, anchored on:
  * the CurveZMQ test key pairs published in the reference
    (jeromq-core/src/main/java/org/zeromq/ZMQ.java:4603-4624,
     jeromq-core/src/test/java/zmq/HeartbeatsTest.java:402-414);
  * the MESSAGE framing of CurveClientMechanism.encode (CurveClientMechanism.java:126-163)
    and CurveServerMechanism.encode (CurveServerMechanism.java:127-163):
      body = "\\x07MESSAGE" || BE64(counter) || box[16:mlen],  mlen = 33 + n
  * the case list of SURVEY.md section 8(c): payload sizes, flags, directions,
    counters and tamper cases.

Writes tests/golden/curve_vectors.json.  Payloads are the counter-based
SplitMix64 byte stream (tests/cz_testlib.py:splitmix_bytes) so the file stays small.
"""
import ctypes
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from cz_testlib import splitmix_bytes  # noqa: E402

SODIUM = ctypes.CDLL("/opt/conda/lib/libsodium.so")
assert SODIUM.sodium_init() >= 0

# org/zeromq/ZMQ.java:4603-4624 (CurveZMQ RFC 26 test keys)
CLIENT_PUB = bytes.fromhex("BB88471D65E2659B30C55A5321CEBB5AAB2B70A398645C26DCA2B2FCB43FC518")
CLIENT_SEC = bytes.fromhex("7BB864B489AFA3671FBE69101F94B38972F24816DFB01B51656B3FEC8DFD0888")
SERVER_PUB = bytes.fromhex("54FCBA24E93249969316FB617C872BB0C1D1FF14800427C594CBFACF1BC2D652")
SERVER_SEC = bytes.fromhex("8E0BDD697628B91D8F245587EE95C5B04D48963F79259877B49CD9063AEAD3B7")


def buf(n):
    return ctypes.create_string_buffer(n)


def scalarmult_base(sk):
    out = buf(32)
    assert SODIUM.crypto_scalarmult_base(out, sk) == 0
    return out.raw


def beforenm(pk, sk):
    out = buf(32)
    assert SODIUM.crypto_box_beforenm(out, pk, sk) == 0
    return out.raw


def hsalsa20(in16, key):
    out = buf(32)
    assert SODIUM.crypto_core_hsalsa20(out, in16, key, None) == 0
    return out.raw


def salsa20_stream(length, nonce8, ic, key):
    out = buf(length)
    zeros = bytes(length)
    assert SODIUM.crypto_stream_salsa20_xor_ic(out, zeros, ctypes.c_ulonglong(length), nonce8,
                                               ctypes.c_uint64(ic), key) == 0
    return out.raw


def poly1305(msg, key):
    out = buf(16)
    assert SODIUM.crypto_onetimeauth_poly1305(out, msg, ctypes.c_ulonglong(len(msg)), key) == 0
    return out.raw


def box_afternm(m, n24, k):
    c = buf(len(m))
    rc = SODIUM.crypto_box_afternm(c, m, ctypes.c_ulonglong(len(m)), n24, k)
    return rc, c.raw


def box_open_afternm(c, n24, k):
    m = buf(len(c))
    rc = SODIUM.crypto_box_open_afternm(m, c, ctypes.c_ulonglong(len(c)), n24, k)
    return rc, m.raw


def curve_nonce(from_server, counter):
    prefix = b"CurveZMQMESSAGES" if from_server else b"CurveZMQMESSAGEC"
    return prefix + counter.to_bytes(8, "big")


def curve_body(payload, flags, counter, from_server, k):
    """CurveClientMechanism.encode / CurveServerMechanism.encode via libsodium."""
    n24 = curve_nonce(from_server, counter)
    m = bytes(32) + bytes([flags]) + payload
    rc, c = box_afternm(m, n24, k)
    assert rc == 0
    return b"\x07MESSAGE" + n24[16:] + c[16:]


def main():
    out = {"generator": "libsodium 1.0.18 via tests/golden/make_golden.py", "keys": {}}
    assert scalarmult_base(CLIENT_SEC) == CLIENT_PUB
    assert scalarmult_base(SERVER_SEC) == SERVER_PUB
    k_client = beforenm(SERVER_PUB, CLIENT_SEC)
    k_server = beforenm(CLIENT_PUB, SERVER_SEC)
    assert k_client == k_server
    k = k_client
    out["keys"] = {
        "client_public": CLIENT_PUB.hex(), "client_secret": CLIENT_SEC.hex(),
        "server_public": SERVER_PUB.hex(), "server_secret": SERVER_SEC.hex(),
        "precom": k.hex(),
        "subkey_c2s": hsalsa20(b"CurveZMQMESSAGEC", k).hex(),
        "subkey_s2c": hsalsa20(b"CurveZMQMESSAGES", k).hex(),
    }

    # HSalsa20 known answers (random inputs)
    hs = []
    for i in range(8):
        key = splitmix_bytes(32, 0x1000 + i)
        in16 = splitmix_bytes(16, 0x2000 + i)
        hs.append({"key": key.hex(), "in": in16.hex(), "out": hsalsa20(in16, key).hex()})
    out["hsalsa20"] = hs

    # Salsa20 keystream with block counter offsets (incl. 32-bit counter carry)
    ss = []
    for i, (length, ic) in enumerate([(64, 0), (200, 1), (130, 0xFFFFFFFF), (64, (1 << 32) + 5), (1000, 7)]):
        key = splitmix_bytes(32, 0x3000 + i)
        nonce8 = splitmix_bytes(8, 0x4000 + i)
        ss.append({"key": key.hex(), "nonce": nonce8.hex(), "ic": ic, "len": length,
                   "stream": salsa20_stream(length, nonce8, ic, key).hex()})
    out["salsa20"] = ss

    # Poly1305 over assorted lengths, plus a key whose s forces the 2^128 wrap
    ps = []
    for i, length in enumerate([0, 1, 15, 16, 17, 31, 32, 33, 63, 64, 65, 255, 256, 1000, 4097]):
        key = splitmix_bytes(32, 0x5000 + i)
        msg = splitmix_bytes(length, 0x6000 + i)
        ps.append({"key": key.hex(), "msg_seed": 0x6000 + i, "len": length, "tag": poly1305(msg, key).hex()})
    for i, length in enumerate([16, 48, 1024]):
        key = bytes([0xFF] * 32)
        msg = bytes([0xFF] * length)
        ps.append({"key": key.hex(), "msg_hex": msg.hex(), "len": length, "tag": poly1305(msg, key).hex()})
    out["poly1305"] = ps

    # NaCl crypto_box_afternm / open with arbitrary 24-byte nonces (jnacl drop-in API)
    bx = []
    for i, n in enumerate([0, 1, 31, 32, 33, 100, 1000, 4096]):
        key = splitmix_bytes(32, 0x7000 + i)
        n24 = splitmix_bytes(24, 0x8000 + i)
        m = bytes(32) + splitmix_bytes(n, 0x9000 + i)
        rc, c = box_afternm(m, n24, key)
        assert rc == 0 and c[:16] == bytes(16)
        rc2, m2 = box_open_afternm(c, n24, key)
        assert rc2 == 0 and m2 == m
        bad = bytearray(c)
        bad[16] ^= 1
        rc3, _ = box_open_afternm(bytes(bad), n24, key)
        assert rc3 == -1
        bx.append({"key": key.hex(), "nonce": n24.hex(), "m_seed": 0x9000 + i, "n": n, "c": c.hex()})
    out["box_afternm"] = bx

    # crypto_box_afternm of an m whose first 32 bytes are NOT zero.  NaCl (and libsodium, and jnacl's
    # port of it) accept it: c = keystream ^ m over all mlen bytes, Poly1305 keyed with
    # c[0:32] = keystream[0:32] ^ m[0:32], tag at c[16:32], c[0:16] = 0.  JeroMQ's public Curve.box
    # (Curve.java:184-193) hands such an m to jnacl.  The open (keyed with the keystream alone) then
    # fails on these boxes, as in NaCl.  Sizes straddle the one-pass / segmented edge (80 KiB).
    bp = []
    for i, mlen in enumerate([32, 33, 133, 4129, 81953]):
        key = splitmix_bytes(32, 0x7100 + i)
        n24 = splitmix_bytes(24, 0x8100 + i)
        m = splitmix_bytes(mlen, 0x9100 + i)
        assert any(m[:32])
        rc, c = box_afternm(m, n24, key)
        assert rc == 0 and c[:16] == bytes(16)
        rc0, c0 = box_afternm(bytes(32) + m[32:], n24, key)
        assert rc0 == 0 and c0[32:] == c[32:] and c0[16:32] != c[16:32]
        rco, _ = box_open_afternm(c, n24, key)
        assert rco == -1
        bp.append({"key": key.hex(), "nonce": n24.hex(), "m_seed": 0x9100 + i, "mlen": mlen,
                   "tag": c[16:32].hex(), "sha256": hashlib.sha256(c).hexdigest(),
                   **({"c": c.hex()} if mlen <= 4129 else {})})
    out["box_afternm_prefix"] = bp

    # CurveZMQ MESSAGE bodies under the RFC test keys (SURVEY.md 8(c) case list)
    sizes = [0, 1, 15, 16, 17, 31, 32, 33, 47, 63, 64, 65, 100, 255, 256, 4096, 65536]
    counters = [2, 3, (1 << 32) - 1, 1 << 32, (1 << 63) - 1]
    msgs = []
    idx = 0
    for n in sizes:
        for from_server in (0, 1):
            for flags in range(4):
                # full counter sweep only on a subset to keep the file small
                cs = counters if (flags == 0 and n <= 4096) else [counters[(idx + flags) % len(counters)]]
                for counter in cs:
                    seed = 0xA0000 + idx
                    payload = splitmix_bytes(n, seed)
                    body = curve_body(payload, flags, counter, from_server, k)
                    assert len(body) == 33 + n
                    rec = {"n": n, "seed": seed, "flags": flags, "counter": counter, "from_server": from_server,
                           "tag": body[16:32].hex(), "sha256": hashlib.sha256(body).hexdigest()}
                    if n <= 4096 or flags == 0:
                        rec["body"] = body.hex()
                    msgs.append(rec)
                    idx += 1
    out["messages"] = msgs

    # The KAT quoted in SURVEY.md 8(c): C->S, payload bytes(range(100)), flags 0, counter 3
    kat = curve_body(bytes(range(100)), 0, 3, 0, k)
    out["survey_kat"] = {"payload_hex": bytes(range(100)).hex(), "flags": 0, "counter": 3, "from_server": 0,
                         "tag": kat[16:32].hex(), "ct8": kat[32:40].hex(), "body": kat.hex()}
    assert out["survey_kat"]["tag"] == "860e3835aa998b0a5b3a9829a03a1189"

    path = os.path.join(HERE, "curve_vectors.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=0, sort_keys=True)
    print(f"wrote {path}: {len(msgs)} MESSAGE vectors, {os.path.getsize(path)} bytes")


if __name__ == "__main__":
    main()
