#!/usr/bin/env python3
"""Golden fixtures for the CURVE handshake key agreement (X25519, crypto_box_beforenm,
crypto_box / crypto_box_open), generated in the build container with libsodium 1.0.18
(/opt/conda/lib/libsodium.so), an independent implementation of the NaCl calls JeroMQ
makes through jnacl: Curve.beforenm / keypair / box / open (Curve.java:100-193).

Cases:
  * RFC 7748 section 5.2 scalar/u inputs and the iterated k = u = 9 ladder (1 and 1000 steps);
  * the CurveZMQ test key pairs published in the reference (org/zeromq/ZMQ.java:4603-4624):
    public = X25519(secret, 9), and beforenm in both directions;
  * 48 random key pairs (seeded), plus u inputs with bit 255 set or >= p (masked/reduced);
  * crypto_box of SplitMix64 payloads under the reference keys.
Writes tests/golden/x25519_vectors.json.
"""
import ctypes
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from cz_testlib import splitmix_bytes  # noqa: E402

S = ctypes.CDLL("/opt/conda/lib/libsodium.so")
assert S.sodium_init() >= 0

CLIENT_PUB = bytes.fromhex("BB88471D65E2659B30C55A5321CEBB5AAB2B70A398645C26DCA2B2FCB43FC518")
CLIENT_SEC = bytes.fromhex("7BB864B489AFA3671FBE69101F94B38972F24816DFB01B51656B3FEC8DFD0888")
SERVER_PUB = bytes.fromhex("54FCBA24E93249969316FB617C872BB0C1D1FF14800427C594CBFACF1BC2D652")
SERVER_SEC = bytes.fromhex("8E0BDD697628B91D8F245587EE95C5B04D48963F79259877B49CD9063AEAD3B7")
P = 2**255 - 19


def x25519(k, u):
    out = ctypes.create_string_buffer(32)
    rc = S.crypto_scalarmult(out, k, u)
    return out.raw if rc == 0 else None


def beforenm(pk, sk):
    out = ctypes.create_string_buffer(32)
    assert S.crypto_box_beforenm(out, pk, sk) == 0
    return out.raw


def box(m, n, pk, sk):
    mm = bytes(32) + m
    c = ctypes.create_string_buffer(len(mm))
    assert S.crypto_box(c, mm, ctypes.c_ulonglong(len(mm)), n, pk, sk) == 0
    return c.raw


def main():
    out = {"generator": "libsodium 1.0.18 via tests/golden/make_golden_x25519.py", "x25519": [], "beforenm": [],
           "box": []}
    rfc = [("a546e36bf0527c9d3b16154b82465edd62144c0ac1fc5a18506a2244ba449ac4",
            "e6db6867583030db3594c1a424b15f7c726624ec26b3353b10a903a6d0ab1c4c"),
           ("4b66e9d4d1b4673c5ad22691957d6af5c11b6421e0ea01d42ca4169e7918ba0d",
            "e5210f12786811d3f4b7959d0538ae2c31dbe7106fc03c3efc4cd549c715a493")]
    for k, u in rfc:
        r = x25519(bytes.fromhex(k), bytes.fromhex(u))
        out["x25519"].append({"k": k, "u": u, "out": r.hex(), "case": "rfc7748-5.2"})
    # iterated: k, u = X25519(k, u), k
    k = u = (9).to_bytes(32, "little")
    for i in range(1, 1001):
        k, u = x25519(k, u), k
        if i in (1, 1000):
            out["iterated_%d" % i] = k.hex()
    assert out["iterated_1"] == "422c8e7a6227d7bca1350b3e2bb7279f7897b87bb6854b783c60e80311ae3079"
    # reference key pairs
    nine = (9).to_bytes(32, "little")
    assert x25519(CLIENT_SEC, nine) == CLIENT_PUB and x25519(SERVER_SEC, nine) == SERVER_PUB
    for sk, pk, name in ((CLIENT_SEC, CLIENT_PUB, "client"), (SERVER_SEC, SERVER_PUB, "server")):
        out["x25519"].append({"k": sk.hex(), "u": nine.hex(), "out": pk.hex(), "case": "ZMQ.java %s keypair" % name})
    kc = beforenm(SERVER_PUB, CLIENT_SEC)
    ks = beforenm(CLIENT_PUB, SERVER_SEC)
    assert kc == ks == bytes.fromhex("0e8790cb0dc8703af2533cc8594eecfbf62ca560a66ebee1259cc0a30435c6f3")
    out["beforenm"].append({"pk": SERVER_PUB.hex(), "sk": CLIENT_SEC.hex(), "k": kc.hex(), "case": "client"})
    out["beforenm"].append({"pk": CLIENT_PUB.hex(), "sk": SERVER_SEC.hex(), "k": ks.hex(), "case": "server"})
    rng = random.Random(0x25519)
    for i in range(48):
        sk = bytes(rng.randrange(256) for _ in range(32))
        sk2 = bytes(rng.randrange(256) for _ in range(32))
        pk = x25519(sk2, nine)
        out["x25519"].append({"k": sk.hex(), "u": pk.hex(), "out": x25519(sk, pk).hex(), "case": "random"})
        out["beforenm"].append({"pk": pk.hex(), "sk": sk.hex(), "k": beforenm(pk, sk).hex(), "case": "random"})
    # u with bit 255 set (masked) and non-canonical u in [p, 2^255) (reduced mod p)
    for i, uval in enumerate([(1 << 255) | 12345, P + 5, P + 18, (1 << 255) | (P - 3)]):
        sk = bytes(rng.randrange(256) for _ in range(32))
        u = (uval % (1 << 256)).to_bytes(32, "little")
        r = x25519(sk, u)
        if r is not None:
            out["x25519"].append({"k": sk.hex(), "u": u.hex(), "out": r.hex(), "case": "non-canonical u"})
    for i, n in enumerate([0, 1, 16, 100, 1000]):
        m = splitmix_bytes(n, 777 + i)
        nonce = splitmix_bytes(24, 999 + i)
        out["box"].append({"m_seed": 777 + i, "n": n, "nonce": nonce.hex(), "pk": SERVER_PUB.hex(),
                           "sk": CLIENT_SEC.hex(), "c": box(m, nonce, SERVER_PUB, CLIENT_SEC).hex()})
    with open(os.path.join(HERE, "x25519_vectors.json"), "w") as f:
        json.dump(out, f, indent=0, sort_keys=True)
    print("x25519 %d, beforenm %d, box %d" % (len(out["x25519"]), len(out["beforenm"]), len(out["box"])))


if __name__ == "__main__":
    main()
