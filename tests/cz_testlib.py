"""Shared helpers for the test suite: synthetic inputs and the CPU oracle loader.

The oracle (oracle/curve_oracle.c -> oracle/liboracle.so) is test
infrastructure: it is loaded here only to check the product, never by the
product itself.
"""
import ctypes
import json
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden", "curve_vectors.json")

_GAMMA = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def splitmix_words(nwords, seed, start=0):
    """Counter-based SplitMix64: word i = mix(seed + (i+1)*gamma).  Matches or_splitmix64 and cz_fill."""
    with np.errstate(over="ignore"):
        idx = np.arange(start, start + nwords, dtype=np.uint64) + np.uint64(1)
        z = np.uint64(seed) + idx * _GAMMA
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def splitmix_bytes(n, seed):
    w = splitmix_words((n + 7) // 8, seed)
    return w.view(np.uint8)[:n].tobytes()


def load_golden():
    with open(GOLDEN) as f:
        return json.load(f)


# ---- oracle ---------------------------------------------------------------
_ORACLE = None


def oracle():
    """Load (building if needed) the CPU oracle.  Test infrastructure only."""
    global _ORACLE
    if _ORACLE is not None:
        return _ORACLE
    path = os.path.join(ROOT, "oracle", "liboracle.so")
    src = os.path.join(ROOT, "oracle", "curve_oracle.c")
    if not os.path.exists(path) or os.path.getmtime(path) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
    lib = ctypes.CDLL(path)
    P = ctypes.c_char_p
    U64 = ctypes.c_uint64
    lib.or_salsa20_core.argtypes = [P, P, P]
    lib.or_hsalsa20.argtypes = [P, P, P]
    lib.or_salsa20_xor_ic.argtypes = [P, P, U64, P, U64, P]
    lib.or_poly1305.argtypes = [P, P, U64, P]
    lib.or_secretbox.argtypes = [P, P, U64, P, P]
    lib.or_secretbox.restype = ctypes.c_int
    lib.or_secretbox_open.argtypes = [P, P, U64, P, P]
    lib.or_secretbox_open.restype = ctypes.c_int
    lib.or_curve_encode.argtypes = [P, P, U64, ctypes.c_uint8, U64, ctypes.c_int, P]
    lib.or_curve_encode.restype = U64
    lib.or_curve_decode.argtypes = [P, ctypes.POINTER(ctypes.c_uint8), ctypes.POINTER(ctypes.c_uint64), P, U64,
                                    ctypes.c_int, P]
    lib.or_curve_decode.restype = ctypes.c_int
    lib.or_splitmix64.argtypes = [U64, U64]
    lib.or_splitmix64.restype = U64
    lib.or_fill.argtypes = [P, U64, U64]
    lib.or_x25519.argtypes = [P, P, P]
    lib.or_scalarmult_base.argtypes = [P, P]
    lib.or_box_beforenm.argtypes = [P, P, P]
    lib.or_seal_batch.argtypes = [ctypes.c_void_p, U64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                  ctypes.c_int, ctypes.c_int]
    _ORACLE = lib
    return lib


def or_hsalsa20(in16, key):
    out = ctypes.create_string_buffer(32)
    oracle().or_hsalsa20(out, in16, key)
    return out.raw


def or_salsa20_stream(length, nonce8, ic, key):
    out = ctypes.create_string_buffer(length)
    oracle().or_salsa20_xor_ic(out, None, length, nonce8, ic, key)
    return out.raw


def or_poly1305(msg, key):
    out = ctypes.create_string_buffer(16)
    oracle().or_poly1305(out, msg, len(msg), key)
    return out.raw


def or_box_afternm(m, n24, k):
    c = ctypes.create_string_buffer(len(m))
    rc = oracle().or_secretbox(c, m, len(m), n24, k)
    return rc, c.raw


def or_box_open_afternm(c, n24, k):
    m = ctypes.create_string_buffer(len(c))
    rc = oracle().or_secretbox_open(m, c, len(c), n24, k)
    return rc, m.raw


def or_curve_encode(payload, flags, counter, from_server, k):
    body = ctypes.create_string_buffer(33 + len(payload))
    n = oracle().or_curve_encode(body, payload, len(payload), flags, counter, from_server, k)
    assert n == 33 + len(payload)
    return body.raw


def or_curve_decode(body, from_server, k):
    payload = ctypes.create_string_buffer(max(1, len(body) - 33))
    flags = ctypes.c_uint8()
    nonce = ctypes.c_uint64()
    rc = oracle().or_curve_decode(payload, ctypes.byref(flags), ctypes.byref(nonce), body, len(body), from_server, k)
    if rc != 0:
        return rc, None, None, None
    return 0, payload.raw[: len(body) - 33], flags.value, nonce.value


# descriptor layout shared with include/curvezmq_mi355x.h (cz_frame_desc, 40 bytes)
DESC_DTYPE = np.dtype([("in_off", "<u8"), ("out_off", "<u8"), ("len", "<u4"), ("key_idx", "<u4"),
                       ("counter", "<u8"), ("flags", "<u4"), ("prev", "<i4")])
assert DESC_DTYPE.itemsize == 40


# ---- ZMTP v2 framing restated (test infrastructure) -------------------------------------
def v2_encode(body, msg_flags=0):
    """V2Encoder.messageReady + sizeReady (zmq/io/coder/v2/V2Encoder.java:24-62): flags byte
    (MORE 1, LARGE 2 when size > 255, COMMAND 4), the size as 1 byte or BE64 (Wire.putUInt64),
    then the body.  msg_flags uses Msg's bits (MORE 1, COMMAND 2)."""
    f = (1 if msg_flags & 1 else 0) | (4 if msg_flags & 2 else 0)
    body = bytes(body)
    if len(body) > 255:
        return bytes([f | 2]) + len(body).to_bytes(8, "big") + body
    return bytes([f, len(body)]) + body


class V2DecoderModel:
    """The V2Decoder state machine (V2Decoder.java:37-105) with Decoder.sizeReady's checks
    (zmq/io/coder/Decoder.java:76-98), fed arbitrary chunks like socket reads.
    Decoded messages are (offset of the body in the whole stream, size, Msg flags)."""

    def __init__(self, maxmsgsize=-1):
        self.maxmsgsize = maxmsgsize
        self.state, self.need, self.tmp = "flags", 1, b""
        self.pos = 0                 # bytes of the stream consumed so far
        self.msgs, self.error = [], None
        self.flags = self.size = self.body_off = 0

    def feed(self, data):
        for b in bytes(data):
            if self.error:
                return
            self.tmp += bytes([b])
            self.pos += 1
            if len(self.tmp) < self.need:
                continue
            if self.state == "flags":
                first = self.tmp[0]
                self.flags = (1 if first & 1 else 0) | (2 if first & 4 else 0)
                self.state, self.need = ("size8", 8) if first & 2 else ("size1", 1)
                self.tmp = b""
            elif self.state in ("size1", "size8"):
                size = int.from_bytes(self.tmp, "big")
                if self.state == "size8" and (size == 0 or size >= 1 << 63):   # long `size <= 0`
                    self.error = "EPROTO"
                    return
                if (self.maxmsgsize >= 0 and size > self.maxmsgsize) or size > 0x7fffffff:
                    self.error = "EMSGSIZE"
                    return
                self.size, self.body_off, self.tmp = size, self.pos, b""
                if size == 0:
                    self.msgs.append((self.body_off, 0, self.flags))
                    self.state, self.need = "flags", 1
                else:
                    self.state, self.need = "body", size
            else:
                self.msgs.append((self.body_off, self.size, self.flags))
                self.state, self.need, self.tmp = "flags", 1, b""


def load_x25519_golden():
    with open(os.path.join(os.path.dirname(GOLDEN), "x25519_vectors.json")) as f:
        return json.load(f)


def or_x25519(k, u):
    out = ctypes.create_string_buffer(32)
    oracle().or_x25519(out, bytes(k), bytes(u))
    return out.raw


def or_beforenm(pk, sk):
    out = ctypes.create_string_buffer(32)
    oracle().or_box_beforenm(out, bytes(pk), bytes(sk))
    return out.raw


def or_box(m, n24, pk, sk):
    """NaCl crypto_box = secretbox under beforenm(pk, sk); m without the 32 zero bytes"""
    k = or_beforenm(pk, sk)
    mm = bytes(32) + bytes(m)
    c = ctypes.create_string_buffer(len(mm))
    assert oracle().or_secretbox(c, mm, len(mm), bytes(n24), k) == 0
    return c.raw


def oracle_check_full(d_in, d_out, desc, precom, from_server=0, chunk_bytes=256 << 20, threads=None):
    """Every frame of a device-sealed batch against the oracle (or_seal_batch), byte for byte.

    d_in / d_out: torch uint8 device tensors holding payloads / bodies at desc's offsets (desc: a
    DESC_DTYPE array, frames in increasing offset order).  The batch is checked in chunks of about
    chunk_bytes of output, so a 4 GiB batch needs ~2 x chunk_bytes of host memory.  The oracle
    writes its bodies over a copy of the device's chunk, so only body bytes are compared (slot
    padding belongs to the caller's layout).  Returns the number of frames checked."""
    import os as _os
    if threads is None:
        threads = max(1, min(16, _os.cpu_count() or 1))
    n = len(desc)
    blen = desc["len"].astype(np.uint64) + np.uint64(33)
    pk = np.frombuffer(bytes(precom), dtype=np.uint8).copy()
    a = 0
    while a < n:
        o0 = int(desc["out_off"][a])
        b = int(np.searchsorted(desc["out_off"], np.uint64(o0 + chunk_bytes), side="left"))
        b = max(b, a + 1)
        i0 = int(desc["in_off"][a])
        i1 = int((desc["in_off"][a:b] + desc["len"][a:b].astype(np.uint64)).max())
        o1 = int((desc["out_off"][a:b] + blen[a:b]).max())
        hin = d_in[i0:max(i1, i0 + 1)].cpu().numpy()
        got = d_out[o0:o1].cpu().numpy()
        want = got.copy()
        cd = desc[a:b].copy()
        cd["in_off"] -= np.uint64(i0)
        cd["out_off"] -= np.uint64(o0)
        oracle().or_seal_batch(cd.ctypes.data, b - a, hin.ctypes.data, want.ctypes.data, pk.ctypes.data,
                               from_server, threads)
        if not np.array_equal(got, want):
            for k in range(a, b):
                s0, s1 = int(cd["out_off"][k - a]), int(cd["out_off"][k - a] + blen[k])
                if not np.array_equal(got[s0:s1], want[s0:s1]):
                    raise AssertionError(f"frame {k} (len {int(desc['len'][k])}) differs from the oracle")
        a = b
    return n
