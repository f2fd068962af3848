"""Mirror of zmq.io.mechanism.curve.Curve (jeromq-core/src/main/java/zmq/io/mechanism/curve/Curve.java)
for the per-message calls, backed by the gfx950 kernels through the C-ABI.

Same names, argument meaning and int return contract (0 success / -1 failure) as
Curve.afternm (Curve.java:129-137), Curve.openAfternm (:139-147),
Curve.secretbox (:159-167) and Curve.secretboxOpen (:169-177).  Each call is one
device launch; use jeromq_amd.batch for throughput.
"""
import ctypes

from . import _lib

NONCE = 24
ZERO = 32
BOXZERO = 16
KEY = 32
BEFORENM = 32


def _outbuf(buf, length):
    if not isinstance(buf, bytearray) or len(buf) < length:
        raise TypeError("output must be a bytearray of at least `length` bytes (caller-allocated, like Java byte[])")
    return (ctypes.c_char * len(buf)).from_buffer(buf)


def _inbuf(data, length, what):
    data = bytes(data)
    if len(data) < length:
        raise ValueError(f"{what} shorter than length")
    return data


class Curve:
    """Per-message NaCl calls of Curve.java, computed on the GPU."""

    def afternm(self, ciphered, plaintext, length, nonce, precom):
        m = _inbuf(plaintext, length, "plaintext")
        return _lib.lib().cz_box_afternm(_outbuf(ciphered, length), m, length, bytes(nonce), bytes(precom))

    def openAfternm(self, plaintext, cipher, length, nonce, precom):
        c = _inbuf(cipher, length, "cipher")
        return _lib.lib().cz_box_open_afternm(_outbuf(plaintext, length), c, length, bytes(nonce), bytes(precom))

    def secretbox(self, ciphertext, plaintext, length, nonce, key):
        m = _inbuf(plaintext, length, "plaintext")
        return _lib.lib().cz_secretbox(_outbuf(ciphertext, length), m, length, bytes(nonce), bytes(key))

    def secretboxOpen(self, plaintext, box, length, nonce, key):
        c = _inbuf(box, length, "box")
        return _lib.lib().cz_secretbox_open(_outbuf(plaintext, length), c, length, bytes(nonce), bytes(key))

    # snake_case aliases
    open_afternm = openAfternm
    secretbox_open = secretboxOpen


def subkey(precom, direction):
    """HSalsa20(precom, "CurveZMQMESSAGE{C|S}") -- the per-connection-direction Salsa20 key."""
    out = ctypes.create_string_buffer(32)
    _lib.check(_lib.lib().cz_subkey(out, bytes(precom), direction), "cz_subkey")
    return out.raw
