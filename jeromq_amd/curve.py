"""Mirror of zmq.io.mechanism.curve.Curve (jeromq-core/src/main/java/zmq/io/mechanism/curve/Curve.java),
backed by the gfx950 kernels through the C-ABI.

Same names, argument meaning and int return contract (0 success / -1 failure) as
Curve.afternm (Curve.java:129-137), Curve.openAfternm (:139-147),
Curve.secretbox (:159-167), Curve.secretboxOpen (:169-177), and the handshake calls
Curve.keypair (:100-115), Curve.beforenm (:124-127), Curve.box (:183-193) and
Curve.open (:149-157).  Each call is one device launch; use jeromq_amd.batch (and
cz_beforenm_batch) for throughput.
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

    # ---- handshake calls (X25519 on the device) ----
    def keypair(self):
        """[public, secret] as 32-byte bytes (Curve.keypair, Curve.java:100-115)."""
        pk, sk = ctypes.create_string_buffer(32), ctypes.create_string_buffer(32)
        rc = _lib.lib().cz_box_keypair(pk, sk)
        assert rc == 0, _lib.last_error()
        return [pk.raw, sk.raw]

    def beforenm(self, outSharedKey, publicKey, secretKey):
        return _lib.lib().cz_box_beforenm(_outbuf(outSharedKey, 32), bytes(publicKey), bytes(secretKey))

    def box(self, ciphertext, plaintext, length, nonce, publicKey, secretKey):
        m = _inbuf(plaintext, length, "plaintext")
        return _lib.lib().cz_box(_outbuf(ciphertext, length), m, length, bytes(nonce), bytes(publicKey),
                                 bytes(secretKey))

    def open(self, plaintext, messagebox, length, nonce, publicKey, secretKey):
        c = _inbuf(messagebox, length, "messagebox")
        return _lib.lib().cz_box_open(_outbuf(plaintext, length), c, length, bytes(nonce), bytes(publicKey),
                                      bytes(secretKey))

    # snake_case aliases
    open_afternm = openAfternm
    secretbox_open = secretboxOpen


def subkey(precom, direction):
    """HSalsa20(precom, "CurveZMQMESSAGE{C|S}") -- the per-connection-direction Salsa20 key."""
    out = ctypes.create_string_buffer(32)
    _lib.check(_lib.lib().cz_subkey(out, bytes(precom), direction), "cz_subkey")
    return out.raw


def scalarmult(n, p):
    """X25519(n, p) (crypto_scalarmult, RFC 7748), computed on the device."""
    out = ctypes.create_string_buffer(32)
    if _lib.lib().cz_scalarmult(out, bytes(n), bytes(p)) != 0:
        raise _lib.CzError("cz_scalarmult failed: " + _lib.last_error())
    return out.raw
