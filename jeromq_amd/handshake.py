"""Mirror of the CURVE Mechanism's handshake half (HELLO / WELCOME / INITIATE / READY / ERROR).

  Mechanism.nextHandshakeCommand / processHandshakeCommand / status / zapMsgAvailable
  CurveClientMechanism.java:80-124, :227-239, :246-429
  CurveServerMechanism.java:77-126, :227-252, :254-517

The state machine is C++ (jeromq_amd/csrc/cz_curve_hs.cpp); every box, open, secretbox, beforenm
and X25519 runs on the GPU.  Commands are ZMTP command bodies (what Msg.buf() holds for a
command frame).  Once status() is READY, mechanism() returns the CONNECTED
CurveClientMechanism / CurveServerMechanism that encodes and decodes MESSAGEs, and an engine
connection comes from engine.add_session(handshake).
"""
import ctypes
import enum

from . import _lib
from .mechanism import CurveClientMechanism, CurveServerMechanism, Msg

# zmq/ZMQ.java:50-70
ZMQ_PAIR, ZMQ_PUB, ZMQ_SUB, ZMQ_REQ, ZMQ_REP, ZMQ_DEALER, ZMQ_ROUTER, ZMQ_PULL, ZMQ_PUSH = range(9)
ZMQ_XPUB, ZMQ_XSUB, ZMQ_STREAM, ZMQ_SERVER, ZMQ_CLIENT, ZMQ_RADIO, ZMQ_DISH = range(9, 16)
ZMQ_CHANNEL, ZMQ_PEER, ZMQ_RAW, ZMQ_SCATTER, ZMQ_GATHER = range(16, 21)

EAGAIN = 35      # zmq.ZError.EAGAIN
EPROTO = 156384712 + 108  # zmq.ZError.EPROTO (ZMQ_HAUSNUMERO + 108)
EINVAL = 22


class Status(enum.Enum):
    """Mechanism.Status (Mechanism.java:28-33)"""
    HANDSHAKING = _lib.CZ_HS_HANDSHAKING
    READY = _lib.CZ_HS_READY
    ERROR = _lib.CZ_HS_ERROR


class _CurveHandshake:
    AS_SERVER = 0
    MAX_COMMAND = 1024

    def __init__(self, public_key, secret_key, server_key, socket_type, identity, ephemeral_secret, entropy):
        h = ctypes.c_void_p()
        ident = bytes(identity or b"")
        ent = bytes(entropy) if entropy is not None else None
        rc = _lib.lib().cz_hs_create(ctypes.byref(h), self.AS_SERVER, public_key, bytes(secret_key), server_key,
                                     socket_type, ident or None, len(ident),
                                     bytes(ephemeral_secret) if ephemeral_secret is not None else None,
                                     ent, len(ent) if ent else 0)
        _lib.check(rc, "cz_hs_create")
        self._h = h
        self.socket_type = socket_type

    def close(self):
        if getattr(self, "_h", None):
            _lib.lib().cz_hs_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def nextHandshakeCommand(self):
        """Returns (rc, Msg): rc 0 with the command to send, EAGAIN when there is none."""
        buf = ctypes.create_string_buffer(self.MAX_COMMAND)
        n = ctypes.c_uint32(0)
        rc = _lib.lib().cz_hs_next_command(self._h, buf, len(buf), ctypes.byref(n))
        if rc == _lib.CZ_EAGAIN:
            return EAGAIN, None
        _lib.check(rc, "nextHandshakeCommand")
        return 0, Msg(buf.raw[:n.value], Msg.COMMAND)

    def processHandshakeCommand(self, msg):
        """0, or EPROTO (event in last_event) / EINVAL (incompatible Socket-Type) as the reference."""
        data = msg.data if isinstance(msg, Msg) else bytes(msg)
        rc = _lib.lib().cz_hs_process_command(self._h, data, len(data))
        if rc == _lib.CZ_OK:
            return 0
        if rc == _lib.CZ_EPROTO:
            return EPROTO
        if rc == _lib.CZ_EINVAL:
            return EINVAL
        raise _lib.CzError(f"processHandshakeCommand ({rc}): {_lib.last_error()}")

    @property
    def last_event(self):
        return _lib.lib().cz_hs_event(self._h) & 0xffffffff

    def status(self):
        return Status(_lib.lib().cz_hs_status(self._h))

    def session(self):
        k = ctypes.create_string_buffer(32)
        n, pn = ctypes.c_uint64(), ctypes.c_uint64()
        _lib.check(_lib.lib().cz_hs_session(self._h, k, ctypes.byref(n), ctypes.byref(pn)), "cz_hs_session")
        return k.raw, n.value, pn.value

    def peer_property(self, name):
        v, n = ctypes.c_void_p(), ctypes.c_uint32()
        if _lib.lib().cz_hs_peer_property(self._h, name.encode(), ctypes.byref(v), ctypes.byref(n)) != _lib.CZ_OK:
            return None
        return ctypes.string_at(v, n.value) if n.value else b""

    def mechanism(self, device=0):
        precom, n, pn = self.session()
        cls = CurveServerMechanism if self.AS_SERVER else CurveClientMechanism
        return cls(precom, cn_nonce=n, cn_peer_nonce=pn, device=device)


class CurveClientHandshake(_CurveHandshake):
    """CurveClientMechanism's handshake: options.curvePublicKey / curveSecretKey / curveServerKey."""
    AS_SERVER = 0

    def __init__(self, public_key, secret_key, server_key, socket_type=ZMQ_PAIR, identity=b"",
                 ephemeral_secret=None, entropy=None):
        super().__init__(bytes(public_key), secret_key, bytes(server_key), socket_type, identity, ephemeral_secret,
                         entropy)


class CurveServerHandshake(_CurveHandshake):
    """CurveServerMechanism's handshake: options.curveSecretKey; zap=True waits for zapReply()."""
    AS_SERVER = 1

    def __init__(self, secret_key, socket_type=ZMQ_PAIR, identity=b"", ephemeral_secret=None, entropy=None,
                 zap=False):
        super().__init__(None, secret_key, None, socket_type, identity, ephemeral_secret, entropy)
        if zap:
            _lib.check(_lib.lib().cz_hs_set_zap(self._h, 1), "cz_hs_set_zap")

    def zapReply(self, status_code):
        rc = _lib.lib().cz_hs_zap_reply(self._h, status_code.encode())
        return 0 if rc == _lib.CZ_OK else EPROTO

    def client_key(self):
        k = ctypes.create_string_buffer(32)
        _lib.check(_lib.lib().cz_hs_client_key(self._h, k), "cz_hs_client_key")
        return k.raw


def metadata(socket_type, identity=b""):
    """The metadata block a socket of this type sends in INITIATE / READY (Mechanism.addProperty)."""
    n = _lib.lib().cz_zmtp_metadata(socket_type, identity or None, len(identity), None, 0)
    buf = ctypes.create_string_buffer(max(n, 1))
    _lib.lib().cz_zmtp_metadata(socket_type, identity or None, len(identity), buf, n)
    return buf.raw[:n]


def check_metadata(buf, socket_type):
    """Metadata.read + parseMetadata's Socket-Type check: 0, EPROTO or EINVAL"""
    rc = _lib.lib().cz_zmtp_metadata_check(bytes(buf), len(buf), socket_type)
    return {_lib.CZ_OK: 0, _lib.CZ_EPROTO: EPROTO, _lib.CZ_EINVAL: EINVAL}[rc]
