"""Mirror of JeroMQ's CURVE Mechanism plugin for MESSAGE traffic (CONNECTED state).

  Mechanism.encode(Msg) / decode(Msg)          Mechanism.java:202-210
  CurveClientMechanism.encode / decode         CurveClientMechanism.java:126-224
  CurveServerMechanism.encode / decode         CurveServerMechanism.java:127-224

The C++ implementation (jeromq_amd/csrc/cz_mechanism.cpp) keeps cnNonce /
cnPeerNonce and runs the crypto on the GPU.  decode returns None on failure and
sets `errno` = EPROTO and `last_event` = the ZMQ_PROTOCOL_ERROR_* code the
reference passes to eventHandshakeFailedProtocol.  encodeBatch / decodeBatch
hand many frames to one device launch (the batching the engine's 8 KiB
OUT_BATCH_SIZE loop cannot, Config.java:31).
"""
import ctypes
import errno as _errno

import numpy as np

from . import _lib


class Msg:
    """Minimal zmq.Msg: payload bytes + MORE / COMMAND flags (Msg.java:96-100)."""
    MORE = 1
    COMMAND = 2

    def __init__(self, data=b"", flags=0):
        self.data = bytes(data)
        self.flags = flags

    def size(self):
        return len(self.data)

    def hasMore(self):
        return bool(self.flags & Msg.MORE)

    def isCommand(self):
        return bool(self.flags & Msg.COMMAND)

    def __repr__(self):
        return f"Msg({len(self.data)} B, flags={self.flags})"


class _CurveMechanism:
    AS_SERVER = 0

    def __init__(self, precom, cn_nonce, cn_peer_nonce, device=0):
        precom = bytes(precom)
        if len(precom) != 32:
            raise ValueError("cnPrecom must be 32 bytes")
        self._h = _lib.lib().cz_mech_create(self.AS_SERVER, precom, cn_nonce, cn_peer_nonce, device)
        if not self._h:
            raise _lib.CzError(f"cz_mech_create: {_lib.last_error()}")
        self.errno = 0
        self.last_event = 0

    def close(self):
        if self._h:
            _lib.lib().cz_mech_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def cnNonce(self):
        return _lib.lib().cz_mech_nonce(self._h)

    @property
    def cnPeerNonce(self):
        return _lib.lib().cz_mech_peer_nonce(self._h)

    def encode(self, msg):
        n = msg.size()
        out = ctypes.create_string_buffer(n + _lib.CZ_MESSAGE_OVERHEAD)
        rc = _lib.lib().cz_mech_encode(self._h, msg.data if n else None, n, msg.flags, out)
        if rc < 0:
            raise _lib.CzError(f"encode: {_lib.last_error()}")
        return Msg(out.raw)

    def decode(self, msg):
        size = msg.size()
        out = ctypes.create_string_buffer(max(1, size))
        flags = ctypes.c_int(0)
        event = ctypes.c_int(0)
        rc = _lib.lib().cz_mech_decode(self._h, msg.data, size, out, ctypes.byref(flags), ctypes.byref(event))
        if rc == _lib.CZ_EPROTO:
            self.errno = _errno.EPROTO
            self.last_event = event.value & 0xffffffff
            return None
        if rc < 0:
            raise _lib.CzError(f"decode: {_lib.last_error()}")
        return Msg(out.raw[:rc], flags.value & (Msg.MORE | Msg.COMMAND))

    def encodeBatch(self, msgs):
        count = len(msgs)
        if count == 0:
            return []
        lens = np.array([m.size() for m in msgs], dtype=np.uint32)
        in_off = np.zeros(count, dtype=np.uint64)
        in_off[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
        out_off = in_off + np.arange(count, dtype=np.uint64) * np.uint64(_lib.CZ_MESSAGE_OVERHEAD)
        flags = np.array([m.flags for m in msgs], dtype=np.uint8)
        hin = b"".join(m.data for m in msgs) or b"\0"
        total_out = int(lens.sum()) + _lib.CZ_MESSAGE_OVERHEAD * count
        hout = ctypes.create_string_buffer(total_out)
        rc = _lib.lib().cz_mech_encode_batch(self._h, count, hin, in_off.ctypes.data, lens.ctypes.data,
                                             flags.ctypes.data, hout, out_off.ctypes.data)
        _lib.check(rc, "encodeBatch")
        raw = hout.raw
        return [Msg(raw[int(o):int(o) + int(n) + _lib.CZ_MESSAGE_OVERHEAD]) for o, n in zip(out_off, lens)]

    def decodeBatch(self, msgs):
        """Decode in order; returns the decoded Msgs up to (not including) the first failure.
        On a failure errno / last_event are set as decode would."""
        count = len(msgs)
        if count == 0:
            return []
        sizes = np.array([m.size() for m in msgs], dtype=np.uint32)
        in_off = np.zeros(count, dtype=np.uint64)
        in_off[1:] = np.cumsum(sizes[:-1], dtype=np.uint64)
        plen = np.maximum(sizes.astype(np.int64) - _lib.CZ_MESSAGE_OVERHEAD, 0).astype(np.uint64)
        out_off = np.zeros(count, dtype=np.uint64)
        out_off[1:] = np.cumsum(plen[:-1], dtype=np.uint64)
        hin = b"".join(m.data for m in msgs) or b"\0"
        hout = ctypes.create_string_buffer(max(1, int(plen.sum())))
        flags = np.zeros(count, dtype=np.uint8)
        failed = ctypes.c_int32(-1)
        event = ctypes.c_int(0)
        rc = _lib.lib().cz_mech_decode_batch(self._h, count, hin, in_off.ctypes.data, sizes.ctypes.data, hout,
                                             out_off.ctypes.data, flags.ctypes.data, ctypes.byref(failed),
                                             ctypes.byref(event))
        _lib.check(rc, "decodeBatch")
        ok = count if failed.value < 0 else failed.value
        if failed.value >= 0:
            self.errno = _errno.EPROTO
            self.last_event = event.value & 0xffffffff
        raw = hout.raw
        return [Msg(raw[int(out_off[i]):int(out_off[i] + plen[i])], int(flags[i])) for i in range(ok)]


class CurveClientMechanism(_CurveMechanism):
    """Client side: seals with "CurveZMQMESSAGEC", opens "CurveZMQMESSAGES".
    A fresh connection's first client MESSAGE uses cnNonce 3 (HELLO=1, INITIATE=2)."""
    AS_SERVER = 0

    def __init__(self, precom, cn_nonce=3, cn_peer_nonce=1, device=0):
        super().__init__(precom, cn_nonce, cn_peer_nonce, device)


class CurveServerMechanism(_CurveMechanism):
    """Server side: seals with "CurveZMQMESSAGES", opens "CurveZMQMESSAGEC".
    A fresh connection's first server MESSAGE uses cnNonce 2 (READY=1)."""
    AS_SERVER = 1

    def __init__(self, precom, cn_nonce=2, cn_peer_nonce=2, device=0):
        super().__init__(precom, cn_nonce, cn_peer_nonce, device)
