"""Batching CURVE engine over the C-ABI (cz_engine_*): the StreamEngine encode/decode
loops (StreamEngine.java:379-535, :1052-1098) for many connections at once, with one
device batch per flush and socket-ready ZMTP v2 wire streams per connection.

    eng = CurveBatchEngine(arena_bytes=1 << 26)
    c = eng.add_connection(precom, as_server=False)          # CurveClientMechanism state
    eng.send(c, b"payload", more=False)
    eng.flush_out(); wire = eng.wire_out(c)                   # bytes for the socket
    eng.recv(c, received_bytes); eng.flush_in()
    for payload, flags in eng.messages_in(c): ...
    eng.error(c)                                              # (CZ_EPROTO, ZMTP event) after a failure
"""
import ctypes

from . import _lib


class _IOVEC(ctypes.Structure):
    _fields_ = [("base", ctypes.c_void_p), ("len", ctypes.c_uint64)]


class CurveBatchEngine:
    def __init__(self, arena_bytes=1 << 26, device=0):
        self._L = _lib.lib()
        h = ctypes.c_void_p()
        _lib.check(self._L.cz_engine_create(ctypes.byref(h), arena_bytes, device), "cz_engine_create")
        self._h = h

    def close(self):
        if self._h:
            self._L.cz_engine_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def add_session(self, handshake):
        """A connection from a completed CURVE handshake (jeromq_amd.handshake): its cnPrecom and nonces."""
        rc = self._L.cz_engine_add_session(self._h, handshake._h)
        if rc < 0:
            _lib.check(rc, "cz_engine_add_session")
        return rc

    def add_connection(self, precom, as_server=False, cn_nonce=None, cn_peer_nonce=None):
        """Per-connection CURVE state after the handshake: client MESSAGEs start at nonce 3
        and expect the server's from 2 (cn_peer_nonce 1); the server the other way round."""
        if cn_nonce is None:
            cn_nonce = 2 if as_server else 3
        if cn_peer_nonce is None:
            cn_peer_nonce = 2 if as_server else 1
        k = (ctypes.c_uint8 * 32).from_buffer_copy(bytes(precom))
        rc = self._L.cz_engine_add_conn(self._h, 1 if as_server else 0, k, cn_nonce, cn_peer_nonce)
        if rc < 0:
            _lib.check(rc, "cz_engine_add_conn")
        return rc

    def remove_connection(self, conn):
        """The connection is gone (StreamEngine teardown): queued messages and received bytes are
        dropped, its subkeys wiped, and its id reused by a later add_connection."""
        _lib.check(self._L.cz_engine_remove_conn(self._h, conn), "cz_engine_remove_conn")

    def msg_alloc(self, n):
        """Pinned payload buffer in the engine arena (ZMQ_MSG_ALLOCATOR); a ctypes array or None."""
        p = self._L.cz_engine_msg_alloc(self._h, n)
        return None if not p else (ctypes.c_uint8 * n).from_address(p)

    def send(self, conn, payload, more=False, command=False):
        flags = (_lib.CZ_MSG_MORE if more else 0) | (_lib.CZ_MSG_COMMAND if command else 0)
        if isinstance(payload, ctypes.Array):
            ptr, n = ctypes.addressof(payload), ctypes.sizeof(payload)
        else:
            b = bytes(payload)
            buf = ctypes.create_string_buffer(b, len(b)) if b else None
            ptr, n = (ctypes.addressof(buf) if buf else None), len(b)
        return self._L.cz_engine_send(self._h, conn, ptr, n, flags)

    def flush_out(self):
        _lib.check(self._L.cz_engine_flush_out(self._h), "cz_engine_flush_out")

    def wire_out(self, conn):
        p, n = ctypes.c_void_p(), ctypes.c_uint64()
        _lib.check(self._L.cz_engine_wire_out(self._h, conn, ctypes.byref(p), ctypes.byref(n)), "cz_engine_wire_out")
        return ctypes.string_at(p.value, n.value) if n.value else b""

    def wire_iov(self, conn):
        """The connection's stream as gather-write pieces [(address, length)] of the flush output."""
        cnt = ctypes.c_uint32()
        _lib.check(self._L.cz_engine_wire_iov(self._h, conn, None, 0, ctypes.byref(cnt)), "cz_engine_wire_iov")
        arr = (_IOVEC * max(cnt.value, 1))()
        _lib.check(self._L.cz_engine_wire_iov(self._h, conn, arr, cnt.value, ctypes.byref(cnt)), "cz_engine_wire_iov")
        return [(arr[k].base, arr[k].len) for k in range(cnt.value)]

    def recv(self, conn, wire):
        b = bytes(wire)
        buf = ctypes.create_string_buffer(b, len(b)) if b else None
        return self._L.cz_engine_recv(self._h, conn, buf, len(b))

    def recv_into(self, conn, read, max_bytes=1 << 20):
        """Zero-copy receive: `read(memoryview)` fills the engine's pinned buffer (e.g.
        sock.recv_into) and returns the byte count, which is committed."""
        p, n = ctypes.c_void_p(), ctypes.c_uint64()
        _lib.check(self._L.cz_engine_recv_buffer(self._h, conn, max_bytes, ctypes.byref(p), ctypes.byref(n)),
                   "cz_engine_recv_buffer")
        view = memoryview((ctypes.c_uint8 * n.value).from_address(p.value)).cast("B")
        got = read(view)
        _lib.check(self._L.cz_engine_recv_commit(self._h, conn, got), "cz_engine_recv_commit")
        return got

    def flush_in(self):
        _lib.check(self._L.cz_engine_flush_in(self._h), "cz_engine_flush_in")

    def messages_in(self, conn):
        cnt = ctypes.c_uint32()
        _lib.check(self._L.cz_engine_msgs_in(self._h, conn, ctypes.byref(cnt)), "cz_engine_msgs_in")
        out = []
        p, n, fl = ctypes.c_void_p(), ctypes.c_uint32(), ctypes.c_int()
        for i in range(cnt.value):
            _lib.check(self._L.cz_engine_msg_in(self._h, conn, i, ctypes.byref(p), ctypes.byref(n), ctypes.byref(fl)),
                       "cz_engine_msg_in")
            out.append((ctypes.string_at(p.value, n.value) if n.value else b"", fl.value))
        return out

    def error(self, conn):
        ev = ctypes.c_int()
        rc = self._L.cz_engine_conn_error(self._h, conn, ctypes.byref(ev))
        return rc, ev.value

    def nonce(self, conn):
        return int(self._L.cz_engine_nonce(self._h, conn))

    def peer_nonce(self, conn):
        return int(self._L.cz_engine_peer_nonce(self._h, conn))
