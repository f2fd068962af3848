#!/usr/bin/env python3
"""Interop fixture: a real CurveZMQ session against libzmq 4.3.4.

Run in the build container only (libzmq lives at /opt/conda/lib/libzmq.so.5; it never travels
to the GPU box).  A libzmq PAIR socket with CURVE_SERVER (the reference's published server key,
org/zeromq/ZMQ.java:4603-4624) echoes every message.  The client side is written here over a
raw TCP socket, following the reference's CurveClientMechanism byte for byte:
  greeting (ZMTP 3.0, mechanism "CURVE"), HELLO (produceHello, :246-275), WELCOME
  (processWelcome, :277-307), INITIATE with the vouch (produceInitiate, :309-372), READY
  (processReady, :374-404), then MESSAGE commands (encode/decode, :126-224) in ZMTP v2
  frames (V2Encoder / V2Decoder).
Its crypto is the oracle (oracle/curve_oracle.c), so libzmq -- an independent CurveZMQ
implementation that interoperates with JeroMQ -- is what validates it: libzmq accepting our
HELLO/INITIATE/MESSAGEs and echoing every payload is the pass condition.

The client's ephemeral secret is fixed, so the MESSAGE key cnPrecom = beforenm(S', c') is known
and recorded together with:
  c2s: every MESSAGE body we sent (libzmq accepted them);
  s2c: every MESSAGE body libzmq sealed, the payload and flags it carries, and the raw
       server-to-client wire bytes after READY (V2-framed, as the engine receives them).
A second session puts libzmq on the CLIENT side (ZMQ_CURVE_SERVERKEY) against a server written
here after CurveServerMechanism (processHello :254-299, produceWelcome :301-358, processInitiate
:360-471, produceReady :473-507), again with the oracle's crypto and with every random draw fixed
(short-term secret s', cookie nonce, cookie key, WELCOME nonce).  libzmq completing the handshake
and exchanging MESSAGEs both ways is the pass condition.

Both sessions record their handshake command bodies (HELLO, WELCOME, INITIATE, READY) and the
injected randomness, so the product state machine (cz_hs_*) can be checked byte for byte against
what libzmq sent and accepted (tests/test_gpu_handshake.py).
Writes tests/golden/libzmq_session.json.
"""
import ctypes
import json
import os
import socket
import struct
import sys
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from cz_testlib import (or_beforenm, or_box, or_curve_decode, or_curve_encode, or_x25519,  # noqa: E402
                        oracle, splitmix_bytes, v2_encode)

Z = ctypes.CDLL("/opt/conda/lib/libzmq.so.5")
ZMQ_PAIR, ZMQ_LINGER, ZMQ_RCVMORE, ZMQ_SNDMORE = 0, 17, 13, 2
ZMQ_CURVE_SERVER, ZMQ_CURVE_SECRETKEY, ZMQ_RCVTIMEO = 47, 49, 27
ZMQ_CURVE_PUBLICKEY, ZMQ_CURVE_SERVERKEY, ZMQ_SNDTIMEO = 48, 50, 28
Z.zmq_ctx_new.restype = ctypes.c_void_p
Z.zmq_socket.restype = ctypes.c_void_p
Z.zmq_socket.argtypes = [ctypes.c_void_p, ctypes.c_int]
for f in ("zmq_setsockopt", "zmq_getsockopt"):
    getattr(Z, f).argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
Z.zmq_bind.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
Z.zmq_connect.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
Z.zmq_recv.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
Z.zmq_send.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
Z.zmq_close.argtypes = [ctypes.c_void_p]
Z.zmq_ctx_term.argtypes = [ctypes.c_void_p]

CLIENT_PUB = bytes.fromhex("BB88471D65E2659B30C55A5321CEBB5AAB2B70A398645C26DCA2B2FCB43FC518")
CLIENT_SEC = bytes.fromhex("7BB864B489AFA3671FBE69101F94B38972F24816DFB01B51656B3FEC8DFD0888")
SERVER_PUB = bytes.fromhex("54FCBA24E93249969316FB617C872BB0C1D1FF14800427C594CBFACF1BC2D652")
SERVER_SEC = bytes.fromhex("8E0BDD697628B91D8F245587EE95C5B04D48963F79259877B49CD9063AEAD3B7")
EPH_SEC = bytes(range(0x40, 0x60))             # client ephemeral secret c' (fixed for the fixture)
SRV_EPH_SEC = bytes(range(0xa0, 0xc0))         # server ephemeral secret s' (second session)
# the server's Curve.random() draws, in order: cookie nonce (16), cookie key (32), WELCOME nonce (16)
SRV_ENTROPY = bytes((7 * i + 3) & 0xff for i in range(64))
NINE = (9).to_bytes(32, "little")

# (payload size, Msg flags): exercises 1-byte and LARGE V2 headers and the MORE flag in MESSAGE
PAYLOADS = [(0, 0), (1, 0), (100, 1), (100, 0), (222, 0), (223, 0), (4096, 0), (20000, 1), (7, 0)]


def box_open(c, n24, pk, sk):
    k = or_beforenm(pk, sk)
    m = ctypes.create_string_buffer(len(c))
    if oracle().or_secretbox_open(m, bytes(c), len(c), n24, k) != 0:
        raise RuntimeError("box open failed")
    return m.raw


def command(body):
    """ZMTP command frame (V2Encoder with the COMMAND flag, V2Protocol.COMMAND_FLAG = 4)"""
    return v2_encode(body, 2)


class Peer:
    def __init__(self, sock):
        self.s = sock
        self.rx = b""
        self.log = None   # bytearray while recording the raw wire

    def exact(self, n):
        while len(self.rx) < n:
            d = self.s.recv(1 << 16)
            if not d:
                raise RuntimeError("connection closed by libzmq")
            self.rx += d
        out, self.rx = self.rx[:n], self.rx[n:]
        if self.log is not None:
            self.log += out
        return out

    def frame(self):
        f = self.exact(1)[0]
        size = int.from_bytes(self.exact(8), "big") if f & 2 else self.exact(1)[0]
        return f, self.exact(size)


def server(port_box, done, echoed):
    ctx = Z.zmq_ctx_new()
    s = Z.zmq_socket(ctx, ZMQ_PAIR)
    one, zero, tmo = ctypes.c_int(1), ctypes.c_int(0), ctypes.c_int(10000)
    Z.zmq_setsockopt(s, ZMQ_CURVE_SERVER, ctypes.byref(one), 4)
    Z.zmq_setsockopt(s, ZMQ_CURVE_SECRETKEY, SERVER_SEC, 32)
    Z.zmq_setsockopt(s, ZMQ_LINGER, ctypes.byref(zero), 4)
    Z.zmq_setsockopt(s, ZMQ_RCVTIMEO, ctypes.byref(tmo), 4)
    assert Z.zmq_bind(s, b"tcp://127.0.0.1:*") == 0
    ep = ctypes.create_string_buffer(256)
    sz = ctypes.c_size_t(256)
    Z.zmq_getsockopt(s, 32, ep, ctypes.byref(sz))          # ZMQ_LAST_ENDPOINT
    port_box.append(int(ep.value.decode().rsplit(":", 1)[1]))
    buf = ctypes.create_string_buffer(1 << 20)
    for _ in PAYLOADS:
        n = Z.zmq_recv(s, buf, len(buf), 0)
        if n < 0:
            break
        more = ctypes.c_int(0)
        msz = ctypes.c_size_t(4)
        Z.zmq_getsockopt(s, ZMQ_RCVMORE, ctypes.byref(more), ctypes.byref(msz))
        echoed.append((buf.raw[:n], more.value))
        Z.zmq_send(s, buf, n, ZMQ_SNDMORE if more.value else 0)
    done.wait(10)
    Z.zmq_close(s)
    Z.zmq_ctx_term(ctx)


def client_thread(port, results, done):
    """libzmq as the CURVE client: sends PAYLOADS, then receives as many replies"""
    ctx = Z.zmq_ctx_new()
    s = Z.zmq_socket(ctx, ZMQ_PAIR)
    zero, tmo = ctypes.c_int(0), ctypes.c_int(10000)
    Z.zmq_setsockopt(s, ZMQ_CURVE_SERVERKEY, SERVER_PUB, 32)
    Z.zmq_setsockopt(s, ZMQ_CURVE_PUBLICKEY, CLIENT_PUB, 32)
    Z.zmq_setsockopt(s, ZMQ_CURVE_SECRETKEY, CLIENT_SEC, 32)
    Z.zmq_setsockopt(s, ZMQ_LINGER, ctypes.byref(zero), 4)
    Z.zmq_setsockopt(s, ZMQ_RCVTIMEO, ctypes.byref(tmo), 4)
    Z.zmq_setsockopt(s, ZMQ_SNDTIMEO, ctypes.byref(tmo), 4)
    assert Z.zmq_connect(s, ("tcp://127.0.0.1:%d" % port).encode()) == 0
    for i, (n, fl) in enumerate(PAYLOADS):
        payload = splitmix_bytes(n, 7000 + i)
        Z.zmq_send(s, payload, n, ZMQ_SNDMORE if fl else 0)
    buf = ctypes.create_string_buffer(1 << 20)
    for _ in PAYLOADS:
        n = Z.zmq_recv(s, buf, len(buf), 0)
        if n < 0:
            break
        more = ctypes.c_int(0)
        msz = ctypes.c_size_t(4)
        Z.zmq_getsockopt(s, ZMQ_RCVMORE, ctypes.byref(more), ctypes.byref(msz))
        results.append((buf.raw[:n], more.value))
    done.wait(10)
    Z.zmq_close(s)
    Z.zmq_ctx_term(ctx)


def server_session():
    """libzmq client -> our CurveServerMechanism restatement (oracle crypto, fixed randomness)"""
    ls = socket.socket()
    ls.bind(("127.0.0.1", 0))
    ls.listen(1)
    results, done = [], threading.Event()
    th = threading.Thread(target=client_thread, args=(ls.getsockname()[1], results, done), daemon=True)
    th.start()
    ls.settimeout(10)
    sock, _ = ls.accept()
    sock.settimeout(10)
    p = Peer(sock)
    greet = b"\xff" + bytes(8) + b"\x7f" + bytes([3, 0]) + b"CURVE".ljust(20, b"\0") + b"\1" + bytes(31)
    sock.sendall(greet)
    peer_greet = p.exact(64)
    assert peer_greet[0] == 0xff and peer_greet[12:17] == b"CURVE"
    # processHello
    f, hello = p.frame()
    assert f & 4 and hello[:6] == b"\x05HELLO" and len(hello) == 200
    cli_eph = hello[80:112]
    box_open(bytes(16) + hello[120:200], b"CurveZMQHELLO---" + hello[112:120], cli_eph, SERVER_SEC)
    # produceWelcome: cookie = secretbox[C' + s'](t), WELCOME = Box[S' + cookie nonce + cookie](S->C')
    srv_eph = or_x25519(SRV_EPH_SEC, NINE)
    cookie_nonce, cookie_key, welcome_nonce = SRV_ENTROPY[:16], SRV_ENTROPY[16:48], SRV_ENTROPY[48:64]
    km = bytes(32) + cli_eph + SRV_EPH_SEC
    kc = ctypes.create_string_buffer(len(km))
    assert oracle().or_secretbox(kc, km, len(km), b"COOKIE--" + cookie_nonce, cookie_key) == 0
    wbox = or_box(srv_eph + cookie_nonce + kc.raw[16:96], b"WELCOME-" + welcome_nonce, cli_eph, SERVER_SEC)
    welcome = b"\x07WELCOME" + welcome_nonce + wbox[16:160]
    assert len(welcome) == 168
    sock.sendall(command(welcome))
    # processInitiate
    f, initiate = p.frame()
    assert f & 4 and initiate[:9] == b"\x08INITIATE" and len(initiate) >= 257
    assert initiate[9:25] == cookie_nonce
    ip = box_open(bytes(16) + initiate[113:], b"CurveZMQINITIATE" + initiate[105:113], cli_eph, SRV_EPH_SEC)
    client_key = ip[32:64]
    assert client_key == CLIENT_PUB
    vp = box_open(bytes(16) + ip[80:160], b"VOUCH---" + ip[64:80], client_key, SRV_EPH_SEC)
    assert vp[32:64] == cli_eph
    assert b"Socket-Type" in ip[160:]
    peer_nonce = int.from_bytes(initiate[105:113], "big")
    precom = or_beforenm(cli_eph, SRV_EPH_SEC)
    # produceReady: Box[metadata](S'->C') under cnPrecom, nonce "CurveZMQREADY---" + BE64(1)
    meta = bytes([11]) + b"Socket-Type" + struct.pack(">I", 4) + b"PAIR"
    rbox = ctypes.create_string_buffer(32 + len(meta))
    assert oracle().or_secretbox(rbox, bytes(32) + meta, 32 + len(meta), b"CurveZMQREADY---" + struct.pack(">Q", 1),
                                 precom) == 0
    ready = b"\x05READY" + struct.pack(">Q", 1) + rbox.raw[16:]
    sock.sendall(command(ready))
    # MESSAGEs: libzmq's (client nonces 3..), then ours (server nonces 2..)
    c2s = []
    for i, (n, fl) in enumerate(PAYLOADS):
        f, body = p.frame()
        st, pl, flags, n_ = or_curve_decode(body, 0, precom)
        assert st == 0 and n_ > peer_nonce, f"libzmq client MESSAGE {i}: status {st}"
        peer_nonce = n_
        assert pl == splitmix_bytes(n, 7000 + i) and flags == fl
        c2s.append({"body": body.hex(), "nonce": n_, "flags": flags, "n": n, "seed": 7000 + i})
    s2c = []
    nonce = 2
    for i, (n, fl) in enumerate(PAYLOADS):
        payload = splitmix_bytes(n, 8000 + i)
        body = or_curve_encode(payload, fl, nonce, 1, precom)
        sock.sendall(v2_encode(body))
        s2c.append({"body": body.hex(), "nonce": nonce, "flags": fl, "n": n, "seed": 8000 + i})
        nonce += 1
    done.set()
    th.join(15)
    assert [r[0] for r in results] == [splitmix_bytes(n, 8000 + i) for i, (n, _) in enumerate(PAYLOADS)], \
        "libzmq client did not receive our MESSAGEs"
    assert [r[1] for r in results] == [fl for _, fl in PAYLOADS]
    sock.close()
    ls.close()
    return {"server_ephemeral_secret": SRV_EPH_SEC.hex(), "entropy": SRV_ENTROPY.hex(),
            "client_ephemeral_public": cli_eph.hex(), "hello": hello.hex(), "welcome": welcome.hex(),
            "initiate": initiate.hex(), "ready": ready.hex(), "precom": precom.hex(), "socket_type": 0,
            "c2s": c2s, "s2c": s2c}


def main():
    assert Z.zmq_has(b"curve") == 1
    port_box, echoed, done = [], [], threading.Event()
    th = threading.Thread(target=server, args=(port_box, done, echoed), daemon=True)
    th.start()
    while not port_box:
        pass
    sock = socket.create_connection(("127.0.0.1", port_box[0]), timeout=10)
    p = Peer(sock)
    # ZMTP 3.0 greeting: signature, version 3.0, mechanism "CURVE", as-server 0, filler
    greet = b"\xff" + bytes(8) + b"\x7f" + bytes([3, 0]) + b"CURVE".ljust(20, b"\0") + b"\0" + bytes(31)
    sock.sendall(greet)
    peer_greet = p.exact(64)
    assert peer_greet[0] == 0xff and peer_greet[9] == 0x7f and peer_greet[12:17] == b"CURVE"
    eph_pub = or_x25519(EPH_SEC, NINE)
    # HELLO (produceHello): Box[64 zero](C'->S), nonce "CurveZMQHELLO---" + BE64(1)
    short = struct.pack(">Q", 1)
    hello_box = or_box(bytes(64), b"CurveZMQHELLO---" + short, SERVER_PUB, EPH_SEC)[16:]
    hello = b"\x05HELLO" + bytes([1, 0]) + bytes(72) + eph_pub + short + hello_box
    assert len(hello) == 200
    sock.sendall(command(hello))
    # WELCOME (processWelcome): Box[S' + cookie](S->C'), nonce "WELCOME-" + 16-byte long nonce
    f, welcome = p.frame()
    assert f & 4 and welcome[:8] == b"\x07WELCOME" and len(welcome) == 168
    wp = box_open(bytes(16) + welcome[24:168], b"WELCOME-" + welcome[8:24], SERVER_PUB, EPH_SEC)
    srv_eph, cookie = wp[32:64], wp[64:160]
    precom = or_beforenm(srv_eph, EPH_SEC)
    # INITIATE (produceInitiate): vouch = Box[C' + S](C->S'), nonce "VOUCH---" + 16 bytes
    vouch_nonce = bytes(range(16))          # the client's one Curve.random(16) draw
    vouch = or_box(eph_pub + SERVER_PUB, b"VOUCH---" + vouch_nonce, srv_eph, CLIENT_SEC)[16:]
    meta = bytes([11]) + b"Socket-Type" + struct.pack(">I", 4) + b"PAIR"
    short = struct.pack(">Q", 2)
    init_box = or_box(CLIENT_PUB + vouch_nonce + vouch + meta, b"CurveZMQINITIATE" + short, srv_eph, EPH_SEC)[16:]
    initiate = b"\x08INITIATE" + cookie + short + init_box
    sock.sendall(command(initiate))
    # READY (processReady): Box[metadata](S'->C'), nonce "CurveZMQREADY---" + BE64
    f, ready = p.frame()
    assert f & 4 and ready[:6] == b"\x05READY", ready[:16]
    ready_nonce = ready[6:14]
    rp = box_open(bytes(16) + ready[14:], b"CurveZMQREADY---" + ready_nonce, srv_eph, EPH_SEC)
    assert b"Socket-Type" in rp and b"PAIR" in rp
    peer_nonce = int.from_bytes(ready_nonce, "big")
    # MESSAGEs: client nonces 3.. (cnNonce after HELLO=1, INITIATE=2)
    c2s, s2c = [], []
    nonce = 3
    p.log = bytearray()
    sent = []
    for i, (n, fl) in enumerate(PAYLOADS):
        payload = splitmix_bytes(n, 5000 + i)
        body = or_curve_encode(payload, fl, nonce, 0, precom)
        c2s.append({"n": n, "seed": 5000 + i, "flags": fl, "nonce": nonce, "body": body.hex()})
        sock.sendall(v2_encode(body))       # MESSAGE frames go without the COMMAND flag (encode: new Msg)
        sent.append((payload, fl))
        nonce += 1
    for i, (payload, fl) in enumerate(sent):
        f, body = p.frame()
        st, pl, flags, n_ = or_curve_decode(body, 1, precom)
        assert st == 0, f"libzmq MESSAGE {i} failed to open: status {st}"
        assert n_ > peer_nonce
        peer_nonce = n_
        assert pl == payload and flags == fl, f"echo {i} differs"
        s2c.append({"body": body.hex(), "nonce": n_, "flags": flags, "n": len(pl), "seed": 5000 + i})
    raw_s2c = bytes(p.log)
    done.set()
    th.join(10)
    assert [e[0] for e in echoed] == [s[0] for s in sent]
    client_hs = {"hello": hello.hex(), "welcome": welcome.hex(), "initiate": initiate.hex(), "ready": ready.hex(),
                 "vouch_nonce": vouch_nonce.hex(), "socket_type": 0}
    server_sess = server_session()
    out = {"generator": "libzmq 4.3.4 (/opt/conda/lib/libzmq.so.5) via tests/golden/make_libzmq_session.py",
           "client_ephemeral_secret": EPH_SEC.hex(), "client_ephemeral_public": eph_pub.hex(),
           "server_ephemeral_public": srv_eph.hex(), "precom": precom.hex(),
           "ready_nonce": int.from_bytes(ready_nonce, "big"), "c2s": c2s, "s2c": s2c,
           "s2c_wire": bytes(raw_s2c).hex(), "client_handshake": client_hs, "server_session": server_sess}
    with open(os.path.join(HERE, "libzmq_session.json"), "w") as f:
        json.dump(out, f, indent=0, sort_keys=True)
    print("handshake ok with libzmq %s; %d messages each way, s2c wire %d bytes" %
          ("4.3.4", len(c2s), len(raw_s2c)))


if __name__ == "__main__":
    main()
