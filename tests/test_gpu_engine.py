"""GPU: the ZMTP v2 pack/unpack kernel and the batching engine (cz_engine_*).

The engine's outbound wire stream for each connection must equal, byte for byte,
what JeroMQ would write: V2Encoder framing (restated in cz_testlib.v2_encode) of
each MESSAGE body sealed by the oracle with that connection's nonces.  Inbound,
the engine must deliver exactly the payloads and flags, keep partial frames
across reads, and tear a connection down at its first bad frame with the
reference's event while other connections carry on.
"""
import ctypes
import numpy as np
import pytest

from cz_testlib import load_golden, or_curve_encode, splitmix_bytes, v2_encode

pytestmark = pytest.mark.gpu

G = load_golden()
PRECOM = bytes.fromhex(G["keys"]["precom"])


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch, torch.device("cuda:0")


@pytest.fixture(scope="module")
def L():
    from jeromq_amd import _lib
    return _lib


def _precom(i):
    """distinct per-connection keys; connection 0 uses the golden key"""
    return PRECOM if i == 0 else splitmix_bytes(32, 4242 + i)


@pytest.mark.parametrize("header", [False, True])
def test_v2_copy_any_alignment(torch_dev, header):
    torch, dev = torch_dev
    from jeromq_amd import wire
    rng = np.random.default_rng(3 + header)
    n = 300
    sizes = rng.choice([0, 1, 3, 15, 16, 17, 63, 64, 255, 256, 300, 1000, 4129, 70000], size=n)
    src = rng.integers(0, 256, size=int(sizes.sum()) + 64 * n + 4096, dtype=np.uint8)
    items = np.zeros(n, dtype=wire.V2_ITEM_DTYPE)
    so = rng.integers(0, 7)
    do = int(rng.integers(0, 13))
    want = np.full(int(sizes.sum()) + 16 * n + 4096, 0xEE, dtype=np.uint8)
    for i, s in enumerate(sizes):
        s = int(s)
        so += int(rng.integers(0, 5))
        fl = int(rng.integers(0, 8)) if header else 0
        items[i] = (so, do, s, (0x100 | fl) if header else 0)
        body = src[so:so + s].tobytes()
        out = v2_encode(body, 0) if header else body
        if header:
            f = (fl & ~2) | (2 if s > 255 else 0)
            out = bytes([f]) + out[1:]
        want[do:do + len(out)] = np.frombuffer(out, dtype=np.uint8)
        so += s
        do += len(out)   # contiguous output, like a wire stream
    d_items = torch.from_numpy(items.view(np.uint8).copy()).to(dev)
    d_src = torch.from_numpy(src).to(dev)
    d_dst = torch.full((len(want),), 0xEE, dtype=torch.uint8, device=dev)
    wire.copy(d_items, d_src, d_dst)
    torch.cuda.synchronize()
    assert np.array_equal(d_dst.cpu().numpy(), want)


def _oracle_wire(msgs, precom, from_server, nonce0):
    return b"".join(v2_encode(or_curve_encode(p, fl, nonce0 + k, from_server, precom))
                    for k, (p, fl) in enumerate(msgs))


def _messages(rng, n, seed):
    sizes = rng.choice([0, 1, 31, 100, 222, 223, 4096, 5000, 65536], size=n)
    return [(splitmix_bytes(int(s), seed + k), int(rng.integers(0, 4))) for k, s in enumerate(sizes)]


def test_engine_roundtrip_many_connections(torch_dev, L):
    from jeromq_amd.engine import CurveBatchEngine
    rng = np.random.default_rng(1)
    ncon = 5
    cli = CurveBatchEngine(arena_bytes=8 << 20)
    srv = CurveBatchEngine(arena_bytes=8 << 20)
    cc = [cli.add_connection(_precom(i), as_server=False) for i in range(ncon)]
    sc = [srv.add_connection(_precom(i), as_server=True) for i in range(ncon)]
    sent = {i: _messages(rng, 12 + 3 * i, 100 * i) for i in range(ncon)}
    # interleave sends across connections, as IO threads would
    order = [(i, k) for i in range(ncon) for k in range(len(sent[i]))]
    rng.shuffle(order)
    order.sort(key=lambda t: t[1])   # keep each connection's own order
    for i, k in order:
        p, fl = sent[i][k]
        assert cli.send(cc[i], p, more=bool(fl & 1), command=bool(fl & 2)) == 0
    cli.flush_out()
    wires = {}
    for i in range(ncon):
        w = cli.wire_out(cc[i])
        assert w == _oracle_wire(sent[i], _precom(i), 0, 3), f"connection {i}"
        wires[i] = w
        assert cli.nonce(cc[i]) == 3 + len(sent[i])
    # server side: feed each connection's stream in random pieces, flushing in between
    got = {i: [] for i in range(ncon)}
    pos = {i: 0 for i in range(ncon)}
    while any(pos[i] < len(wires[i]) for i in range(ncon)):
        for i in range(ncon):
            if pos[i] < len(wires[i]):
                step = int(rng.integers(1, 40000))
                srv.recv(sc[i], wires[i][pos[i]:pos[i] + step])
                pos[i] += step
        srv.flush_in()
        for i in range(ncon):
            got[i] += srv.messages_in(sc[i])
    for i in range(ncon):
        assert srv.error(sc[i]) == (0, 0)
        assert [(p, fl) for p, fl in got[i]] == sent[i]
        assert srv.peer_nonce(sc[i]) == 3 + len(sent[i]) - 1


def test_engine_server_to_client_and_msg_alloc(torch_dev, L):
    from jeromq_amd.engine import CurveBatchEngine
    srv = CurveBatchEngine(arena_bytes=1 << 20)
    cli = CurveBatchEngine(arena_bytes=1 << 20)
    s = srv.add_connection(PRECOM, as_server=True)
    c = cli.add_connection(PRECOM, as_server=False)
    msgs = [(bytes([7]) * n, 1 if n % 2 else 0) for n in (5, 300, 4096)]
    for p, fl in msgs:
        buf = srv.msg_alloc(len(p))           # pinned arena buffer: sent without a copy
        buf[:] = p
        assert srv.send(s, buf, more=bool(fl)) == 0
    srv.flush_out()
    w = srv.wire_out(s)
    assert w == _oracle_wire(msgs, PRECOM, 1, 2)
    cli.recv(c, w)
    cli.flush_in()
    assert cli.messages_in(c) == msgs


def test_engine_failures_tear_down_one_connection(torch_dev, L):
    from jeromq_amd.engine import CurveBatchEngine
    rng = np.random.default_rng(5)
    cli = CurveBatchEngine()
    srv = CurveBatchEngine()
    cc = [cli.add_connection(_precom(i)) for i in range(4)]
    sc = [srv.add_connection(_precom(i), as_server=True) for i in range(4)]
    sent = {i: _messages(rng, 6, 900 + i) for i in range(4)}
    for i in range(4):
        for p, fl in sent[i]:
            cli.send(cc[i], p, more=bool(fl & 1), command=bool(fl & 2))
    cli.flush_out()
    w = {i: bytearray(cli.wire_out(cc[i])) for i in range(4)}
    # conn 1: flip a ciphertext byte in frame 3; conn 2: replay frame 1 after frame 2;
    # conn 3: a LARGE header with size 0 after frame 4 (framing error)
    from jeromq_amd import wire as v2
    frames = {i: v2.parse(bytes(w[i]))[0] for i in range(4)}
    f3 = frames[1][3]
    w[1][int(f3["body_off"]) + int(f3["size"]) - 1] ^= 1
    f1, f2 = frames[2][1], frames[2][2]
    hdr1 = v2.header_size(int(f1["size"]))
    frame1 = bytes(w[2][int(f1["body_off"]) - hdr1:int(f1["body_off"]) + int(f1["size"])])
    end2 = int(f2["body_off"]) + int(f2["size"])
    w[2] = w[2][:end2] + frame1 + w[2][end2:]
    f4 = frames[3][4]
    end4 = int(f4["body_off"]) + int(f4["size"])
    w[3] = w[3][:end4] + bytes([2]) + bytes(8) + w[3][end4:]
    for i in range(4):
        srv.recv(sc[i], bytes(w[i]))
    srv.flush_in()
    assert srv.error(sc[0]) == (0, 0) and srv.messages_in(sc[0]) == sent[0]
    assert srv.error(sc[1]) == (L.CZ_EPROTO, L.CZ_ZMTP_CRYPTOGRAPHIC)
    assert srv.messages_in(sc[1]) == sent[1][:3]
    # the bad-tag frame passed the replay check, so cnPeerNonce = its nonce (CurveClientMechanism.java:193),
    # as cz_mech_decode does: client nonces start at 3, frame 3 carries nonce 6
    assert srv.peer_nonce(sc[1]) == 6 and srv.peer_nonce(sc[2]) == 5
    assert srv.error(sc[2]) == (L.CZ_EPROTO, L.CZ_ZMTP_INVALID_SEQUENCE)   # server-side replay event
    assert srv.messages_in(sc[2]) == sent[2][:3]
    assert srv.error(sc[3]) == (L.CZ_EPROTO, 0)                            # V2Decoder EPROTO, no event
    assert srv.messages_in(sc[3]) == sent[3][:5]
    # a torn-down connection refuses further traffic; the others keep working
    assert srv.recv(sc[1], b"\x00\x01x") == L.CZ_EPROTO
    assert srv.send(sc[0], b"still fine") == 0


def test_engine_remove_conn_drops_its_traffic_and_reuses_the_id(torch_dev, L):
    """cz_engine_remove_conn (StreamEngine teardown of an attached connection):
    the removed connection's queued messages leave the flush and its partial input is dropped, the
    other connections' wire streams and deliveries are unchanged, every call on the removed id fails,
    and the next add_conn takes the id back with fresh keys and nonces."""
    from jeromq_amd import _lib
    from jeromq_amd.engine import CurveBatchEngine
    rng = np.random.default_rng(11)
    cli, srv = CurveBatchEngine(arena_bytes=4 << 20), CurveBatchEngine(arena_bytes=4 << 20)
    cc = [cli.add_connection(_precom(i)) for i in range(3)]
    sc = [srv.add_connection(_precom(i), as_server=True) for i in range(3)]
    sent = {i: _messages(rng, 5, 700 + i) for i in range(3)}
    for k in range(5):                       # interleaved across the three connections
        for i in range(3):
            p, fl = sent[i][k]
            assert cli.send(cc[i], p, more=bool(fl & 1), command=bool(fl & 2)) == 0
    cli.remove_connection(cc[1])
    cli.flush_out()
    for i in (0, 2):
        assert cli.wire_out(cc[i]) == _oracle_wire(sent[i], _precom(i), 0, 3), f"connection {i}"
    lib = _lib.lib()
    assert cli.send(cc[1], b"x") == L.CZ_EINVAL
    assert lib.cz_engine_remove_conn(cli._h, cc[1]) == L.CZ_EINVAL     # already removed
    assert lib.cz_engine_remove_conn(cli._h, 99) == L.CZ_EINVAL
    # server: connection 1 has half a frame buffered when it goes; the others deliver everything
    w0, w2 = cli.wire_out(cc[0]), cli.wire_out(cc[2])
    srv.recv(sc[0], w0)
    srv.recv(sc[1], w0[:77])
    srv.recv(sc[2], w2)
    srv.remove_connection(sc[1])
    srv.flush_in()
    assert srv.messages_in(sc[0]) == sent[0] and srv.messages_in(sc[2]) == sent[2]
    assert srv.recv(sc[1], b"\x00") == L.CZ_EINVAL
    # the id comes back with a new key and new nonces; the neighbours' keys are untouched
    key = splitmix_bytes(32, 31337)
    assert cli.add_connection(key, cn_nonce=1000) == cc[1]
    assert srv.add_connection(key, as_server=True, cn_peer_nonce=999) == sc[1]
    more = _messages(rng, 4, 880)
    for p, fl in more:
        assert cli.send(cc[1], p, more=bool(fl & 1)) == 0
    assert cli.send(cc[0], b"after") == 0
    cli.flush_out()
    w = cli.wire_out(cc[1])
    assert w == _oracle_wire([(p, fl & 1) for p, fl in more], key, 0, 1000)
    assert cli.wire_out(cc[0]) == _oracle_wire([(b"after", 0)], _precom(0), 0, 3 + 5)
    srv.recv(sc[1], w)
    srv.flush_in()
    assert srv.messages_in(sc[1]) == [(p, fl & 1) for p, fl in more] and srv.error(sc[1]) == (0, 0)


def test_engine_rejects_oversized_message(torch_dev, L):
    from jeromq_amd import _lib
    from jeromq_amd.engine import CurveBatchEngine
    e = CurveBatchEngine(arena_bytes=4096)
    c = e.add_connection(PRECOM)
    buf = ctypes.create_string_buffer(16)
    assert _lib.lib().cz_engine_send(e._h, c, buf, L.CZ_MESSAGE_MAX + 1, 0) == L.CZ_EMSGSIZE
    assert _lib.lib().cz_engine_send(e._h, c, buf, 0xffffffff, 0) == L.CZ_EMSGSIZE
    assert e.send(c, b"ok") == 0


def test_engine_zero_copy_receive_from_socket(torch_dev, L):
    """cz_engine_recv_buffer / _commit: bytes read from a socket straight into the engine's
    pinned buffer (the V2Decoder getBuffer() pattern), in small reads that split frames."""
    import socket
    from jeromq_amd.engine import CurveBatchEngine
    cli = CurveBatchEngine(arena_bytes=1 << 20)
    srv = CurveBatchEngine(arena_bytes=1 << 20)
    c = cli.add_connection(PRECOM)
    s = srv.add_connection(PRECOM, as_server=True)
    msgs = [(splitmix_bytes(n, 60 + n), n % 2) for n in (0, 17, 255, 256, 3000, 40000)]
    for p, fl in msgs:
        cli.send(c, p, more=bool(fl))
    cli.flush_out()
    w = cli.wire_out(c)
    a, b = socket.socketpair()
    try:
        a.sendall(w)
        a.shutdown(socket.SHUT_WR)
        got = []
        while True:
            n = srv.recv_into(s, lambda mv: b.recv_into(mv, 777), max_bytes=777)
            if n == 0:
                break
            srv.flush_in()
            got += srv.messages_in(s)
    finally:
        a.close()
        b.close()
    assert srv.error(s) == (0, 0) and got == msgs


def test_engine_pipelined_flush_out_and_iov(torch_dev, L):
    """A flush of tens of MiB runs as several pipelined groups (~8 MiB+ each: H2D of one group
    overlapping the seal + D2H of the one before).  Sends interleave across connections and payloads are allocated in the
    arena out of send order, so a group's arena range reaches past its own messages.  Each
    connection's stream, gathered (wire_out) or as writev pieces (wire_iov), equals the
    V2-framed oracle seal of its messages in its own send order."""
    from jeromq_amd.engine import CurveBatchEngine
    rng = np.random.default_rng(11)
    ncon = 6
    cli = CurveBatchEngine(arena_bytes=128 << 20)
    cc = [cli.add_connection(_precom(i)) for i in range(ncon)]
    sizes = {i: [int(s) for s in rng.choice([0, 33, 1000, 4096, 65536, 262144, 1 << 20], size=24, p=[.1, .1, .1, .1, .2, .2, .2])]
             for i in range(ncon)}
    sent = {i: [(splitmix_bytes(s, 900 + 50 * i + k), k & 3) for k, s in enumerate(sizes[i])] for i in range(ncon)}
    # connection 0 queues all its messages together (one piece); the others interleave
    order = [(0, k) for k in range(24)]
    rest = [(i, k) for i in range(1, ncon) for k in range(24)]
    rest.sort(key=lambda t: (t[1], rng.random()))
    order += rest
    # allocate every arena buffer first, in reverse send order for the interleaved part
    bufs = {}
    for i, k in order[:24] + order[24:][::-1]:
        p = sent[i][k][0]
        bufs[(i, k)] = cli.msg_alloc(len(p)) if p else None
        if p:
            bufs[(i, k)][:] = p
    for i, k in order:
        p, fl = sent[i][k]
        payload = bufs[(i, k)] if p else b""
        assert cli.send(cc[i], payload, more=bool(fl & 1), command=bool(fl & 2)) == 0
    cli.flush_out()
    for i in range(ncon):
        want = _oracle_wire(sent[i], _precom(i), 0, 3)
        assert cli.wire_out(cc[i]) == want, f"connection {i}"
        pieces = cli.wire_iov(cc[i])
        assert b"".join(ctypes.string_at(a, n) for a, n in pieces) == want
        if i == 0:
            assert len(pieces) == 1
        else:
            assert len(pieces) > 1
    # a second, small flush on the same engine (one group) still chains the nonces
    cli.send(cc[1], b"after")
    cli.flush_out()
    assert cli.wire_out(cc[1]) == v2_encode(or_curve_encode(b"after", 0, 3 + 24, 0, _precom(1)))
    assert cli.wire_out(cc[2]) == b"" and cli.wire_iov(cc[2]) == []


@pytest.mark.parametrize("seed", range(3))
def test_engine_fuzz_roundtrip(torch_dev, L, seed):
    """Randomized engine traffic: 1..10 connections, edge-biased sizes up to 1 MiB, sends
    interleaved at random, several flush_out calls; every connection's wire stream equals the
    V2-framed oracle seal of its messages, and the server engine, fed the streams in random
    pieces across flush_in calls (tens of MiB, so both flushes run as several pipelined groups),
    delivers exactly what was sent with the reference's nonce bookkeeping."""
    from jeromq_amd.engine import CurveBatchEngine
    rng = np.random.default_rng(500 + seed)
    ncon = int(rng.integers(1, 11))
    cli = CurveBatchEngine(arena_bytes=192 << 20)
    srv = CurveBatchEngine(arena_bytes=1 << 20)
    cc = [cli.add_connection(_precom(i)) for i in range(ncon)]
    sc = [srv.add_connection(_precom(i), as_server=True) for i in range(ncon)]
    edges = [0, 1, 30, 31, 32, 222, 223, 255, 256, 4096, 65536, 300000]
    sent = {i: [] for i in range(ncon)}
    wires = {i: bytearray() for i in range(ncon)}
    nonce = {i: 3 for i in range(ncon)}
    for _flush in range(int(rng.integers(1, 4))):
        queued = {i: [] for i in range(ncon)}
        for _ in range(int(rng.integers(20, 160))):
            i = int(rng.integers(0, ncon))
            r = rng.random()
            n = (int(rng.choice(edges)) if r < 0.45 else int(rng.integers(0, 20000)) if r < 0.85
                 else int(rng.integers(256 << 10, 1 << 20)))
            msg = (splitmix_bytes(n, int(rng.integers(0, 1 << 30))), int(rng.integers(0, 4)))
            assert cli.send(cc[i], msg[0], more=bool(msg[1] & 1), command=bool(msg[1] & 2)) == 0
            queued[i].append(msg)
        cli.flush_out()
        for i in range(ncon):
            w = cli.wire_out(cc[i])
            assert w == _oracle_wire(queued[i], _precom(i), 0, nonce[i]), f"connection {i}"
            assert b"".join(ctypes.string_at(a, n) for a, n in cli.wire_iov(cc[i])) == w
            nonce[i] += len(queued[i])
            sent[i] += queued[i]
            wires[i] += w
    got = {i: [] for i in range(ncon)}
    pos = {i: 0 for i in range(ncon)}
    while any(pos[i] < len(wires[i]) for i in range(ncon)):
        for i in range(ncon):
            if pos[i] < len(wires[i]) and rng.random() < 0.8:
                step = int(rng.integers(1, 3 << 20))
                srv.recv(sc[i], bytes(wires[i][pos[i]:pos[i] + step]))
                pos[i] += step
        srv.flush_in()
        for i in range(ncon):
            got[i] += srv.messages_in(sc[i])
    for i in range(ncon):
        assert srv.error(sc[i]) == (0, 0)
        assert got[i] == sent[i], f"connection {i}"
        if sent[i]:
            assert srv.peer_nonce(sc[i]) == 3 + len(sent[i]) - 1


def test_engine_full_size_flush(torch_dev, L):
    """bench.py's engine line at full size: 1024 connections x 256 x 4 KiB (1 GiB per flush, 16
    pipelined groups, 128-block segments).  32 connections' whole wire streams against the oracle,
    and every one of the 262144 messages delivered intact by the server engine's flush_in."""
    from jeromq_amd.engine import CurveBatchEngine
    nconn, per, n = 1024, 256, 4096
    cli = CurveBatchEngine(arena_bytes=nconn * per * n + (1 << 20))
    srv = CurveBatchEngine(arena_bytes=1 << 20)
    cc = [cli.add_connection(_precom(c)) for c in range(nconn)]
    sc = [srv.add_connection(_precom(c), as_server=True) for c in range(nconn)]
    payload = np.frombuffer(splitmix_bytes(per * n + 64 * nconn, 77), dtype=np.uint8)
    for c in range(nconn):                     # each connection's messages: a window shifted by 64 c
        for k in range(per):
            buf = cli.msg_alloc(n)
            ctypes.memmove(buf, payload[64 * c + k * n:64 * c + (k + 1) * n].ctypes.data, n)
            cli.send(cc[c], buf, more=(k % 8 == 0))
    cli.flush_out()
    for c in list(range(0, nconn, 37)) + [nconn - 1]:
        msgs = [(payload[64 * c + k * n:64 * c + (k + 1) * n].tobytes(), int(k % 8 == 0)) for k in range(per)]
        assert cli.wire_out(cc[c]) == _oracle_wire(msgs, _precom(c), 0, 3), f"connection {c}"
    for c in range(nconn):
        srv.recv(sc[c], cli.wire_out(cc[c]))
    srv.flush_in()
    for c in range(nconn):
        got = srv.messages_in(sc[c])
        assert len(got) == per and srv.error(sc[c]) == (0, 0), c
        for k in range(per):
            assert got[k][0] == payload[64 * c + k * n:64 * c + (k + 1) * n].tobytes(), (c, k)
        assert srv.peer_nonce(sc[c]) == 3 + per - 1
