"""ZMTP v2 framing on the host: cz_v2_parse against the V2Decoder restatement
(tests/cz_testlib.py, following V2Decoder.java:37-105) and the reference's own
coder test cases (zmq/io/coder/V2DecoderTest.java, AbstractDecoderTest.java,
V2EncoderTest.java), rebuilt here as byte vectors.  CPU only."""
import numpy as np
import pytest

from cz_testlib import V2DecoderModel, v2_encode

from jeromq_amd import _lib, wire


def test_header_size_matches_encoder():
    for n in (0, 1, 255):
        assert wire.header_size(n) == 2 == len(v2_encode(b"x" * n)) - n
    for n in (256, 70000):
        assert wire.header_size(n) == 9 == len(v2_encode(b"x" * n)) - n


def test_reference_encoder_cases():
    # V2EncoderTest.testReader: "hello" -> 7 bytes; testReaderLong: 200 bytes -> 64 + 138
    assert len(v2_encode(b"hello")) == 7
    assert len(v2_encode(b"0123456789" * 20)) == 202


def test_reference_decoder_cases():
    short = bytes([1, 5]) + b"hello"                       # V2DecoderTest.readShortMessage
    f, used, rc = wire.parse(short)
    assert rc == 0 and used == 7 and len(f) == 1 and f[0]["msg_flags"] == _lib.CZ_MSG_MORE
    long1 = bytes([1, 200]) + b"0123456789" * 6 + b"01"    # readLongMessage1: first 64 bytes
    f, used, rc = wire.parse(long1)
    assert rc == 0 and used == 0 and len(f) == 0          # body incomplete: nothing consumed
    body = (b"0123456789" * 20)[:199] + b"x"               # + "23456789" + readLongMessage2 ('x' last)
    f, used, rc = wire.parse(bytes([1, 200]) + body)
    assert used == 202 and f[0]["size"] == 200 and f[0]["body_off"] == 2
    extra = bytes([2]) + (330).to_bytes(8, "big") + (b"0123456789" * 33)[:329] + b"x"   # readExtraLongMessage
    f, used, rc = wire.parse(extra)
    assert rc == 0 and used == 339 and f[0]["size"] == 330 and f[0]["body_off"] == 9
    # testReaderMultipleMsg: two short messages fed as 7, then 6 + 1 bytes
    two = short + short
    f, used, rc = wire.parse(two[:13])
    assert used == 7 and len(f) == 1
    f, used, rc = wire.parse(two)
    assert used == 14 and len(f) == 2 and f[1]["body_off"] == 9


def _stream(rng, n):
    out, bodies = b"", []
    for _ in range(n):
        size = int(rng.choice([0, 1, 7, 33, 133, 254, 255, 256, 257, 1000, 4129, 70000]))
        fl = int(rng.integers(0, 4))
        body = rng.integers(0, 256, size=size, dtype=np.uint8).tobytes()
        out += v2_encode(body, fl)
        bodies.append((body, fl))
    return out, bodies


def _model(data, maxmsgsize=-1, chunks=None):
    m = V2DecoderModel(maxmsgsize)
    if chunks is None:
        m.feed(data)
    else:
        for c in chunks:
            m.feed(c)
    return m


@pytest.mark.parametrize("seed", range(4))
def test_parse_matches_decoder_model(seed):
    rng = np.random.default_rng(seed)
    data, bodies = _stream(rng, 40)
    f, used, rc = wire.parse(data)
    m = _model(data)
    assert rc == 0 and m.error is None
    assert used == len(data)
    assert [(int(x["body_off"]), int(x["size"]), int(x["msg_flags"])) for x in f] == m.msgs
    for (body, fl), x in zip(bodies, f):
        o = int(x["body_off"])
        assert data[o:o + len(body)] == body and int(x["msg_flags"]) == fl


def test_every_cut_point_consumes_only_whole_frames():
    rng = np.random.default_rng(9)
    data, _ = _stream(rng, 12)
    data = data[:3000]
    for cut in range(len(data) + 1):
        f, used, rc = wire.parse(data[:cut])
        m = _model(data[:cut])
        assert rc == 0
        assert [(int(x["body_off"]), int(x["size"]), int(x["msg_flags"])) for x in f] == m.msgs
        ends = [o + s for o, s, _ in m.msgs]
        assert used == (ends[-1] if ends else 0)


@pytest.mark.parametrize("hdr,want", [
    (bytes([2]) + (0).to_bytes(8, "big"), _lib.CZ_EPROTO),            # V2Decoder: size <= 0
    (bytes([2]) + (1 << 63).to_bytes(8, "big"), _lib.CZ_EPROTO),      # negative as a Java long
    (bytes([2]) + (1 << 31).to_bytes(8, "big"), _lib.CZ_EMSGSIZE),    # > Integer.MAX_VALUE
])
def test_bad_headers_after_good_frames(hdr, want):
    good = v2_encode(b"abc") + v2_encode(b"z" * 300, 1)
    f, used, rc = wire.parse(good + hdr + b"tail")
    assert rc == want and len(f) == 2 and used == len(good)
    m = _model(good + hdr + b"tail")
    assert m.error == ("EPROTO" if want == _lib.CZ_EPROTO else "EMSGSIZE") and len(m.msgs) == 2


def test_maxmsgsize():
    data = v2_encode(b"a" * 100) + v2_encode(b"b" * 600)
    f, used, rc = wire.parse(data, maxmsgsize=512)       # V2DecoderTest builds its decoder with 512
    assert rc == _lib.CZ_EMSGSIZE and len(f) == 1 and used == 102
    assert _model(data, 512).error == "EMSGSIZE"
    f, used, rc = wire.parse(data, maxmsgsize=600)
    assert rc == 0 and len(f) == 2


def test_parse_cap():
    data = b"".join(v2_encode(bytes([i])) for i in range(10))
    f, used, rc = wire.parse(data, cap=4)
    assert len(f) == 4 and used == 12 and rc == 0
