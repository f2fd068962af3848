"""CPU: the host-only parts of the CURVE handshake (jeromq_amd/csrc/cz_curve_hs.cpp): the metadata
block a socket sends (Mechanism.addProperty, Mechanism.java:101-116), Metadata.read's parse rules
(zmq/io/Metadata.java:365-417) with parseMetadata's Socket-Type check (Sockets.compatible,
zmq/socket/Sockets.java:241-244), and that a handshake cannot be created without the GPU."""
import ctypes
import os
import struct

import pytest


@pytest.fixture(scope="module")
def hs():
    from jeromq_amd.build import build_library
    build_library()
    from jeromq_amd import handshake
    return handshake


def prop(name, value):
    return bytes([len(name)]) + name + struct.pack(">I", len(value)) + value


def test_metadata_block(hs):
    assert hs.metadata(hs.ZMQ_PAIR) == prop(b"Socket-Type", b"PAIR")
    assert hs.metadata(hs.ZMQ_PUB) == prop(b"Socket-Type", b"PUB")
    # Identity only for REQ / DEALER / ROUTER (CurveClientMechanism.java:364-366)
    assert hs.metadata(hs.ZMQ_DEALER, b"abc") == prop(b"Socket-Type", b"DEALER") + prop(b"Identity", b"abc")
    assert hs.metadata(hs.ZMQ_REQ) == prop(b"Socket-Type", b"REQ") + prop(b"Identity", b"")
    assert hs.metadata(hs.ZMQ_PUSH, b"abc") == prop(b"Socket-Type", b"PUSH")


COMPAT = {"PAIR": ["PAIR"], "PUB": ["SUB", "XSUB"], "SUB": ["PUB", "XPUB"], "REQ": ["REP", "ROUTER"],
          "REP": ["REQ", "DEALER"], "DEALER": ["REP", "DEALER", "ROUTER"], "ROUTER": ["REQ", "DEALER", "ROUTER"],
          "PULL": ["PUSH"], "PUSH": ["PULL"], "XPUB": ["SUB", "XSUB"], "XSUB": ["PUB", "XPUB"], "STREAM": [],
          "SERVER": ["CLIENT"], "CLIENT": ["SERVER"], "RADIO": ["DISH"], "DISH": ["RADIO"], "CHANNEL": ["CHANNEL"],
          "PEER": ["PEER"], "RAW": [], "SCATTER": ["GATHER"], "GATHER": ["SCATTER"]}
NAMES = list(COMPAT)


def test_socket_type_compatibility(hs):
    for t, name in enumerate(NAMES):
        for peer in NAMES:
            rc = hs.check_metadata(prop(b"Socket-Type", peer.encode()), t)
            assert rc == (0 if peer in COMPAT[name] else hs.EINVAL), (name, peer)


def test_metadata_parse_rules(hs):
    ok = prop(b"Socket-Type", b"PAIR") + prop(b"Identity", b"x" * 300) + prop(b"X-Custom", b"")
    assert hs.check_metadata(ok, hs.ZMQ_PAIR) == 0
    assert hs.check_metadata(b"", hs.ZMQ_PAIR) == 0
    assert hs.check_metadata(b"\x00", hs.ZMQ_PAIR) == hs.EPROTO         # loop never runs, 1 byte left over
    assert hs.check_metadata(ok + b"\x00\x00", hs.ZMQ_PAIR) == hs.EPROTO  # zero name length with 2 bytes left
    assert hs.check_metadata(ok[:-1], hs.ZMQ_PAIR) == hs.EPROTO          # truncated value length
    assert hs.check_metadata(prop(b"A", b"abc")[:-1], hs.ZMQ_PAIR) == hs.EPROTO
    assert hs.check_metadata(b"\x05abc", hs.ZMQ_PAIR) == hs.EPROTO       # name longer than what is left
    neg = bytes([1]) + b"A" + b"\xff\xff\xff\xff"                       # negative value length
    assert hs.check_metadata(neg + b"zz", hs.ZMQ_PAIR) == hs.EPROTO
    assert hs.check_metadata(neg, hs.ZMQ_PAIR) == 0                      # the loop breaks with nothing left over


@pytest.mark.skipif(os.path.exists("/dev/kfd") and os.access("/dev/kfd", os.R_OK), reason="GPU present")
def test_handshake_needs_the_gpu(hs):
    from jeromq_amd import _lib
    h = ctypes.c_void_p()
    rc = _lib.lib().cz_hs_create(ctypes.byref(h), 0, bytes(32), bytes(32), bytes(32), 0, None, 0, None, None, 0)
    assert rc == _lib.CZ_EHIP and not h.value
    with pytest.raises(_lib.CzError):
        hs.CurveServerHandshake(bytes(32))
