"""Interop with libzmq 4.3.4, CPU side.

tests/golden/libzmq_session.json was captured by tests/golden/make_libzmq_session.py: a full
CurveZMQ handshake and 9 MESSAGEs each way against a libzmq CURVE server.  Here the oracle and the
host V2 parser are checked against what libzmq produced and accepted; the GPU kernels are checked
against the same capture in test_gpu_interop.py.  The live re-run needs libzmq (container only)."""
import json
import os

import pytest

from cz_testlib import or_curve_decode, or_curve_encode, splitmix_bytes

from jeromq_amd import wire

HERE = os.path.dirname(os.path.abspath(__file__))
S = json.load(open(os.path.join(HERE, "golden", "libzmq_session.json")))
PRECOM = bytes.fromhex(S["precom"])


def test_oracle_seals_what_libzmq_accepted():
    for m in S["c2s"]:
        body = or_curve_encode(splitmix_bytes(m["n"], m["seed"]), m["flags"], m["nonce"], 0, PRECOM)
        assert body.hex() == m["body"]


def test_oracle_opens_libzmq_messages():
    for m in S["s2c"]:
        st, pl, fl, nonce = or_curve_decode(bytes.fromhex(m["body"]), 1, PRECOM)
        assert st == 0 and pl == splitmix_bytes(m["n"], m["seed"]) and fl == m["flags"] and nonce == m["nonce"]


def test_v2_parse_of_libzmq_stream():
    raw = bytes.fromhex(S["s2c_wire"])
    frames, used, rc = wire.parse(raw)
    assert rc == 0 and used == len(raw) and len(frames) == len(S["s2c"])
    for f, m in zip(frames, S["s2c"]):
        o = int(f["body_off"])
        assert raw[o:o + int(f["size"])].hex() == m["body"]
        assert int(f["msg_flags"]) == 0          # MESSAGE frames carry no wire flags


@pytest.mark.skipif(not os.path.exists("/opt/conda/lib/libzmq.so.5"), reason="libzmq not in this image")
def test_live_libzmq_session(tmp_path):
    """Re-run the handshake + echo against libzmq and compare with the committed capture."""
    import subprocess
    import sys
    gen = os.path.join(HERE, "golden", "make_libzmq_session.py")
    before = open(os.path.join(HERE, "golden", "libzmq_session.json")).read()
    try:
        r = subprocess.run([sys.executable, gen], capture_output=True, text=True, timeout=60)
        assert r.returncode == 0, r.stderr[-2000:]
        after = json.load(open(os.path.join(HERE, "golden", "libzmq_session.json")))
        # c2s bodies are deterministic (fixed client ephemeral key, but the server's S' is fresh):
        # compare the parts that do not depend on libzmq's random ephemeral key
        assert [m["n"] for m in after["c2s"]] == [m["n"] for m in S["c2s"]]
        assert len(after["s2c"]) == len(S["s2c"])
    finally:
        with open(os.path.join(HERE, "golden", "libzmq_session.json"), "w") as f:
            f.write(before)
