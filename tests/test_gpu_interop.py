"""GPU: the kernels against a real libzmq 4.3.4 CURVE session (tests/golden/libzmq_session.json).

libzmq accepted the client MESSAGE bodies recorded in c2s and sealed the s2c bodies itself;
the device mechanism and the batching engine must reproduce the former bit for bit and open
the latter -- including parsing libzmq's raw V2 byte stream."""
import json
import os

import pytest

from cz_testlib import splitmix_bytes

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
S = json.load(open(os.path.join(HERE, "golden", "libzmq_session.json")))
PRECOM = bytes.fromhex(S["precom"])


@pytest.fixture(scope="module")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return True


def test_mechanism_matches_libzmq(gpu):
    from jeromq_amd.mechanism import CurveClientMechanism, Msg
    mech = CurveClientMechanism(PRECOM, cn_nonce=3, cn_peer_nonce=S["ready_nonce"])
    for m in S["c2s"]:
        out = mech.encode(Msg(splitmix_bytes(m["n"], m["seed"]), flags=m["flags"]))
        assert bytes(out.data).hex() == m["body"]
    for m in S["s2c"]:
        got = mech.decode(Msg(bytes.fromhex(m["body"])))
        assert got is not None and bytes(got.data) == splitmix_bytes(m["n"], m["seed"])
        assert got.flags == m["flags"]


def test_engine_on_libzmq_wire(gpu):
    from cz_testlib import v2_encode
    from jeromq_amd.engine import CurveBatchEngine
    eng = CurveBatchEngine(arena_bytes=1 << 20)
    c = eng.add_connection(PRECOM, as_server=False, cn_nonce=3, cn_peer_nonce=S["ready_nonce"])
    raw = bytes.fromhex(S["s2c_wire"])
    eng.recv(c, raw[:1000])          # split like TCP reads
    eng.flush_in()
    eng.recv(c, raw[1000:])
    got = eng.messages_in(c)
    eng.flush_in()
    got += eng.messages_in(c)
    assert eng.error(c) == (0, 0)
    assert got == [(splitmix_bytes(m["n"], m["seed"]), m["flags"]) for m in S["s2c"]]
    for m in S["c2s"]:
        eng.send(c, splitmix_bytes(m["n"], m["seed"]), more=bool(m["flags"] & 1))
    eng.flush_out()
    assert eng.wire_out(c) == b"".join(v2_encode(bytes.fromhex(m["body"])) for m in S["c2s"])
