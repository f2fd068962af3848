"""The last hop of the Java integration: jni/patches/jeromq-gpu-curve.patch wires
GpuCurveIoHook into the reference's StreamEngine and Poller.

No JDK exists in this image, so the patch is checked as text against the reference sources (read,
never built or run): it applies cleanly with `patch -p1` (dry run, then for real) to a temporary copy
of StreamEngine.java and Poller.java; every GpuCurveIoHook member the patched code calls exists in
jni/java/zmq/io/GpuCurveIoHook.java with that many parameters; every Sink method is implemented; the
reference members the patched code relies on exist; braces balance.  The reference file:line anchors:
StreamEngine.java:379-535 (inEvent / outEvent), :958-1005 (mechanismReady), :1052-1111 (pullAndEncode,
decodeAndPush), :1170-1207 (heartbeats); Poller.java:194-284 (the loop)."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PATCH = os.path.join(ROOT, "jni", "patches", "jeromq-gpu-curve.patch")
HOOK = os.path.join(ROOT, "jni", "java", "zmq", "io", "GpuCurveIoHook.java")
REF = "/root/reference"
FILES = ["jeromq-core/src/main/java/zmq/io/StreamEngine.java", "jeromq-core/src/main/java/zmq/poll/Poller.java"]

pytestmark = pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "jeromq-core")),
                                reason="reference sources not present (build container only)")


def _strip(code):
    """Java without comments and string / char literals (for brace and call counting)."""
    code = re.sub(r"/\*.*?\*/", "", code, flags=re.S)
    code = re.sub(r"//[^\n]*", "", code)
    return re.sub(r"\"(?:\\.|[^\"\\])*\"|'(?:\\.|[^'\\])'", "\"\"", code)


@pytest.fixture(scope="module")
def patched(tmp_path_factory):
    d = tmp_path_factory.mktemp("ref")
    for f in FILES:
        os.makedirs(os.path.join(d, os.path.dirname(f)), exist_ok=True)
        shutil.copy(os.path.join(REF, f), os.path.join(d, f))
    with open(PATCH) as p:
        dry = subprocess.run(["patch", "-p1", "--dry-run"], stdin=p, cwd=d, capture_output=True, text=True)
    assert dry.returncode == 0, dry.stdout + dry.stderr
    with open(PATCH) as p:
        real = subprocess.run(["patch", "-p1", "--no-backup-if-mismatch"], stdin=p, cwd=d, capture_output=True,
                              text=True)
    assert real.returncode == 0 and "fuzz" not in real.stdout.lower() and "offset" not in real.stdout.lower(), \
        real.stdout
    return {os.path.basename(f): open(os.path.join(d, f)).read() for f in FILES}


def _args(code, start):
    """top-level argument count of the call whose '(' ends at code[start - 1]"""
    depth, i, n = 1, start, 0
    while depth:
        ch = code[i]
        depth += ch in "([{"
        depth -= ch in ")]}"
        n += ch == "," and depth == 1
        i += 1
    return n + (1 if code[start:i - 1].strip() else 0)


def _hook_api():
    src = _strip(open(HOOK).read())
    api = {}
    for m in re.finditer(r"public (?:static )?[\w<>\[\]]+ (\w+)\(([^)]*)\)", src):
        api[m.group(1)] = len([a for a in m.group(2).split(",") if a.strip()])
    sink = re.search(r"interface Sink\s*\{(.*?)\n    \}", src, re.S).group(1)
    sink_methods = dict((m.group(1), len([a for a in m.group(2).split(",") if a.strip()]))
                        for m in re.finditer(r"\b[\w<>\[\]]+ (\w+)\(([^)]*)\);", sink))
    return api, sink_methods


def test_patch_applies_cleanly_to_the_reference(patched):
    for name, text in patched.items():
        code = _strip(text)
        assert code.count("{") == code.count("}") and code.count("(") == code.count(")"), name


def test_patched_code_calls_only_hook_members_that_exist(patched):
    api, sink = _hook_api()
    calls = 0
    for name, text in patched.items():
        code = _strip(text)
        for m in re.finditer(r"\b(gpuHook|gpuCurve)\.(\w+)\(", code):
            meth = m.group(2)
            assert meth in api, (name, meth)
            assert _args(code, m.end()) == api[meth], (name, meth)
            calls += 1
        for m in re.finditer(r"\bGpuCurveIoHook\.([a-z]\w*)\(", code):   # static calls (not Sink)
            assert m.group(1) in api and _args(code, m.end()) == api[m.group(1)], (name, m.group(1))
            calls += 1
    se = _strip(patched["StreamEngine.java"])
    po = _strip(patched["Poller.java"])
    # the wiring the hook's header describes: attach at READY, hand over the decoder's leftover bytes,
    # delegate both events, resume after back-pressure, detach on teardown; one endOfLoop per iteration
    for must in ("gpuHook.attach(mechanism, gpuSink, fd)", "gpuHook.detach(gpuConn)", "gpuHook.outEvent(gpuConn)",
                 "gpuHook.inEvent(gpuConn, fd)", "gpuHook.handOver(gpuConn, inpos, insize)", "gpuHook.resume(gpuConn)",
                 "gpuHook.writeBacklog(gpuConn)", "ioThread.getPoller().gpuCurveHook()"):
        assert must in se, must
    for must in ("GpuCurveIoHook.fromSystemProperties()", "gpuCurve.endOfLoop()", "gpuCurve.close()"):
        assert must in po, must
    assert po.count("flushGpuCurve();") == 2       # after the handlers, and on a select timeout
    assert calls >= 11
    # every Sink method is implemented by the patched StreamEngine, with its parameter count
    body = se[se.index("new GpuCurveIoHook.Sink()"):]
    for meth, n in sink.items():
        m = re.search(r"public [\w<>\[\]]+ " + meth + r"\(([^)]*)\)", body)
        assert m, meth
        assert len([a for a in m.group(1).split(",") if a.strip()]) == n, meth


def test_attached_connections_never_reach_the_cpu_mechanism(patched):
    """After attach the mechanism's nonce counters belong to the engine: no encode / decode may run on
    the CPU -- pullAndEncode is swapped for the plain session pull, heartbeats are left plaintext for
    the hook, the first inbound message skips mechanism.decode, and back-pressure never returns to
    decodeAndPush."""
    se = _strip(patched["StreamEngine.java"])
    ready = se[se.index("private void mechanismReady()"):se.index("new GpuCurveIoHook.Sink()")]
    assert "nextMsg = pullMsgFromSession;" in ready.split("gpuHook.attach(")[1]
    for fn in ("private Msg producePingMessage()", "private Msg producePongMessage("):
        body = se[se.index(fn):]
        body = body[:body.index("return msg;")]
        assert "if (gpuConn < 0) {\n            msg = mechanism.encode(msg);" in body, fn
        assert "nextMsg = gpuConn >= 0 ? pullMsgFromSession : pullAndEncode;" in body, fn
    assert "processMsg = gpuConn >= 0 ? pushDecoded : decodeAndPush;" in se
    assert "if (errno.is(ZError.EAGAIN) && gpuConn < 0) {\n                processMsg = pushOneThenDecodeAndPush;" in se
    hs = se[se.index("private Msg nextHandshakeCommand()"):]
    hs = hs[:hs.index("return pullAndEncode.get();")]
    assert "gpuHook.outEvent(gpuConn);\n                return null;" in hs


def test_reference_members_the_patch_relies_on_exist():
    """read as text: the reference is never built or run here"""
    base = os.path.join(REF, "jeromq-core/src/main/java/zmq")
    need = {
        "io/IOThread.java": ["Poller getPoller()"],
        "io/IOObject.java": ["public final void setPollIn(Handle handle)", "public final void setPollOut(Handle handle)",
                             "public final void resetPollIn(Handle handle)", "public final void resetPollOut(Handle handle)"],
        "io/SessionBase.java": ["public void flush()"],
        "util/Errno.java": ["public boolean is(int err)"],
        "Options.java": ["public Mechanisms mechanism"],
        "io/mechanism/Mechanisms.java": ["CURVE"],
        "SocketBase.java": ["public final void eventHandshakeFailedProtocol(String addr, int errno)"],
        "poll/PollerBase.java": ["protected final Thread worker;"],
        "io/StreamEngine.java": ["private SocketChannel fd;", "private ByteBuffer inpos;", "private int insize;",
                                 "private int outsize;", "private boolean plugged;", "private Supplier<Msg> nextMsg;",
                                 "private Function<Msg, Boolean> processMsg;", "private boolean inputStopped;",
                                 "private boolean outputStopped;", "private void error(ErrorReason error)",
                                 "private final Supplier<Msg> pullMsgFromSession"],
        "poll/Poller.java": ["private final UncaughtExceptionHandler exnotification;"],
    }
    for f, members in need.items():
        text = open(os.path.join(base, f)).read()
        for m in members:
            assert m in text, (f, m)
