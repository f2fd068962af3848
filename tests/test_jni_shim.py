"""The JNI binding (jni/curvezmq_jni.c, INTEGRATION.md sections 2-3) compiled and driven through a
fake JNIEnv (jni/fake_jni_env.c) -- there is no JDK in this image, so jni/jni_min.h restates the JNI
types and the function-table slots the shim calls (indices pinned by static asserts).

CPU: the shim compiles with -Wall -Wextra -Werror; every Java native the INTEGRATION classes declare
is exported under its JNI-mangled name; short / null arrays and wrong direct buffers are refused
before anything is read or the library entered; no Java array is pinned while the library runs
(inputs copied in with GetByteArrayRegion, outputs copied back with SetByteArrayRegion on success;
the library entry points are --wrap'ed in the test build to catch a call made under a pin).
GPU: one MESSAGE box sealed and opened through the jnacl natives (in a VM that hands out copies),
a uniform batch through GpuCurveBatch over direct buffers, and an engine round trip through
GpuCurveEngine, all against the oracle."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from cz_testlib import or_curve_encode, splitmix_bytes, v2_encode

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JNI = os.path.join(ROOT, "jni")
LIBDIR = os.path.join(ROOT, "jeromq_amd")
PRECOM = bytes.fromhex("0e8790cb0dc8703af2533cc8594eecfbf62ca560a66ebee1259cc0a30435c6f3")
JNI_ABORT = 2
CZ_EINVAL = -22

JNACL = "Java_com_neilalexander_jnacl_crypto_curve25519xsalsa20poly1305_"
SECRETBOX = "Java_com_neilalexander_jnacl_crypto_xsalsa20poly1305_"
BATCH = "Java_zmq_io_mechanism_curve_GpuCurveBatch_"
ENGINE = "Java_zmq_io_GpuCurveEngine_"
# the natives the Java classes of INTEGRATION.md declare, JNI-mangled ('_' in a name -> '_1')
NATIVES = ([JNACL + n for n in ("crypto_1box_1afternm", "crypto_1box_1open_1afternm", "crypto_1box_1beforenm",
                                "crypto_1box", "crypto_1box_1open", "crypto_1box_1keypair")]
           + [SECRETBOX + n for n in ("crypto_1secretbox", "crypto_1secretbox_1open")]
           + [BATCH + n for n in ("create", "destroy", "setKeys", "seal", "open", "sealUniform", "openUniform",
                                  "hostAlloc", "hostFree")]
           + [ENGINE + n for n in ("create", "destroy", "addConn", "removeConn", "msgAlloc", "send", "flushOut",
                                   "wireOut", "wireIov", "recv", "flushIn", "msgsIn", "msgIn", "connError")])
# library entry points the byte[] natives call (interposed in the test build)
from jeromq_amd.build import JNI_WRAPPED as WRAPPED  # noqa: E402

vp, i32, i64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64


@pytest.fixture(scope="module")
def shim(tmp_path_factory):
    if not os.path.exists(os.path.join(LIBDIR, "libcurvezmq_mi355x.so")):
        pytest.skip("library not built")
    out = str(tmp_path_factory.mktemp("jni") / "libcz_jni_test.so")
    # the library calls of the byte[] natives go through the fake's counting wrappers (--wrap), so a
    # call made while a Java array is pinned is seen
    wraps = ",".join("--wrap=" + f for f in WRAPPED)
    subprocess.run(["gcc", "-std=c11", "-O2", "-Wall", "-Wextra", "-Werror", "-DCZ_JNI_MIN", "-shared", "-fPIC",
                    "-I" + JNI, "-I" + os.path.join(ROOT, "include"), os.path.join(JNI, "curvezmq_jni.c"),
                    os.path.join(JNI, "fake_jni_env.c"), "-L" + LIBDIR, "-lcurvezmq_mi355x",
                    "-Wl,-rpath," + LIBDIR, "-Wl," + wraps, "-o", out], check=True)
    from jeromq_amd import _lib
    _lib._torch_runtime_first()   # the shim's library on torch's HIP runtime, as _lib.lib() loads it
    L = ctypes.CDLL(out)
    for f in ("fake_env", "fake_byte_array", "fake_int_array", "fake_direct", "fake_heap_buffer", "fake_elem",
              "fake_addr"):
        getattr(L, f).restype = vp
    L.fake_byte_array.argtypes = [vp, i32]
    L.fake_int_array.argtypes = [vp, i32]
    L.fake_direct.argtypes = [vp, i64]
    L.fake_cap.restype = i64
    for f in ("fake_pins", "fake_releases", "fake_last_mode", "fake_kind", "fake_len", "fake_addr", "fake_cap",
              "fake_gets", "fake_sets"):
        getattr(L, f).argtypes = [vp]
    L.fake_elem.argtypes = [vp, i32]
    L.fake_pin.argtypes = [vp]
    L.fake_unpin.argtypes = [vp]
    L.fake_fail_new_at.argtypes = [i32]
    for n in NATIVES:
        fn = getattr(L, n)
        fn.restype = vp if n.endswith(("hostAlloc", "msgAlloc", "wireOut", "wireIov", "msgIn")) else i32
        if n.startswith((JNACL, SECRETBOX)):   # (env, cls, byte[] ..., int len, byte[] ...)
            fn.argtypes = ([vp, vp, vp, vp, i32, vp, vp] if "afternm" in n or "secretbox" in n
                           else [vp, vp, vp, vp, i32, vp, vp, vp] if n.endswith(("crypto_1box", "crypto_1box_1open"))
                           else [vp, vp, vp, vp, vp] if n.endswith("beforenm") else [vp, vp, vp, vp])
    getattr(L, BATCH + "create").restype = i64
    getattr(L, ENGINE + "create").restype = i64
    L.env = L.fake_env()
    return L


class Arr:
    """A Java byte[] / int[] over a numpy buffer."""

    def __init__(self, L, data, ints=False):
        self.np = np.ascontiguousarray(data)
        self.obj = (L.fake_int_array if ints else L.fake_byte_array)(self.np.ctypes.data, len(self.np))
        self.L = L

    def pins(self):
        return self.L.fake_pins(self.obj)

    def releases(self):
        return self.L.fake_releases(self.obj)

    def mode(self):
        return self.L.fake_last_mode(self.obj)

    def gets(self):
        return self.L.fake_gets(self.obj)

    def sets(self):
        return self.L.fake_sets(self.obj)


def _u8(b):
    return np.frombuffer(bytes(b), dtype=np.uint8).copy()


def _box_args(L, mlen=132, n_len=24, k_len=32, c_len=None):
    m = np.zeros(mlen, dtype=np.uint8)
    m[32:] = _u8(splitmix_bytes(mlen - 32, 3))
    return (Arr(L, np.zeros(c_len if c_len is not None else mlen, dtype=np.uint8)), Arr(L, m),
            Arr(L, _u8(b"CurveZMQMESSAGEC" + (3).to_bytes(8, "big"))[:n_len]), Arr(L, _u8(PRECOM)[:k_len]))


def test_shim_compiles_and_exports_every_native(shim):
    nm = subprocess.run(["nm", "-D", "--defined-only", shim._name], capture_output=True, text=True, check=True).stdout
    syms = {ln.split()[-1] for ln in nm.splitlines() if ln.strip()}
    missing = [n for n in NATIVES if n not in syms]
    assert not missing, missing
    # the committed Java declarations (jni/java) mangle to exactly these natives
    import re
    declared = set()
    for dp, _, files in os.walk(os.path.join(JNI, "java")):
        for f in files:
            src = open(os.path.join(dp, f)).read()
            pkg = re.search(r"^package ([\w.]+);", src, re.M).group(1)
            cls = f[:-len(".java")]
            for meth in re.findall(r"static native [\w\[\]]+ (\w+)\(", src):
                declared.add("Java_" + (pkg + "." + cls).replace("_", "_1").replace(".", "_") + "_"
                             + meth.replace("_", "_1"))
    assert declared == set(NATIVES), declared ^ set(NATIVES)


def _java_sources():
    import re
    out = {}
    for dp, _, files in os.walk(os.path.join(JNI, "java")):
        for f in files:
            if f.endswith(".java"):
                out[os.path.relpath(os.path.join(dp, f), os.path.join(JNI, "java"))] = open(os.path.join(dp, f)).read()
    return out


def test_java_callers_call_only_declared_natives():
    """The Java callers (GpuCurveIoHook, GpuCurveMessageBatch, the GPU CURVE
    mechanisms) cannot be compiled here (no JDK): check that every GpuCurveEngine / GpuCurveBatch call
    they make names a native the classes declare -- and so, by the mangling test above, a symbol the
    shim exports -- with the declared number of arguments; that each file's package and class match
    its path; and that braces and parentheses balance outside comments and strings."""
    import re
    srcs = _java_sources()
    natives = {}
    for path, src in srcs.items():
        cls = os.path.basename(path)[:-len(".java")]
        for ret, meth, args in re.findall(r"static native ([\w\[\]]+) (\w+)\(([^)]*)\)", src):
            natives[(cls, meth)] = len([a for a in args.split(",") if a.strip()])
    calls = 0
    for path, src in srcs.items():
        code = re.sub(r"//[^\n]*|\"(?:\\.|[^\"\\])*\"", "", src)
        pkg = re.search(r"^package ([\w.]+);", src, re.M).group(1)
        assert path == os.path.join(*pkg.split("."), os.path.basename(path)), path
        cls = os.path.basename(path)[:-len(".java")]
        assert re.search(r"\b(class|interface) " + cls + r"\b", code), path
        assert code.count("{") == code.count("}") and code.count("(") == code.count(")"), path
        for m in re.finditer(r"\b(GpuCurveEngine|GpuCurveBatch)\.(\w+)\(", code):
            owner, meth = m.group(1), m.group(2)
            assert (owner, meth) in natives, (path, owner, meth)
            # count the call's top-level arguments
            depth, i, nargs, start = 1, m.end(), 0, m.end()
            while depth:
                ch = code[i]
                depth += ch in "([{"
                depth -= ch in ")]}"
                if ch == "," and depth == 1:
                    nargs += 1
                i += 1
            nargs += 1 if code[start:i - 1].strip() else 0
            assert nargs == natives[(owner, meth)], (path, owner, meth, nargs)
            calls += 1
    assert calls >= 20
    for f in ("zmq/io/GpuCurveIoHook.java", "zmq/io/mechanism/curve/GpuCurveMessageBatch.java", "zmq/io/mechanism/curve/GpuCurveClientMechanism.java",
              "zmq/io/mechanism/curve/GpuCurveServerMechanism.java"):
        assert f in srcs, f


REF_JAVA = "/root/reference/jeromq-core/src/main/java/zmq"


@pytest.mark.skipif(not os.path.isdir(REF_JAVA), reason="reference sources not present (build container only)")
def test_java_callers_use_reference_api_that_exists():
    """Every JeroMQ member the Java callers rely on exists in the reference with that signature
    (read as text: the reference is never built or run here)."""
    need = {
        "Msg.java": ["public Msg(final ByteBuffer src)", "public Msg(byte[] src)", "public Msg(int capacity)",
                     "public boolean hasMore()", "public boolean isCommand()", "public void setFlags(int flags)",
                     "public ByteBuffer buf()", "public int size()", "public Msg put(ByteBuffer src, int off, int len)",
                     "public static final int MORE", "public static final int COMMAND"],
        "io/SessionBase.java": ["public SocketBase getSocket()", "public String getEndpoint()"],
        "SocketBase.java": ["public final void eventHandshakeFailedProtocol(String addr, int errno)"],
        "Options.java": ["public final Errno errno", "public boolean asServer"],
        "util/Errno.java": ["public void set(int errno)"],
        "io/mechanism/Mechanism.java": ["protected final SessionBase session;", "public Msg decode(Msg msg)",
                                        "public Msg encode(Msg msg)", "public abstract Status status();"],
        "io/mechanism/curve/CurveClientMechanism.java": ["public class CurveClientMechanism extends Mechanism",
                                                         "public CurveClientMechanism(SessionBase session, Options options)",
                                                         "private final byte[] cnPrecom", "private long cnNonce;",
                                                         "private long cnPeerNonce;"],
        "io/mechanism/curve/CurveServerMechanism.java": [
            "public class CurveServerMechanism extends Mechanism",
            "public CurveServerMechanism(SessionBase session, Address peerAddress, Options options)",
            "private final byte[] cnPrecom", "private long cnNonce;", "private long cnPeerNonce;"],
        "ZMQ.java": ["ZMQ_PROTOCOL_ERROR_ZMTP_UNEXPECTED_COMMAND ", "ZMQ_PROTOCOL_ERROR_ZMTP_MALFORMED_COMMAND_MESSAGE ",
                     "ZMQ_PROTOCOL_ERROR_ZMTP_CRYPTOGRAPHIC ", "ZMQ_PROTOCOL_ERROR_ZMTP_INVALID_SEQUENCE "],
        "ZError.java": ["public static final int EPROTO"],
    }
    for f, members in need.items():
        text = open(os.path.join(REF_JAVA, f)).read()
        for m in members:
            assert m in text, (f, m)


@pytest.mark.parametrize("case", ["short_c", "short_m", "short_nonce", "short_key", "mlen_below_32", "null_m"])
def test_jnacl_length_guards_touch_nothing(shim, case):
    L = shim
    L.fake_reset_log()
    L.fake_reset_lib_calls()
    mlen = 132
    kw = {"short_c": dict(c_len=131), "short_nonce": dict(n_len=23), "short_key": dict(k_len=31)}.get(case, {})
    c, m, n, k = _box_args(L, mlen=mlen, **kw)
    marg = None if case == "null_m" else m.obj
    if case == "short_m":
        m = Arr(L, np.zeros(mlen - 1, dtype=np.uint8))
        marg = m.obj
    if case == "mlen_below_32":
        mlen = 31
    rc = getattr(L, JNACL + "crypto_1box_1afternm")(L.env, None, c.obj, marg, mlen, n.obj, k.obj)
    assert rc == -1
    assert L.fake_nmodes() == 0 and L.fake_outstanding() == 0 and L.fake_lib_calls() == 0
    assert all(a.pins() == 0 and a.gets() == 0 and a.sets() == 0 for a in (c, m, n, k))


def test_jnacl_pending_exception_stops_before_the_library(shim):
    """A VM exception raised while the inputs are copied in (ExceptionCheck) ends the call with -1:
    the library is not entered and nothing is written back."""
    L = shim
    c, m, n, k = _box_args(L)
    L.fake_reset_refs()
    L.fake_reset_lib_calls()
    L.fake_raise()
    try:
        rc = getattr(L, JNACL + "crypto_1box_1afternm")(L.env, None, c.obj, m.obj, 132, n.obj, k.obj)
    finally:
        L.fake_reset_refs()
    assert rc == -1 and L.fake_lib_calls() == 0 and c.sets() == 0 and not c.np.any()


def test_jnacl_never_pins_across_the_library_call(shim):
    """no Java array is pinned while the library runs (a GPU launch + sync): every
    byte[] native reads its inputs once with GetByteArrayRegion, makes its one library call (counted
    by the --wrap'ed entry point, which also records whether any array was pinned at that moment),
    and writes its outputs back with SetByteArrayRegion only when the call succeeded.  Without a GPU
    the calls return -1 and the output arrays stay untouched; with one they seal.  The detector itself
    is checked by calling with an array held pinned."""
    L = shim
    for fn in (JNACL + "crypto_1box_1afternm", JNACL + "crypto_1box_1open_1afternm",
               SECRETBOX + "crypto_1secretbox", SECRETBOX + "crypto_1secretbox_1open"):
        c, m, n, k = _box_args(L)
        L.fake_reset_log()
        L.fake_reset_lib_calls()
        rc = getattr(L, fn)(L.env, None, c.obj, m.obj, 132, n.obj, k.obj)
        assert L.fake_lib_calls() == 1 and L.fake_lib_calls_pinned() == 0, fn
        assert L.fake_outstanding() == 0 and L.fake_calls_in_critical() == 0 and L.fake_nmodes() == 0
        assert [a.pins() for a in (c, m, n, k)] == [0, 0, 0, 0]
        assert [a.gets() for a in (c, m, n, k)] == [0, 1, 1, 1]        # inputs read once, the output never
        assert c.sets() == (1 if rc == 0 else 0) and m.sets() == n.sets() == k.sets() == 0
    pk, sk = Arr(L, np.zeros(32, np.uint8)), Arr(L, np.zeros(32, np.uint8))
    L.fake_reset_lib_calls()
    rc = getattr(L, JNACL + "crypto_1box_1keypair")(L.env, None, pk.obj, sk.obj)
    assert L.fake_lib_calls() == 1 and L.fake_lib_calls_pinned() == 0 and pk.pins() == sk.pins() == 0
    assert pk.sets() == sk.sets() == (1 if rc == 0 else 0)
    # a box above the kept staging size (1 MiB): staged, freed after its call, then a small one again
    for mlen in (3 << 20, 132):
        big_c, big_m = Arr(L, np.zeros(mlen, np.uint8)), Arr(L, np.zeros(mlen, np.uint8))
        _, _, n, k = _box_args(L)
        L.fake_reset_lib_calls()
        rc = getattr(L, JNACL + "crypto_1box_1afternm")(L.env, None, big_c.obj, big_m.obj, mlen, n.obj, k.obj)
        assert L.fake_lib_calls() == 1 and L.fake_lib_calls_pinned() == 0 and big_m.gets() == 1
        assert big_c.sets() == (1 if rc == 0 else 0)
    # the detector: a call made while some array is pinned is counted as such
    c, m, n, k = _box_args(L)
    other = Arr(L, np.zeros(8, np.uint8))
    L.fake_reset_lib_calls()
    L.fake_pin(other.obj)
    try:
        getattr(L, JNACL + "crypto_1box_1afternm")(L.env, None, c.obj, m.obj, 132, n.obj, k.obj)
    finally:
        L.fake_unpin(other.obj)
    assert L.fake_lib_calls() == 1 and L.fake_lib_calls_pinned() == 1 and L.fake_outstanding() == 0


def test_batch_and_engine_refuse_bad_buffers(shim):
    L = shim
    heap = L.fake_heap_buffer()
    buf = np.zeros(1 << 16, dtype=np.uint8)
    d = L.fake_direct(buf.ctypes.data, buf.nbytes)
    short = L.fake_direct(buf.ctypes.data, 39)
    seal = getattr(L, BATCH + "seal")
    seal.argtypes = [vp, vp, i64, vp, i32, vp, vp]
    assert seal(L.env, None, 1, short, 1, d, d) == CZ_EINVAL        # descs shorter than count x 40
    assert seal(L.env, None, 1, d, 1, heap, d) == CZ_EINVAL         # heap (non-direct) input
    assert seal(L.env, None, 0, d, 1, d, d) == CZ_EINVAL            # no context
    su = getattr(L, BATCH + "sealUniform")
    su.argtypes = [vp, vp, i64, i32, i32, vp, i64, vp, i64, i64, vp, i32]
    # 4 frames of 100 B at stride 112 into 144-byte slots need 3*112+100 in, 4*144 out
    assert su(L.env, None, 1, 4, 100, L.fake_direct(buf.ctypes.data, 3 * 112 + 99), 112, d, 144, 3, None, 0) \
        == CZ_EINVAL
    assert su(L.env, None, 1, 4, 100, d, 112, L.fake_direct(buf.ctypes.data, 4 * 144 - 1), 144, 3, None, 0) \
        == CZ_EINVAL
    assert su(L.env, None, 1, 4, 100, d, 112, d, 144, 3, L.fake_direct(buf.ctypes.data, 3), 0) == CZ_EINVAL
    ou = getattr(L, BATCH + "openUniform")
    ou.argtypes = [vp, vp, i64, i32, i32, vp, i64, vp, i64, i64, ctypes.c_uint8, vp, i32]
    assert ou(L.env, None, 1, 4, 32, d, 144, d, 112, 2, 1, d, 0) == CZ_EINVAL   # size below 33
    assert ou(L.env, None, 1, 4, 133, d, 144, d, 112, 2, 1, L.fake_direct(buf.ctypes.data, 7), 0) == CZ_EINVAL
    send = getattr(L, ENGINE + "send")
    send.argtypes = [vp, vp, i64, i32, vp, i32, i32]
    assert send(L.env, None, 1, 0, L.fake_direct(buf.ctypes.data, 10), 11, 0) == CZ_EINVAL
    assert send(L.env, None, 0, 0, d, 10, 0) == CZ_EINVAL
    ce = getattr(L, ENGINE + "connError")
    ce.argtypes = [vp, vp, i64, i32, vp]
    assert ce(L.env, None, 1, 0, Arr(L, np.zeros(0, np.int32), ints=True).obj) == CZ_EINVAL
    assert getattr(L, ENGINE + "flushOut")(L.env, None, ctypes.c_int64(0)) == CZ_EINVAL


def test_uniform_strides_that_overflow_are_refused(shim):
    """count x stride products are checked before the library is entered: a 2^62 stride over 4 frames
    wraps a signed 64-bit need to 0 (so any buffer would pass) -- refused with CZ_EINVAL, as is a
    stride whose (count - 1) * stride + len overflows."""
    L = shim
    buf = np.zeros(1 << 12, dtype=np.uint8)
    d = L.fake_direct(buf.ctypes.data, buf.nbytes)
    su = getattr(L, BATCH + "sealUniform")
    su.argtypes = [vp, vp, i64, i32, i32, vp, i64, vp, i64, i64, vp, i32]
    assert su(L.env, None, 1, 4, 100, d, 112, d, 1 << 62, 3, None, 0) == CZ_EINVAL
    assert su(L.env, None, 1, 4, 100, d, 1 << 62, d, 144, 3, None, 0) == CZ_EINVAL
    assert su(L.env, None, 1, 3, 100, d, (1 << 62) + 1, d, 144, 3, None, 0) == CZ_EINVAL
    ou = getattr(L, BATCH + "openUniform")
    ou.argtypes = [vp, vp, i64, i32, i32, vp, i64, vp, i64, i64, ctypes.c_uint8, vp, i32]
    assert ou(L.env, None, 1, 4, 133, d, 144, d, 1 << 62, 2, 1, d, 0) == CZ_EINVAL
    assert ou(L.env, None, 1, 4, 133, d, 1 << 62, d, 112, 2, 1, d, 0) == CZ_EINVAL


def _has_gpu():
    """device_count() does not initialize torch's HIP runtime.  is_available() would, and torch
    bundles its own libamdhip64: a process that has loaded the library (here through the shim) and
    then initializes torch's runtime before the library's first HIP call leaves the library with no
    device (tools/diag/hip_init_order.py: lib-torch-call fails; lib-call, lib-count-call and
    torch-lib-call work)."""
    try:
        import torch
        return torch.cuda.device_count() > 0
    except Exception:
        return False


@pytest.mark.gpu
def test_jni_seal_open_through_the_shim(shim):
    """One MESSAGE box through crypto_box_afternm / crypto_box_open_afternm as JeroMQ's Curve.java
    calls them, in a VM that hands out copies (so a wrong release mode loses the output): the box
    equals the oracle's MESSAGE body; the open gives back m; a tampered box is -1."""
    if not _has_gpu():
        pytest.skip("no GPU")
    L = shim
    L.fake_set_copy_mode(1)
    try:
        payload = splitmix_bytes(100, 11)
        m = np.zeros(133, dtype=np.uint8)
        m[32] = 1                                  # flags byte (MORE)
        m[33:] = _u8(payload)
        c, n, k = (Arr(L, np.zeros(133, np.uint8)), Arr(L, _u8(b"CurveZMQMESSAGEC" + (3).to_bytes(8, "big"))),
                   Arr(L, _u8(PRECOM)))
        ma = Arr(L, m)
        from jeromq_amd import _lib
        rc = getattr(L, JNACL + "crypto_1box_1afternm")(L.env, None, c.obj, ma.obj, 133, n.obj, k.obj)
        assert rc == 0, _lib.last_error()
        body = or_curve_encode(payload, 1, 3, 0, PRECOM)     # "\x07MESSAGE" || nonce[16:24] || box[16:]
        assert c.np[:16].tobytes() == bytes(16) and c.np[16:].tobytes() == body[16:]
        back = Arr(L, np.full(133, 0xAA, np.uint8))
        assert getattr(L, JNACL + "crypto_1box_1open_1afternm")(L.env, None, back.obj, c.obj, 133, n.obj, k.obj) == 0
        assert back.np[:32].tobytes() == bytes(32) and back.np[32:].tobytes() == m[32:].tobytes()
        c.np[60] ^= 1
        assert getattr(L, JNACL + "crypto_1box_1open_1afternm")(L.env, None, back.obj, c.obj, 133, n.obj, k.obj) == -1
        assert L.fake_outstanding() == 0
        # NaCl for every m: a box whose m[0:32] is not zero seals (rc 0) to libsodium's bytes, through
        # crypto_box_afternm and crypto_secretbox alike (golden vectors, tests/golden/make_golden.py)
        from cz_testlib import load_golden
        for v in load_golden()["box_afternm_prefix"]:
            if "c" not in v:
                continue
            mlen = v["mlen"]
            for fn in (JNACL + "crypto_1box_1afternm", SECRETBOX + "crypto_1secretbox"):
                cc = Arr(L, np.full(mlen, 0x5A, np.uint8))
                mm = Arr(L, _u8(splitmix_bytes(mlen, v["m_seed"])))
                assert getattr(L, fn)(L.env, None, cc.obj, mm.obj, mlen, Arr(L, _u8(bytes.fromhex(v["nonce"]))).obj,
                                      Arr(L, _u8(bytes.fromhex(v["key"]))).obj) == 0, (fn, mlen)
                assert cc.np.tobytes().hex() == v["c"], (fn, mlen)
        # a 3 MiB box (past the 1 MiB of staging kept between calls) round-trips, and the 133-byte box
        # after it seals to the same bytes as before
        big = np.zeros(3 << 20, dtype=np.uint8)
        big[32:] = _u8(splitmix_bytes(big.size - 32, 12))
        bc, bm = Arr(L, np.zeros(big.size, np.uint8)), Arr(L, big)
        assert getattr(L, JNACL + "crypto_1box_1afternm")(L.env, None, bc.obj, bm.obj, big.size, n.obj, k.obj) == 0
        bb = Arr(L, np.zeros(big.size, np.uint8))
        assert getattr(L, JNACL + "crypto_1box_1open_1afternm")(L.env, None, bb.obj, bc.obj, big.size, n.obj, k.obj) == 0
        assert np.array_equal(bb.np, big)
        c2 = Arr(L, np.zeros(133, np.uint8))
        assert getattr(L, JNACL + "crypto_1box_1afternm")(L.env, None, c2.obj, ma.obj, 133, n.obj, k.obj) == 0
        assert c2.np[16:].tobytes() == body[16:]
        assert L.fake_outstanding() == 0 and L.fake_calls_in_critical() == 0 and L.fake_lib_calls_pinned() == 0
    finally:
        L.fake_set_copy_mode(0)


@pytest.mark.gpu
def test_jni_batch_and_engine_through_the_shim(shim):
    """GpuCurveBatch.sealUniform over pinned direct buffers from hostAlloc, and a GpuCurveEngine
    send -> flushOut -> wireOut, against the oracle."""
    if not _has_gpu():
        pytest.skip("no GPU")
    L = shim
    create = getattr(L, BATCH + "create")
    create.argtypes = [vp, vp, i32]
    ctx = create(L.env, None, 0)
    assert ctx
    ha = getattr(L, BATCH + "hostAlloc")
    ha.argtypes = [vp, vp, i64]
    count, n, ist, ost = 64, 4096, 4096, 4224
    bin_, bout, keys = ha(L.env, None, count * ist), ha(L.env, None, count * ost), ha(L.env, None, 32)
    assert bin_ and bout and keys and L.fake_cap(bin_) == count * ist
    hin = np.ctypeslib.as_array((ctypes.c_uint8 * (count * ist)).from_address(L.fake_addr(bin_)))
    hin[:] = _u8(splitmix_bytes(count * ist, 21))
    ctypes.memmove(L.fake_addr(keys), PRECOM, 32)
    sk = getattr(L, BATCH + "setKeys")
    sk.argtypes = [vp, vp, i64, vp, i32, i32]
    assert sk(L.env, None, ctx, keys, 1, 0) == 0
    su = getattr(L, BATCH + "sealUniform")
    su.argtypes = [vp, vp, i64, i32, i32, vp, i64, vp, i64, i64, vp, i32]
    assert su(L.env, None, ctx, count, n, bin_, ist, bout, ost, 5, None, 0) == 0
    hout = np.ctypeslib.as_array((ctypes.c_uint8 * (count * ost)).from_address(L.fake_addr(bout)))
    for i in (0, 31, count - 1):
        assert hout[i * ost:i * ost + n + 33].tobytes() == or_curve_encode(hin[i * ist:(i + 1) * ist].tobytes(), 0,
                                                                           5 + i, 0, PRECOM)
    hf = getattr(L, BATCH + "hostFree")
    hf.argtypes = [vp, vp, vp]
    for b in (bin_, bout, keys):
        hf(L.env, None, b)
    getattr(L, BATCH + "destroy").argtypes = [vp, vp, i64]
    getattr(L, BATCH + "destroy")(L.env, None, ctx)

    ec = getattr(L, ENGINE + "create")
    ec.argtypes = [vp, vp, i64, i32]
    e = ec(L.env, None, 1 << 20, 0)
    assert e
    add = getattr(L, ENGINE + "addConn")
    add.argtypes = [vp, vp, i64, ctypes.c_uint8, vp, i64, i64]
    conn = add(L.env, None, e, 0, Arr(L, _u8(PRECOM)).obj, 3, 2)
    assert conn == 0
    ma = getattr(L, ENGINE + "msgAlloc")
    ma.argtypes = [vp, vp, i64, i32]
    payloads = [splitmix_bytes(sz, 40 + sz) for sz in (0, 100, 5000)]
    send = getattr(L, ENGINE + "send")
    send.argtypes = [vp, vp, i64, i32, vp, i32, i32]
    for j, p in enumerate(payloads):
        b = ma(L.env, None, e, len(p))
        assert b and L.fake_cap(b) == len(p)
        if p:
            ctypes.memmove(L.fake_addr(b), p, len(p))
        assert send(L.env, None, e, conn, b, len(p), 1 if j == 0 else 0) == 0
    getattr(L, ENGINE + "flushOut").argtypes = [vp, vp, i64]
    assert getattr(L, ENGINE + "flushOut")(L.env, None, e) == 0
    wo = getattr(L, ENGINE + "wireOut")
    wo.argtypes = [vp, vp, i64, i32]
    w = wo(L.env, None, e, conn)
    got = ctypes.string_at(L.fake_addr(w), L.fake_cap(w))
    want = b"".join(v2_encode(or_curve_encode(p, 1 if j == 0 else 0, 3 + j, 0, PRECOM)) for j, p in enumerate(payloads))
    assert got == want
    wi = getattr(L, ENGINE + "wireIov")
    wi.argtypes = [vp, vp, i64, i32]
    L.fake_reset_refs()
    arr = wi(L.env, None, e, conn)
    pieces = [L.fake_elem(arr, i) for i in range(L.fake_len(arr))]
    assert b"".join(ctypes.string_at(L.fake_addr(p), L.fake_cap(p)) for p in pieces) == want
    # each piece's local reference is deleted once stored: only the returned array stays live
    assert L.fake_live_refs() == 1 and L.fake_max_live_refs() <= 3 and not L.fake_exception()
    # an allocation that fails (exception pending) ends the call: NULL, no reference left behind
    L.fake_reset_refs()
    L.fake_fail_new_at(0)
    assert not wi(L.env, None, e, conn)
    assert L.fake_exception() and L.fake_live_refs() == 0
    L.fake_reset_refs()
    getattr(L, ENGINE + "destroy").argtypes = [vp, vp, i64]
    getattr(L, ENGINE + "destroy")(L.env, None, e)
