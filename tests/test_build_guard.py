"""The product library is built only from the committed sources and flags.

jeromq_amd/build.py refuses CZ_EXTRA_FLAGS for the product output (jeromq_amd/libcurvezmq_mi355x.so),
so a variable left set on a build box cannot ship an A/B variant or a wrong-output diagnostic; A/B
builds name another output with CZ_LIB_OUT.  The one diagnostic hook left in the kernels
(cz_diag.h, CZ_DIAG_NOSTORE_ALL) and the round-6 clock stamps (CZ_DIAG_CLOCK, tools/clock_stamp.py) also
#error when compiled with -DCZ_PRODUCT_BUILD."""
import os
import subprocess

import pytest

from jeromq_amd import build

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_product_build_refuses_extra_flags(monkeypatch):
    with pytest.raises(build.ProductFlagsError):
        build.compile_flags(build.PRODUCT_LIB, "-DCZ_DIAG_NOSTORE_ALL")
    monkeypatch.setenv("CZ_EXTRA_FLAGS", "-DCZ_DIAG_NOSTORE_ALL")
    with pytest.raises(build.ProductFlagsError):  # before any compile starts
        build.build_library(force=True, verbose=False, lib=build.PRODUCT_LIB)
    flags = build.compile_flags(build.PRODUCT_LIB, "")
    assert "-DCZ_PRODUCT_BUILD" in flags and not any(f.startswith("-DCZ_DIAG") for f in flags)


def test_ab_builds_take_their_flags(tmp_path):
    flags = build.compile_flags(str(tmp_path / "libcz_ab.so"), "-DCZ_DIAG_NOSTORE_ALL -DCZ_UNIFORM_WAVES_PER_EU=2")
    assert "-DCZ_DIAG_NOSTORE_ALL" in flags and "-DCZ_PRODUCT_BUILD" not in flags


@pytest.mark.parametrize("defs, ok", [(["-DCZ_PRODUCT_BUILD"], True), (["-DCZ_DIAG_NOSTORE_ALL"], True),
                                      (["-DCZ_PRODUCT_BUILD", "-DCZ_DIAG_NOSTORE_ALL"], False),
                                      (["-DCZ_DIAG_CLOCK"], True), (["-DCZ_PRODUCT_BUILD", "-DCZ_DIAG_CLOCK"], False)])
def test_diag_header_refuses_product_builds(tmp_path, defs, ok):
    src = tmp_path / "d.cpp"
    src.write_text('#include "cz_diag.h"\nstruct V { unsigned x, w; };\n'
                   'int f(V v) { int r = 0; CZ_DIAG_STORE_GUARD(v) r = 1; return r; }\n')
    r = subprocess.run(["g++", "-fsyntax-only", *defs, "-I", os.path.join(ROOT, "jeromq_amd", "csrc"), str(src)],
                       capture_output=True, text=True)
    assert (r.returncode == 0) == ok, r.stderr
    if not ok:
        assert "never in the product library" in r.stderr


def test_no_rejected_variant_switches_in_product_sources():
    """Variants measured and rejected live in the git history, not behind #ifdefs in the product."""
    gone = ["CZ_FLUSH2", "CZ_UGLD", "CZ_BOX_FENCE", "CZ_SEAL_LOAD_NT", "CZ_AL8_X4", "CZ_SEG_SINGLE_KERNEL",
            "CZ_SALSA_LAZY_SPLIT", "CZ_SALSA_EAGER", "CZ_DIAG_NOLOAD", "CZ_DIAG_NOTAG", "CZ_DIAG_L2STORE",
            "CZ_DIAG_NOSHIFTROW", "CZ_NACL_SEGMENTED", "CZ_CTX_LANES_ONLY"]
    csrc = os.path.join(ROOT, "jeromq_amd", "csrc")
    for f in os.listdir(csrc):
        if f.endswith((".hip", ".cpp", ".h")) and f != "cz_diag.h":
            text = open(os.path.join(csrc, f)).read()
            assert not [g for g in gone if g in text], f
            assert "CZ_DIAG_NOSTORE_ALL" not in text or f == "cz_diag.h", f


def test_loader_imports_torch_before_the_library():
    """One HIP runtime per process: jeromq_amd._lib.lib() imports torch, whose
    bundled libamdhip64 then serves the library's HIP calls, before it dlopens the library."""
    import inspect
    import sys
    from jeromq_amd import _lib
    src = inspect.getsource(_lib.lib)
    assert src.index("_torch_runtime_first()") < src.index("ctypes.CDLL(LIB_PATH)")
    _lib._torch_runtime_first()
    assert "torch" in sys.modules
