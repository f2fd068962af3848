"""The build is gated on the ISA scan of the binary it links (jeromq_amd/build.py:isa_gate,
VERDICT r03 next #2): a deliberately injected wide buffer store with a register soffset -- the
construct behind round 3's silent wrong-output bug -- is compiled through build_library and must be
refused with no library installed, while the same kernel with soffset 0 builds.  The shipped
library itself is scanned the same way.  CPU only (hipcc cross-compiles gfx950)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
needs_hipcc = pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")

KERNEL = r"""
#include <hip/hip_runtime.h>
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
extern "C" __global__ void k_line_store(u32x4* out, const u32x4* in, unsigned soff) {
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(out, 0, 0x7fffffff, 0x00020000);
    u32x4 v = in[threadIdx.x];
    __builtin_amdgcn_raw_buffer_store_b128(v, r, threadIdx.x * 16, SOFFSET, 0);
}
"""


def _build(tmp_path, soffset):
    from jeromq_amd import build
    src = tmp_path / f"k_{soffset}.hip"
    src.write_text(KERNEL.replace("SOFFSET", soffset))
    lib = str(tmp_path / f"k_{soffset}.so")
    return build, lib, lambda: build.build_library(force=True, verbose=False, sources=[src.name], lib=lib,
                                                   src_dir=str(tmp_path))


@needs_hipcc
def test_gate_refuses_register_soffset_store(tmp_path):
    build, lib, run = _build(tmp_path, "soff")
    with pytest.raises(build.IsaHazardError, match="register soffset"):
        run()
    assert not os.path.exists(lib) and not [f for f in os.listdir(tmp_path) if f.endswith(".tmp")]


@needs_hipcc
def test_gate_passes_constant_soffset_store(tmp_path):
    build, lib, run = _build(tmp_path, "0")
    assert run() == lib and os.path.exists(lib)
    n_co, n_ins = build.isa_gate(lib)
    assert n_co == 1 and n_ins > 5


def test_shipped_library_passes_the_gate():
    """The in-tree product library (built by __graft_entry__.build) holds no store hazard."""
    from jeromq_amd import build
    if not os.path.exists(build.LIB):
        pytest.skip("library not built")
    n_co, n_ins = build.isa_gate(build.LIB)
    assert n_co == 4           # cz_kernels.hip (three parts, build.SOURCES) and cz_x25519.hip
    assert n_ins > 100000


def test_scanner_classes_on_listings():
    """The three hazard classes on hand-written llvm-objdump-style listings."""
    from isa_store_hazard import scan
    d, s, r = scan("global_store_dwordx4 v[2:3], v[4:7], off\nv_add_u32_e32 v5, v1, v2\n")
    assert len(d) == 1 and not s and not r
    d, s, r = scan("global_store_dwordx4 v[2:3], v[4:7], off\ns_nop 0\nv_add_u32_e32 v5, v1, v2\n")
    assert not d
    d, s, r = scan("v_readfirstlane_b32 s4, v1\nglobal_store_dword v1, v2, s[4:5]\n")
    assert len(s) == 1
    d, s, r = scan("v_readfirstlane_b32 s4, v1\ns_nop 4\nglobal_store_dword v1, v2, s[4:5]\n")
    assert not s
    d, s, r = scan("buffer_store_dwordx4 v[0:3], v4, s[4:7], s2 offen\n")
    assert len(r) == 1
    d, s, r = scan("buffer_store_dwordx4 v[0:3], v4, s[4:7], 0 offen\n")
    assert not r
