"""CPU-side checks of the drop-in boundary: the C-ABI library loads, exports every
function include/curvezmq_mi355x.h declares, the descriptor layout matches, and
without a GPU every compute entry point fails loudly (no CPU fallback)."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from cz_testlib import DESC_DTYPE, ROOT

HEADER = os.path.join(ROOT, "include", "curvezmq_mi355x.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(cz_[a-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    from jeromq_amd import _lib
    from jeromq_amd.build import build_library
    build_library()
    return _lib.lib()


def test_header_declares_the_boundary():
    fns = declared_functions()
    for must in ["cz_box_afternm", "cz_box_open_afternm", "cz_seal_batch", "cz_open_batch", "cz_subkeys",
                 "cz_seal_uniform", "cz_mech_encode", "cz_mech_decode"]:
        assert must in fns


def test_library_exports_every_declared_symbol(lib):
    missing = [f for f in declared_functions() if not hasattr(lib, f)]
    assert not missing, missing


def test_python_binding_covers_header():
    from jeromq_amd import _lib
    assert set(declared_functions()) == set(_lib.SIGNATURES)


def test_exported_symbols_via_nm(lib):
    from jeromq_amd import _lib
    out = subprocess.check_output(["nm", "-D", "--defined-only", _lib.LIB_PATH], text=True)
    syms = {line.split()[-1] for line in out.splitlines() if line.strip()}
    assert set(declared_functions()) <= syms


def test_desc_layout_matches_c(tmp_path):
    c = tmp_path / "layout.c"
    c.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "curvezmq_mi355x.h"\n'
                 'int main(void){printf("%zu %zu %zu %zu %zu %zu %zu %zu\\n", sizeof(cz_frame_desc),'
                 'offsetof(cz_frame_desc,in_off),offsetof(cz_frame_desc,out_off),offsetof(cz_frame_desc,len),'
                 'offsetof(cz_frame_desc,key_idx),offsetof(cz_frame_desc,counter),offsetof(cz_frame_desc,flags),'
                 'offsetof(cz_frame_desc,prev));return 0;}\n')
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.dirname(HEADER), str(c), "-o",
                           str(exe)])
    vals = list(map(int, subprocess.check_output([str(exe)], text=True).split()))
    assert vals[0] == DESC_DTYPE.itemsize == 40
    assert vals[1:] == [DESC_DTYPE.fields[k][1] for k in ("in_off", "out_off", "len", "key_idx", "counter", "flags",
                                                          "prev")]
    from jeromq_amd._lib import cz_frame_desc
    assert ctypes.sizeof(cz_frame_desc) == 40


def test_header_compiles_as_cxx(tmp_path):
    c = tmp_path / "h.cpp"
    c.write_text('#include "curvezmq_mi355x.h"\nint main(){cz_frame_desc d{}; return (int)d.len;}\n')
    subprocess.check_call(["g++", "-Wall", "-Werror", "-I", os.path.dirname(HEADER), str(c), "-o",
                           str(tmp_path / "h")])


@pytest.mark.skipif(os.path.exists("/dev/kfd") and os.access("/dev/kfd", os.R_OK), reason="GPU present")
def test_no_cpu_fallback_without_gpu(lib):
    from jeromq_amd import _lib
    assert lib.cz_device_ok() == 0
    c = ctypes.create_string_buffer(64)
    assert lib.cz_box_afternm(c, bytes(64), 64, bytes(24), bytes(32)) == -1
    assert "no HIP device" in _lib.last_error()
    out = ctypes.create_string_buffer(32)
    assert lib.cz_subkey(out, bytes(32), 0) == _lib.CZ_EHIP
    h = ctypes.c_void_p()
    assert lib.cz_ctx_create(ctypes.byref(h), 0) == _lib.CZ_EHIP
    assert not lib.cz_mech_create(0, bytes(32), 3, 1, 0)


def test_host_free_refuses_foreign_pointers(lib):
    """cz_host_free releases only live cz_host_alloc base addresses: a foreign or interior pointer
    is CZ_EINVAL and never reaches hipHostFree (hostFree of any direct ByteBuffer)."""
    from jeromq_amd import _lib
    buf = ctypes.create_string_buffer(64)
    assert lib.cz_host_free(ctypes.addressof(buf)) == _lib.CZ_EINVAL
    assert lib.cz_host_free(ctypes.addressof(buf) + 16) == _lib.CZ_EINVAL
    assert lib.cz_host_free(None) == _lib.CZ_OK


def test_plan_order_host_logic(lib):
    from jeromq_amd.batch import plan_order
    d = np.zeros(6, dtype=DESC_DTYPE)
    d["len"] = [5, 100, 5, 7, 100, 0]
    assert list(plan_order(d)) == [1, 4, 3, 0, 2, 5]


def test_argument_validation(lib):
    from jeromq_amd import _lib
    assert lib.cz_seal_uniform(4, 100, None, 100, None, 133, None, 0, None, None) == _lib.CZ_EINVAL
    assert lib.cz_seal_uniform(4, 100, 16, 50, 16, 133, 16, 0, None, None) == _lib.CZ_EINVAL  # stride < len
    assert lib.cz_subkeys(16, 16, 1, 7, None) == _lib.CZ_EINVAL


def test_plan_segments_orders_by_length_then_line_phase(lib):
    """cz_plan_segments (host): longest first; within one length, segments whose input starts on
    a 128-byte line before those starting 64 bytes into one (seal), so waves hold one phase; then
    by the output's line class (bit 6 of its offset), so waves of outputs packed at any byte offset
    hold one EmitShiftLines class."""
    import numpy as np
    from jeromq_amd.batch import DESC_DTYPE, SegmentPlan
    rng = np.random.default_rng(3)
    lens = (64 * rng.integers(1, 300, size=700)).astype(np.uint64)
    d = np.zeros(len(lens), dtype=DESC_DTYPE)
    d["len"] = lens
    d["in_off"][1:] = np.cumsum(lens[:-1])  # 64-byte packing: both phases occur
    d["out_off"][1:] = np.cumsum(lens[:-1] + np.uint64(40))  # 8-byte packed bodies: both classes occur
    plan = SegmentPlan(d, open_=False, seg_blocks=8)
    seg = plan.segments
    mlen = lens[seg["frame"]] + np.uint64(33)
    nb = seg["nblocks"].astype(np.int64)
    ph = ((d["in_off"][seg["frame"]] + np.uint64(64) * seg["first_block"].astype(np.uint64)) >> np.uint64(6)) & np.uint64(1)
    oc = ((d["out_off"][seg["frame"]] + np.uint64(64) * seg["first_block"].astype(np.uint64)) >> np.uint64(6)) & np.uint64(1)
    key = 4 * nb + 2 * (1 - ph.astype(np.int64)) + (1 - oc.astype(np.int64))
    assert np.all(np.diff(key) <= 0)
    assert len(set(oc.tolist())) == 2
    # every box block of every frame covered exactly once
    cover = {}
    for s in seg:
        cover.setdefault(int(s["frame"]), []).append((int(s["first_block"]), int(s["nblocks"])))
    for f, parts in cover.items():
        parts.sort()
        nblk = (int(lens[f]) + 33 + 63) // 64
        assert parts[0][0] == 0 and sum(n for _, n in parts) == nblk
        for (a, n), (b, _) in zip(parts, parts[1:]):
            assert a + n == b
    assert len(cover) == len(lens) and int(mlen.min()) >= 97
