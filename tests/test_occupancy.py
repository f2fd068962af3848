"""Occupancy guard for the shipped kernels (CPU: reads the code objects' AMDGPU metadata).

Every hot kernel here is VALU-issue-bound and hides its memory latency with 3 waves per SIMD
(DESIGN.md section 5).  A change that adds a few live registers can silently take a kernel to 2
waves: round 5's whole-unit edge change took the dense seal (k_seal_uniform<ST_SHIFT>) from 164 to
177 VGPRs and cost it ~2% until a waves_per_eu bound put it back.  On gfx950 a wave64 has 512
VGPRs per lane of its SIMD to share (arch + acc, allocated in granules of 8), so 3 waves need at
most 168."""
import os
import re
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# demangled-name pattern -> minimum waves per SIMD
MIN_WAVES = [
    (r"k_seal_uniformILi1ELb1ELi0E", 3),      # the headline: EmitLines, whole-line loads
    (r"k_seal_uniformILi3ELb1ELi0E", 3),      # dense bodies: EmitShiftLines (class-static, WHOLE)
    (r"k_seal_uniformILi1ELb1ELi2E", 3),      # box-layout input
    (r"k_seal_uniform_inaILi[13]ELb1E", 3),   # payloads off 16-byte alignment, line staging
    (r"k_open_uniformILi[13]ELb1E", 3),       # uniform opens, line staging
    (r"k_seal_segments_lines", 3),            # Zipf seal, line-staged waves
    (r"k_open_segments", 3),                  # Zipf open
    (r"k_nacl_one", 3),                       # the jnacl drop-in
]


def _kernels(lib):
    from jeromq_amd import build
    out = []
    for co in build.device_code_objects(lib):
        with tempfile.NamedTemporaryFile(suffix=".co") as f:
            f.write(co)
            f.flush()
            notes = subprocess.run([os.path.join(build.LLVM_BIN, "llvm-readelf"), "--notes", f.name],
                                   check=True, capture_output=True, text=True).stdout
        for blk in notes.split("  - .agpr_count:")[1:]:
            name = re.search(r"^\s+\.name:\s+(\S+)", blk, re.M)
            vg = re.search(r"^\s+\.vgpr_count:\s+(\d+)", blk, re.M)
            ag = re.match(r"\s*(\d+)", blk)
            if name and vg:
                out.append((name.group(1), int(vg.group(1)), int(ag.group(1)) if ag else 0))
    return out


def waves_per_simd(vgpr, agpr):
    alloc = (vgpr + 7) // 8 * 8 + (agpr + 7) // 8 * 8
    return 512 // max(alloc, 8)


def test_hot_kernels_keep_their_occupancy():
    from jeromq_amd import build
    if not os.path.exists(build.PRODUCT_LIB):
        pytest.skip("library not built")
    ks = _kernels(build.PRODUCT_LIB)
    assert ks, "no kernel metadata found"
    seen = set()
    for name, vg, ag in ks:
        for pat, need in MIN_WAVES:
            if re.search(pat, name):
                seen.add(pat)
                got = waves_per_simd(vg, ag)
                assert got >= need, f"{name}: {vg} VGPRs + {ag} AGPRs = {got} waves per SIMD, need {need}"
    missing = [p for p, _ in MIN_WAVES if p not in seen]
    assert not missing, f"kernels not found in the library: {missing}"


def test_waves_per_simd_arithmetic():
    assert waves_per_simd(168, 0) == 3
    assert waves_per_simd(177, 0) == 2
    assert waves_per_simd(147, 0) == 3
    assert waves_per_simd(128, 0) == 4
