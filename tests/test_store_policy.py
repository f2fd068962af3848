"""The line stores' cache policy in the shipped library ("Non-temporal line
stores"): the seal kernels and the opens of unaligned bodies / plaintext / segments store their
lines non-temporal (`nt`); the aligned open into 4 KiB plaintext slots and the carried-line open
keep the default policy, which measured faster for them.  CPU only: the gfx950 code object is cut
out of the .so and disassembled (jeromq_amd/build.py)."""
import os
import re
import subprocess
import sys
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
REGION = "_ZN12_GLOBAL__N_114k_seal_uniformILi2ELb0ELi0E"  # 100 B seal: EmitRegion's whole-region stores


@pytest.fixture(scope="module")
def line_stores():
    """kernel symbol -> list of the policy suffixes of its buffer_store_dwordx4 line stores"""
    from jeromq_amd import build
    if not os.path.exists(build.LIB):
        pytest.skip("library not built")
    out = {}
    for co in build.device_code_objects(build.LIB):
        with tempfile.NamedTemporaryFile(suffix=".co") as f:
            f.write(co)
            f.flush()
            text = subprocess.run([os.path.join(build.LLVM_BIN, "llvm-objdump"), "-d", "--mcpu=gfx950", f.name],
                                  check=True, capture_output=True, text=True).stdout
        cur = None
        for ln in text.splitlines():
            m = re.match(r"^[0-9a-f]+ <(.+)>:$", ln)
            if m:
                cur = m.group(1)
                out.setdefault(cur, [])
                continue
            t = ln.split("//")[0].strip()
            if cur and (t.startswith("buffer_store_dwordx4") or
                        (cur.startswith(REGION) and t.startswith("global_store_dwordx4"))):
                out[cur].append(" nt" in f" {t} ")
    return out


def _kernel(stores, prefix):
    names = [k for k in stores if k.startswith(prefix)]
    assert names, prefix
    return [x for k in names for x in stores[k]]


@pytest.mark.parametrize("prefix", [
    "_ZN12_GLOBAL__N_114k_seal_uniformILi1ELb1ELi0E",      # headline: EmitLines
    "_ZN12_GLOBAL__N_114k_seal_uniformILi3ELb1ELi0E",      # dense bodies: EmitShiftLinesUni
    "_ZN12_GLOBAL__N_114k_seal_uniformILi1ELb1ELi2E",      # box-layout input
    "_ZN12_GLOBAL__N_121k_seal_segments_lines",            # Zipf seal
    "_ZN12_GLOBAL__N_114k_open_uniformILi1ELb1ELi1E",      # open of dense bodies
    "_ZN12_GLOBAL__N_115k_open_segments",                  # Zipf open
])
def test_nontemporal_line_stores(line_stores, prefix):
    st = _kernel(line_stores, prefix)
    assert st and all(st), f"{prefix}: {st.count(False)} of {len(st)} line stores without nt"


@pytest.mark.parametrize("prefix", [
    "_ZN12_GLOBAL__N_114k_open_uniformILi1ELb1ELi16E",     # aligned open, 4 KiB plaintext slots
    "_ZN12_GLOBAL__N_120k_open_uniform_carryILi8E",        # carried-line open, 8-byte aligned bodies
])
def test_default_policy_line_stores(line_stores, prefix):
    st = _kernel(line_stores, prefix)
    assert st and not any(st), f"{prefix}: {sum(st)} of {len(st)} line stores nt"


def test_region_seal_stores_nontemporal(line_stores):
    """The 100 B seal's region stores (global_store_dwordx4 of the staged 64-slot region) are nt."""
    st = _kernel(line_stores, REGION)
    assert st and any(st), "no nt region store in the 100 B seal"
