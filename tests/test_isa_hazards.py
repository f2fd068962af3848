"""The product kernels' gfx950 ISA holds no VMEM store hazard the compiler does not count
(tools/isa_store_hazard.py).  Round 2: an inline-asm global_store_dwordx4
(since retired) whose store-data and VALU-written-SGPR wait states the compiler did not count; a
rescheduled build stored a later VALU result into 4 lanes' output.  Round 3: buffer stores with a
register soffset, for which LLVM assumes no store-data hazard; a new Zipf flush stored LDS
addresses into a few lines per batch.  Compiles cz_kernels.hip device-only (about 90 s on this
container's CPUs; no GPU needed)."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


@pytest.mark.slow
@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_kernel_isa_has_no_asm_store_hazards(tmp_path):
    from isa_store_hazard import scan
    src = os.path.join(ROOT, "jeromq_amd", "csrc", "cz_kernels.hip")
    out = tmp_path / "cz_kernels.s"
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only", "-S", "-w",
                    "-o", str(out), src], check=True, cwd=str(tmp_path), timeout=900)
    data_hz, sgpr_hz, soff_reg = scan(out.read_text())
    assert data_hz == [], f"store data rewritten at distance 1: {data_hz[:3]}"
    assert sgpr_hz == [], f"VALU-written SGPR read by VMEM within 5 states: {sgpr_hz[:3]}"
    assert soff_reg == [], f"wide buffer stores with a register soffset: {soff_reg[:3]}"
    shutil.rmtree(tmp_path, ignore_errors=True)
