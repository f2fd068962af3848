"""Build libcurvezmq_mi355x.so in-tree for gfx950 with hipcc (no JIT cache, no torch extension).

The .so lands next to this file so it travels to the GPU box with the repo
snapshot and is what jeromq_amd._lib loads.
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.environ.get("CZ_LIB_OUT", os.path.join(HERE, "libcurvezmq_mi355x.so"))
SOURCES = ["cz_kernels.hip", "cz_x25519.hip", "cz_host.cpp", "cz_mechanism.cpp", "cz_wire.cpp", "cz_engine.cpp", "cz_handshake.cpp", "cz_curve_hs.cpp"]
HEADERS = ["cz_device.h", "cz_internal.h", "cz_salsa_lazy.h", os.path.join("..", "..", "include", "curvezmq_mi355x.h")]
ARCH = os.environ.get("CZ_OFFLOAD_ARCH", "gfx950")


def _stale():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(os.path.join(CSRC, f)) > t for f in SOURCES + HEADERS)


def build_library(force=False, verbose=True):
    if not force and not _stale():
        return LIB
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    extra = os.environ.get("CZ_EXTRA_FLAGS", "").split()  # A/B experiments only (e.g. -DCZ_SEAL_WAVES_PER_EU=5)
    cmd = [hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wall",
           "-o", LIB + ".tmp"] + extra + [os.path.join(CSRC, f) for f in SOURCES]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd, cwd=CSRC)
    os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    build_library(force="--force" in sys.argv)
    print(LIB)
