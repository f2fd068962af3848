"""Diagnostic: does the library's first HIP call succeed when torch's HIP runtime was initialized
between the library's load and that call?  One order per subprocess:
  python tools/diag/hip_init_order.py lib-torch-call | torch-lib-call | lib-count-call | lib-call | ...
("import": import torch only; "tensor": a torch op on the GPU; with no argument every order below runs
in its own process)"""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
LIB = os.path.join(ROOT, "jeromq_amd", "libcurvezmq_mi355x.so")


def run(order):
    steps = order.split("-")
    L = None
    for s in steps:
        if s == "lib":
            L = ctypes.CDLL(LIB)
        elif s == "torch":
            import torch
            print("torch.cuda.is_available", torch.cuda.is_available())
        elif s == "import":
            import torch  # noqa: F401  (torch's HIP runtime loaded, not initialized)
        elif s == "tensor":
            import torch
            print("torch tensor", float(torch.ones(4, device="cuda").sum().item()))
        elif s == "count":
            import torch
            print("torch.cuda.device_count", torch.cuda.device_count())
        elif s == "call":
            L.cz_last_error.restype = ctypes.c_char_p
            c = (ctypes.c_uint8 * 133)()
            m = (ctypes.c_uint8 * 133)()
            n = (ctypes.c_uint8 * 24)()
            k = (ctypes.c_uint8 * 32)(*range(32))
            rc = L.cz_box_afternm(c, m, ctypes.c_uint64(133), n, k)
            print(order, "rc", rc, L.cz_last_error().decode())


if __name__ == "__main__":
    if len(sys.argv) > 1:
        run(sys.argv[1])
    else:
        for order in ("lib-call", "lib-count-call", "torch-lib-call", "lib-torch-call", "lib-call-tensor-call",
                      "tensor-lib-call-tensor", "lib-tensor-call", "import-lib-torch-call", "import-lib-call-tensor-call"):
            r = subprocess.run([sys.executable, __file__, order], capture_output=True, text=True, timeout=120)
            print(order, "exit", r.returncode, r.stdout.strip().replace("\n", " | "), r.stderr.strip()[-300:])
