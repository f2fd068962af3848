#!/usr/bin/env python3
"""Interleaved A/B of library BUILDS in ONE process: every build is loaded side by side (each .so
registers its own code objects) and the rounds alternate between them on the same batches, so the
box's clock and thermal state are shared.

  python tools/ab_lib.py --spec "100b" jeromq_amd/libcz_base.so jeromq_amd/libcz_tail.so

Each build runs the bench workload (bench.Workload of the spec), is spot-checked against the
oracle first, then timed `steps` launches per round with HIP events.  Prints per-build median /
min kernel ms, payload GiB/s and the ratio to the first build.
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import bench  # noqa: E402
from ab_cfg import make  # noqa: E402
from jeromq_amd import _lib  # noqa: E402


def load(path):
    L = ctypes.CDLL(os.path.abspath(path))
    for name, (res, args) in _lib.SIGNATURES.items():
        if hasattr(L, name):
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
    return L


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--spec", action="append", default=None, help="bench config (+ layout flags); repeatable")
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--frames", type=int, default=bench.FRAMES)
    ap.add_argument("--no-verify", action="store_true", help="diagnostic builds (CZ_DIAG_*) write wrong bytes")
    ap.add_argument("--own-plan", action="store_true",
                    help="each build plans its own batch (segment order is the planner's: cz_plan_segments)")
    a = ap.parse_args()
    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    libs = [load(p) for p in a.libs]
    s = torch.cuda.current_stream()
    for spec in a.spec or ["4k"]:
        wls = []
        for L in (libs if a.own_plan else libs[:1]):
            _lib._LIB = L
            wls.append(make(spec, a.frames, dev))
        pick = (lambda k: wls[k]) if a.own_plan else (lambda k: wls[0])
        for k, L in enumerate(libs):
            _lib._LIB = L
            pick(k).step()
            if not a.no_verify:
                pick(k).verify_sample()
        for _ in range(10):
            for k, L in enumerate(libs):
                _lib._LIB = L
                pick(k).step()
        torch.cuda.synchronize()
        times = [[] for _ in libs]
        for _ in range(a.rounds):
            for k, L in enumerate(libs):
                _lib._LIB = L
                wl = pick(k)
                wl.step()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                for _ in range(a.steps):
                    wl.step()
                e1.record(s)
                torch.cuda.synchronize()
                times[k].append(e0.elapsed_time(e1) / a.steps)
        base = None
        for path, t in zip(a.libs, times):
            t = np.array(t)
            med = float(np.median(t))
            gib = wl.payload_bytes / (med * 1e-3) / 2**30
            base = base or gib
            print(f"{spec:32s} {os.path.basename(path):28s} median {med:.4f} ms  min {t.min():.4f} ms  "
                  f"{gib:8.1f} GiB/s  x{gib / base:.4f}", flush=True)
        del wl, wls
        torch.cuda.empty_cache()
    _lib._LIB = libs[0]


if __name__ == "__main__":
    main()
