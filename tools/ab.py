#!/usr/bin/env python3
"""Interleaved A/B of kernel variants in ONE process (cdna guide 5.4 rule 24).

  python tools/ab.py --config 4k --knob pair --values 1 0 --rounds 8 --steps 5

Each round times `steps` launches per variant with HIP events on the launch stream;
prints per-variant median / min ms and the derived GiB/s.  Parity of each variant is
spot-checked against the oracle before timing.
"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from jeromq_amd import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="4k")
    ap.add_argument("--knob", default="pair")
    ap.add_argument("--values", type=int, nargs="+", default=[1, 0])
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--frames", type=int, default=bench.FRAMES)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    wl = bench.Workload(a.config, a.frames, 0, torch.device("cuda:0"))
    lib = _lib.lib()
    times = {v: [] for v in a.values}
    for v in a.values:
        lib.cz_tune(a.knob.encode(), v)
        wl.step()
        wl.verify_sample()
    s = torch.cuda.current_stream()
    for _ in range(a.rounds):
        for v in a.values:
            lib.cz_tune(a.knob.encode(), v)
            wl.step()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(a.steps):
                wl.step()
            e1.record(s)
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1) / a.steps)
    for v in a.values:
        t = np.array(times[v])
        print(f"{a.config} {a.knob}={v}: median {np.median(t):.4f} ms  min {t.min():.4f} ms  "
              f"-> {wl.payload_bytes / (np.median(t) * 1e-3) / 2**30:.1f} GiB/s  "
              f"({(wl.read_bytes + wl.write_bytes) / (np.median(t) * 1e-3) / 1e9:.0f} GB/s alg)")


if __name__ == "__main__":
    main()
