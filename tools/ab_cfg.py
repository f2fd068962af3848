#!/usr/bin/env python3
"""Interleaved timing of several bench configs (or layouts) in ONE process on one GPU, so that
box-to-box clock differences cancel: every round times each workload back to back.

  python tools/ab_cfg.py --rounds 8 --steps 5 4k open4k "open4k --out-stride 4129"
  python tools/ab_cfg.py zipf_open "zipf_open --tune open_seg_carry=0"

A spec's `--tune key=value` (repeatable) sets that cz_tune knob around each of its steps and puts
it back after, so one library's paths can be A/B'd against each other.

Each spec is a bench.py config name plus optional bench layout flags.  Parity of every workload is
spot-checked against the oracle first (bench.Workload.verify_sample).  Prints per-spec median /
min kernel ms and payload GiB/s, and the ratio of every spec to the first.
"""
import argparse
import os
import shlex
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def make(spec, frames, dev):
    toks = shlex.split(spec)
    ap = argparse.ArgumentParser()
    ap.add_argument("config")
    ap.add_argument("--in-stride", type=int, default=0)
    ap.add_argument("--out-stride", type=int, default=0)
    ap.add_argument("--plain-stride", type=int, default=0)
    ap.add_argument("--in-align", type=int, default=64)
    ap.add_argument("--out-align", type=int, default=128)
    ap.add_argument("--seg-blocks", type=int, default=128)
    ap.add_argument("--fixed-len", type=int, default=0, help="zipf configs: every frame this long")
    ap.add_argument("--tune", action="append", default=[])
    a = ap.parse_args(toks)
    tune = [(k, int(v)) for k, v in (t.split("=") for t in a.tune)]
    with tuned(tune):
        wl = bench.Workload(a.config, frames, 0, dev, out_align=a.out_align, seg_blocks=a.seg_blocks,
                            in_align=a.in_align, plain_stride=a.plain_stride, in_stride=a.in_stride,
                            out_stride=a.out_stride, fixed_len=a.fixed_len)
    wl.tune = tune
    return wl


class tuned:
    def __init__(self, knobs):
        self.knobs, self.old = knobs, []

    def __enter__(self):
        from jeromq_amd import _lib
        for k, v in self.knobs:
            old = _lib.lib().cz_tune(k.encode(), v)
            if old < 0:
                raise SystemExit(f"cz_tune: unknown knob {k}")
            self.old.append((k, old))

    def __exit__(self, *exc):
        from jeromq_amd import _lib
        for k, v in reversed(self.old):
            _lib.lib().cz_tune(k.encode(), v)
        self.old = []


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("specs", nargs="+")
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--frames", type=int, default=bench.FRAMES)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    wls = []
    for sp in a.specs:
        wl = make(sp, a.frames, dev)
        with tuned(wl.tune):
            wl.step()
            wl.verify_sample()
        wls.append(wl)
    # ramp the clock out of idle
    for _ in range(20):
        for wl in wls:
            with tuned(wl.tune):
                wl.step()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    times = [[] for _ in wls]
    for _ in range(a.rounds):
        for k, wl in enumerate(wls):
            with tuned(wl.tune):
                wl.step()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                for _ in range(a.steps):
                    wl.step()
                e1.record(s)
                torch.cuda.synchronize()
            times[k].append(e0.elapsed_time(e1) / a.steps)
    base = None
    for sp, wl, t in zip(a.specs, wls, times):
        t = np.array(t)
        med = float(np.median(t))
        gib = wl.payload_bytes / (med * 1e-3) / 2**30
        base = base or gib
        print(f"{sp:40s} median {med:.4f} ms  min {t.min():.4f} ms  {gib:8.1f} GiB/s  "
              f"({(wl.read_bytes + wl.write_bytes) / (med * 1e-3) / 1e9:.0f} GB/s alg)  x{gib / base:.4f}", flush=True)


if __name__ == "__main__":
    main()
