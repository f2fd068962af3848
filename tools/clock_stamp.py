"""The headline kernel's shader clock, stamped in-kernel and unprofiled.

  bash tools/build_variant.sh clock -DCZ_DIAG_CLOCK
  CZ_LIB=$PWD/jeromq_amd/libcz_clock.so python tools/clock_stamp.py [--ramp-s 3] [--launches 20]
      [--config 4k|4k_dense|4k_box|100b|open4k] [--plain-stride 4224]

The diagnostic build stamps s_memtime (shader clock counter) and s_memrealtime (constant 100 MHz
counter) per wave of k_seal_uniform when the wave starts and when it leaves (cz_kernels.hip,
CZ_DIAG_CLOCK).  After --ramp-s seconds of back-to-back launches of the 2^20 x 4 KiB seal (the MI355X
guide's DVFS give-back rule: the clock settles only after seconds of load), every measured launch
is timed with HIP events on its stream and its wave stamps are read back.  Per wave,
clock = d(memtime) / d(realtime) x 100 MHz; the realtime span of a whole launch against its HIP-event
time checks the 100 MHz.  VALU busy at that clock = VALU wave-instructions per launch (the committed
rocprofv3 count, profiles/pmc_traffic.json "4k") x 4 cycles / 1024 SIMDs / (clock x kernel time).
Prints one JSON line.  A measurement tool: no product path imports it."""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from jeromq_amd import _lib  # noqa: E402

RT_HZ = 100e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ramp-s", type=float, default=3.0)
    ap.add_argument("--launches", type=int, default=20)
    ap.add_argument("--frames", type=int, default=1 << 20)
    ap.add_argument("--config", default="4k", choices=["4k", "4k_dense", "4k_box", "100b", "open4k", "zipf"],
                    help="a bench config on k_seal_uniform, open4k on k_open_uniform, zipf on k_seal_segments_lines")
    ap.add_argument("--plain-stride", type=int, default=0, help="open4k: plaintext slot stride")
    a = ap.parse_args()
    if "CZ_LIB" not in os.environ:
        raise SystemExit("set CZ_LIB to a -DCZ_DIAG_CLOCK build (tools/build_variant.sh clock -DCZ_DIAG_CLOCK)")
    L = _lib.lib()
    if not hasattr(L, "cz_diag_clock_read"):
        raise SystemExit(f"{_lib.LIB_PATH} has no cz_diag_clock_read: not a -DCZ_DIAG_CLOCK build")
    read = {"open4k": L.cz_diag_clock_read_open, "zipf": L.cz_diag_clock_read_seg}.get(a.config, L.cz_diag_clock_read)
    read.restype = ctypes.c_int
    read.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
    dev = torch.device("cuda:0")
    torch.cuda.set_device(0)
    wl = bench.Workload(a.config, a.frames, 0, dev, plain_stride=a.plain_stride)
    # zipf: the lines kernel's waves over the segment list (the waves it leaves to the REST kernel
    # stamp a few cycles each and weigh nothing in the duration-weighted clock)
    waves = (wl.plan.nseg + 63) // 64 if a.config == "zipf" else (a.frames + 63) // 64
    s = torch.cuda.current_stream()
    t0 = time.perf_counter()
    ramp = 0
    while time.perf_counter() - t0 < a.ramp_s:
        for _ in range(8):
            wl.step()
        ramp += 8
        torch.cuda.synchronize()
    ramp_s = time.perf_counter() - t0
    wl.verify_sample()  # the stamps do not change a byte
    buf = np.zeros(waves * 4, dtype=np.uint64)
    rows = []
    for _ in range(a.launches):
        ea, eb = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ea.record(s)
        wl.step()
        eb.record(s)
        torch.cuda.synchronize()
        n = read(buf.ctypes.data, waves)
        assert n == waves, n
        st = buf.reshape(waves, 4).astype(np.float64)
        dt, dr = st[:, 2] - st[:, 0], st[:, 3] - st[:, 1]
        ok = dr > 0
        clk = dt[ok] / dr[ok] * RT_HZ / 1e9
        kern_s = ea.elapsed_time(eb) / 1e3
        span_rt = (st[:, 3].max() - st[:, 1].min())
        rows.append({"kernel_ms": kern_s * 1e3, "clock_ghz_median": float(np.median(clk)),
                     "clock_ghz_weighted": float(dt[ok].sum() / dr[ok].sum() * RT_HZ / 1e9),
                     "clock_ghz_p10": float(np.percentile(clk, 10)), "clock_ghz_p90": float(np.percentile(clk, 90)),
                     "realtime_hz_check": span_rt / kern_s,
                     "wave_us_median": float(np.median(dr[ok])) / RT_HZ * 1e6,
                     "resident_waves_mean": float(dr[ok].sum() / span_rt)})
        for _ in range(4):   # queued ahead of the next measured launch: it starts with no idle gap
            wl.step()
    pmc = bench.load_pmc(a.config)
    valu = pmc.get("valu_insts_per_launch")
    # per-wave median for the uniform kernels (every wave alike); duration-weighted for the segment
    # kernel, whose early-exit waves would otherwise count as much as a 128-block segment
    clk_key = "clock_ghz_weighted" if a.config == "zipf" else "clock_ghz_median"
    clk = statistics.median(r[clk_key] for r in rows)
    kms = statistics.median(r["kernel_ms"] for r in rows)
    kern = {"open4k": "k_open_uniform", "zipf": "k_seal_segments_lines (+ REST and combine launches in the timed step)"}.get(
        a.config, "k_seal_uniform")
    res = {"what": f"{kern} (bench config {a.config}" + (f", {a.plain_stride}-byte plaintext slots" if a.plain_stride else "")
           + f", {a.frames} frames), per-wave s_memtime / s_memrealtime stamps, unprofiled",
           "lib": os.path.basename(_lib.LIB_PATH), "ramp_launches": ramp, "ramp_s": round(ramp_s, 2),
           "launches": len(rows), "kernel_ms_median": round(kms, 4),
           "clock_ghz_median": round(statistics.median(r["clock_ghz_median"] for r in rows), 4),
           "clock_ghz_weighted": round(statistics.median(r["clock_ghz_weighted"] for r in rows), 4),
           "clock_used": clk_key,
           "clock_ghz_p10_median": round(statistics.median(r["clock_ghz_p10"] for r in rows), 4),
           "clock_ghz_p90_median": round(statistics.median(r["clock_ghz_p90"] for r in rows), 4),
           "realtime_hz_check_median": round(statistics.median(r["realtime_hz_check"] for r in rows), 0),
           "wave_us_median": round(statistics.median(r["wave_us_median"] for r in rows), 2),
           "resident_waves_mean": round(statistics.median(r["resident_waves_mean"] for r in rows), 1),
           "valu_insts_per_launch": valu, "valu_source": pmc.get("valu_source")}
    if valu:
        res["valu_frac_at_clock"] = round(valu * 4 / 1024 / (clk * 1e9) / (kms / 1e3), 4)
        res["valu_frac_at_2.4GHz"] = round(valu * 4 / 1024 / 2.4e9 / (kms / 1e3), 4)
    res["per_launch"] = [{k: round(v, 4) for k, v in r.items()} for r in rows]
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
