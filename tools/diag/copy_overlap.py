"""Diagnostic: host<->device copy throughput by copy size, one direction at a time and both at once
(H2D and D2H on two streams), pinned host memory.  Explains why the host-staged pipeline
(cz_ctx_*_uniform, bench.py --config e2e4k --chunk-frames C) collapses below 32 MiB chunks.
  python tools/diag/copy_overlap.py   -> one JSON line per copy size"""
import json
import time

import torch


def main():
    dev = torch.device("cuda:0")
    total = 1 << 30
    s_in, s_out = torch.cuda.Stream(), torch.cuda.Stream()
    hin = torch.empty(total, dtype=torch.uint8).pin_memory()
    hout = torch.empty(total, dtype=torch.uint8).pin_memory()
    din = torch.empty(total, dtype=torch.uint8, device=dev)
    dout = torch.empty(total, dtype=torch.uint8, device=dev)
    for mib in (4, 8, 16, 24, 32, 64):
        size = mib << 20
        n = total // size

        def run(h2d, d2h):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(n):
                if h2d:
                    with torch.cuda.stream(s_in):
                        din[i * size:(i + 1) * size].copy_(hin[i * size:(i + 1) * size], non_blocking=True)
                if d2h:
                    with torch.cuda.stream(s_out):
                        hout[i * size:(i + 1) * size].copy_(dout[i * size:(i + 1) * size], non_blocking=True)
            torch.cuda.synchronize()
            return time.perf_counter() - t0

        run(True, True)
        r = {"copy_MiB": mib, "copies": n,
             "h2d_GBps": round(total / min(run(True, False) for _ in range(3)) / 1e9, 2),
             "d2h_GBps": round(total / min(run(False, True) for _ in range(3)) / 1e9, 2),
             "bidir_GBps_total": round(2 * total / min(run(True, True) for _ in range(3)) / 1e9, 2)}
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
