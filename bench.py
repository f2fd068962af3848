#!/usr/bin/env python3
"""CURVE encrypt+MAC throughput on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1]): 2^20 x 4 KiB CurveZMQ MESSAGE frames,
device-resident, sealed per step by one launch of the gfx950 seal kernel
(Mechanism.encode for every frame: XSalsa20 XOR + Poly1305 tag + MESSAGE
framing, CurveClientMechanism.java:126-163).  One connection direction (C->S,
the RFC test keys of org/zeromq/ZMQ.java:4603-4624), counters 3.., every 8th
frame MORE.  Payload bytes: counter-based SplitMix64, generated on device.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config 4k|100b|zipf|zipf_lane|open4k|e2e4k]

N > 1 (torch.distributed.run, one rank per GPU): every rank seals its own 2^20
frames (counters offset by rank * 2^20): no collective on the timed path ("weak"); barriers and
the max-over-ranks timing run on a gloo control group.  Rank 0 prints ONE JSON line.  `value` =
payload GiB/s over all ranks.  The 4k line also carries `seal_open_verify` (configs[4]: seal, then
open + tag-verify of the same frames, timed apart from `value`).  At N > 1 the RCCL scatter ->
seal -> gather leg runs AFTER that line is out, under a watchdog; rank 0 prints its result on a
`SCATTER_GATHER {...}` line (not a JSON line), which `python bench.py --gpus N` merges into the
line it relays.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from jeromq_amd import _lib, batch  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s)
PRECOM = bytes.fromhex("0e8790cb0dc8703af2533cc8594eecfbf62ca560a66ebee1259cc0a30435c6f3")  # beforenm(RFC keys)
FRAMES = 1 << 20


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--ramp-ms", type=float, default=150.0,
                    help="untimed launches before the W warmup steps until this much GPU time has passed: "
                         "the clock needs ~100 ms of load to leave its idle state")
    ap.add_argument("--seg-blocks", type=int, default=128, help="zipf: segment length in 64-byte blocks")
    ap.add_argument("--in-align", type=int, default=64,
                    help="zipf: input payload slot alignment in bytes (lengths are 64-byte multiples)")
    ap.add_argument("--out-align", type=int, default=128,
                    help="zipf: output slot alignment in bytes (the caller's packing choice)")
    ap.add_argument("--in-stride", type=int, default=0,
                    help="4k/100b/open4k: payload slot stride in bytes (0 = the payload size rounded to 16)")
    ap.add_argument("--out-stride", type=int, default=0,
                    help="4k/100b/open4k: body slot stride in bytes (0 = the config's own layout)")
    ap.add_argument("--plain-stride", type=int, default=0,
                    help="open4k: plaintext slot stride in bytes (0 = the payload stride, 4096)")
    ap.add_argument("--config", default="4k", choices=["4k", "4k_dense", "4k_box", "100b", "zipf", "zipf_open", "zipf_lane", "open4k", "e2e4k",
                                                          "engine", "nacl", "beforenm", "jni"])
    ap.add_argument("--frames", type=int, default=FRAMES)
    ap.add_argument("--chunk-frames", type=int, default=16384, help="e2e4k: frames per pipeline chunk")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-scatter", action="store_true",
                    help="N>1, 4k: skip the separately timed RCCL scatter -> seal -> gather leg")
    ap.add_argument("--leg-deadline", type=float, default=LEG_DEADLINE_S,
                    help="N>1: seconds the scatter/gather leg may take after the main line before the ranks exit")
    ap.add_argument("--no-verify", action="store_true",
                    help="skip the parity spot check (diagnostic builds with CZ_DIAG_* only)")
    ap.add_argument("--no-roundtrip", action="store_true",
                    help="4k: skip the separately timed seal -> open+verify leg (BASELINE.json configs[4])")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU-baseline sample duration")
    return ap.parse_args()


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


# The N > 1 ranks print the weak-scaling line first (one JSON line, everything `value` needs), then
# run the separately timed RCCL scatter -> seal -> gather leg, whose result rank 0 prints on a line
# of its own behind this tag: not a JSON line, so a reader that takes the lines starting with "{"
# still sees exactly one, and a hang or error in the leg cannot cost the scaling line.
SG_TAG = "SCATTER_GATHER "
LEG_DEADLINE_S = 240.0       # ranks: the leg's own watchdog (then the ranks exit 0, line already out)
LAUNCH_LEG_DEADLINE_S = 300.0  # launcher: after the main line, the wait for the leg before it kills the ranks


def _kill_group(p):
    """End the child torch.distributed.run and its ranks: the process group started for it
    (start_new_session), never a pattern.  SIGTERM, then SIGKILL after 10 s."""
    import signal
    try:
        pg = os.getpgid(p.pid)
    except (ProcessLookupError, AttributeError):
        return
    for sig, wait_s in ((signal.SIGTERM, 10.0), (signal.SIGKILL, 10.0)):
        try:
            os.killpg(pg, sig)
        except ProcessLookupError:
            return
        try:
            p.wait(timeout=wait_s)
            return
        except Exception:  # subprocess.TimeoutExpired
            pass


def launch_ranks(gpus, argv, popen=None, cmd=None, kill=None, leg_deadline_s=LAUNCH_LEG_DEADLINE_S):
    """`python bench.py --gpus N` with N > 1 and no launcher around it: start the N ranks as a CHILD
    `torch.distributed.run` (one process per GPU, rendezvous on 127.0.0.1, its own session so the
    ranks can be ended as one process group), relay rank 0's JSON line and return an exit status.
    This process never touches the GPU (torch.cuda stays uninitialised, the library is not loaded)
    and never execs: the ranks are its children.

    The main line is checked before it is relayed: exactly one JSON line, n_gpus == N, one per_rank
    entry per rank, the slowest-rank roofline and the CPU baseline; anything else is an error (the
    child's exit status, or 1), so a run that silently timed fewer GPUs cannot pass.  After the main
    line the ranks run the RCCL scatter/gather leg: its SG_TAG line is merged into the relayed line
    as "scatter_gather".  If the leg has not reported within leg_deadline_s of the main line, the
    child's process group is killed and the main line goes out with scatter_gather = {"error": ...};
    an error the leg reports, or a non-zero exit after a good main line, is recorded the same way.
    popen / cmd / kill: stand-ins for tests."""
    import queue
    import subprocess
    import threading
    if cmd is None:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC: RCCL needs it on this pool
    print("launching: " + " ".join(cmd), file=sys.stderr, flush=True)
    p = (popen or subprocess.Popen)(cmd, stdout=subprocess.PIPE, text=True, env=env, cwd=ROOT,
                                    start_new_session=True)
    kill = kill or _kill_group
    q = queue.Queue()

    def reader():
        for ln in p.stdout:
            q.put(ln)
        q.put(None)
    threading.Thread(target=reader, daemon=True).start()
    lines, sg, eof, deadline = [], None, False, None
    while not eof:
        timeout = None if deadline is None else max(deadline - time.monotonic(), 0.0)
        try:
            ln = q.get(timeout=timeout)
        except queue.Empty:
            break                       # the leg's deadline passed
        if ln is None:
            eof = True
        elif ln.startswith("{"):        # ranks' other stdout goes to stderr; the JSON line is held for the check
            lines.append(ln.strip())
            if deadline is None:
                deadline = time.monotonic() + leg_deadline_s
        elif ln.startswith(SG_TAG):
            try:
                sg = json.loads(ln[len(SG_TAG):])
            except ValueError:
                sg = {"error": "unparsable leg line: " + ln.strip()[:200]}
        else:
            sys.stderr.write(ln)
            sys.stderr.flush()
    killed = False
    if not eof:
        print(f"ranks still running {leg_deadline_s:.0f} s after the main line: killing their process group",
              file=sys.stderr, flush=True)
        kill(p)
        killed = True
    rc = p.wait()
    assert not torch.cuda.is_initialized(), "launcher process initialised the GPU"
    if len(lines) != 1:
        print(f"expected one JSON line from rank 0, got {len(lines)} (ranks exit {rc})", file=sys.stderr)
        return rc if rc and not killed else 1
    line = json.loads(lines[0])
    per = line.get("per_rank") or []
    if line.get("n_gpus") != gpus or len(per) != gpus or sorted(r["rank"] for r in per) != list(range(gpus)):
        print(f"rank line does not cover {gpus} GPUs: n_gpus={line.get('n_gpus')}, per_rank={len(per)}",
              file=sys.stderr)
        return 1
    # an N > 1 line is as self-describing as the N = 1 line: the roofline from the slowest rank's
    # kernel time (with the per-rank spread) and the CPU baseline
    roof = line.get("roofline") or {}
    missing = [k for k in ("achieved", "frac", "frac_min", "frac_max", "kernel_ms_max") if roof.get(k) is None]
    if "--no-cpu-baseline" not in argv and not line.get("cpu_baseline"):
        missing.append("cpu_baseline")
    if line.get("value") is not None and missing:
        print(f"rank line lacks {missing}", file=sys.stderr)
        return 1
    pending = isinstance(line.get("scatter_gather"), dict) and line["scatter_gather"].get("pending")
    if sg is not None:
        line["scatter_gather"] = sg
    elif killed:
        line["scatter_gather"] = {"error": f"timeout: no result {leg_deadline_s:.0f} s after the main line; "
                                           "ranks killed by the launcher"}
    elif pending:
        line["scatter_gather"] = {"error": f"ranks exited (status {rc}) without reporting the leg"}
    if rc != 0:
        line["ranks_exit_status"] = rc   # after a good main line: recorded, not fatal
    line["launcher"] = "bench.py --gpus: child torch.distributed.run"
    print(json.dumps(line), flush=True)
    return 0


def multi_rank_roofline(kernel_s, alg_bytes):
    """The N > 1 line's roofline: `achieved` / `frac` / `kernel_ms` from the SLOWEST rank's average
    kernel time (the one that sets the job's time), with the fastest and slowest ranks' fractions
    beside it.  kernel_s: every rank's average kernel time in seconds."""
    slow, fast = max(kernel_s), min(kernel_s)
    achieved = alg_bytes / slow / 1e9
    return {"achieved": round(achieved, 2), "frac": round(achieved / HBM_PEAK_GBS, 4),
            "kernel_ms": round(slow * 1e3, 4), "kernel_ms_min": round(fast * 1e3, 4),
            "kernel_ms_max": round(slow * 1e3, 4),
            "frac_min": round(alg_bytes / slow / 1e9 / HBM_PEAK_GBS, 4),
            "frac_max": round(alg_bytes / fast / 1e9 / HBM_PEAK_GBS, 4),
            "kernel_time_from": "slowest rank (per-rank figures in per_rank)"}


def setup_dist(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
    ndev = torch.cuda.device_count()
    # "nccl" is RCCL on ROCm; CZ_DIST_BACKEND=gloo rehearses N ranks on fewer GPUs (tests only)
    backend = os.environ.get("CZ_DIST_BACKEND", "nccl") if world > 1 else None
    if world > 1 and ndev < world and backend == "nccl":
        raise SystemExit(f"{world} ranks need {world} GPUs for RCCL, {ndev} visible "
                         "(CZ_DIST_BACKEND=gloo rehearses N ranks on one GPU)")
    if ndev and local >= ndev:  # gloo rehearsal of N ranks on fewer GPUs; identity on a full node
        local %= ndev
    global DATA_BACKEND
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        # The default group is the CONTROL plane: barriers, the max-over-ranks timing and the per-rank
        # figures, all host scalars, on gloo.  The timed path has no collective (frames are
        # independent), so the weak-scaling line never depends on RCCL.  RCCL ("nccl", over xGMI)
        # carries the data of the scatter/gather leg only, in a group of its own made after the
        # line is out (data_group).
        dist.init_process_group("gloo")
        assert dist.get_world_size() == world
        DATA_BACKEND = backend
    else:
        torch.cuda.set_device(0)
    return world, rank, local


DATA_BACKEND = None  # N > 1: the scatter/gather leg's backend ("nccl" = RCCL; "gloo" in rehearsals)


def data_group():
    """The scatter/gather leg's process group: a new RCCL group (collective: every rank calls it),
    or the default gloo group in a gloo rehearsal (CZ_DIST_BACKEND=gloo)."""
    import torch.distributed as dist
    if DATA_BACKEND == "nccl":
        return dist.new_group(backend="nccl")
    return None


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def _reduce(world, x, op):
    if world == 1:
        return x
    import torch.distributed as dist
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=op)
    return float(t.item())


def max_over_ranks(world, x):
    """slowest rank's time (the contract's max over ranks)"""
    import torch.distributed as dist
    return _reduce(world, x, dist.ReduceOp.MAX if world > 1 else None)


def sum_over_ranks(world, x):
    import torch.distributed as dist
    return _reduce(world, x, dist.ReduceOp.SUM if world > 1 else None)


def shard_plan(rank, frames_per_rank, cfg="4k"):
    """Rank r seals frames [r*F, (r+1)*F) of the global batch: nonce counters 3 + r*F ..,
    its own payload seed.  Frames are independent, so no data crosses ranks (weak scaling)."""
    counter0 = 3 + rank * frames_per_rank
    seed = 0x5EED0000 + {"4k": 1, "4k_dense": 1, "4k_box": 1, "100b": 2, "zipf": 3, "zipf_open": 3, "zipf_lane": 3, "open4k": 4}[cfg] + 1000 * rank
    return counter0, seed


class Workload:
    """Builds one rank's device-resident batch and the per-step launch."""

    def __init__(self, cfg, frames, rank, dev, out_align=128, seg_blocks=128, in_align=64, plain_stride=0,
                 in_stride=0, out_stride=0, fixed_len=0):
        self.cfg = cfg
        self.dev = dev
        key = torch.tensor(list(PRECOM), dtype=torch.uint8, device=dev).view(1, 32)
        self.subkey = batch.subkeys(key, _lib.CZ_DIR_C2S)[0].contiguous()
        self.counter0, seed = shard_plan(rank, frames, cfg)
        self.count = frames
        if cfg == "4k_box":
            # the reference's own box layout as input (CurveClientMechanism.java:144-153): slot i =
            # 0^32 || flags || payload, 4224-byte slots in and out
            n = 4096
            self.n = n
            self.in_stride = self.out_stride = 4224
            self.d_in = torch.empty(frames * self.in_stride, dtype=torch.uint8, device=dev)
            batch.fill(self.d_in, seed)
            box = self.d_in.view(frames, self.in_stride)
            box[:, :32] = 0
            box[:, 32] = 0
            box[::8, 32] = 1
            self.d_out = torch.empty(frames * self.out_stride, dtype=torch.uint8, device=dev)
            self.payload_bytes = frames * n
            self.read_bytes = frames * (n + 1)   # flags byte + payload (box bytes 0..31 are not read)
            self.write_bytes = frames * (n + 33)
        elif cfg in ("4k", "4k_dense", "100b", "open4k"):
            n = 4096 if cfg != "100b" else 100
            self.n = n
            self.in_stride = (n + 15) // 16 * 16
            # 4 KiB: 128-byte body slots (full-line LDS-staged stores); 100 B: dense 16-byte slots
            # (64 slots fit the LDS region stager)
            self.out_stride = (n + 33 + 127) // 128 * 128 if n >= 1024 else (n + 33 + 15) // 16 * 16
            if cfg == "4k_dense":  # bodies back to back (4129-byte slots), as the wire packs them
                self.out_stride = n + 33
            if in_stride:
                assert in_stride >= n, "--in-stride below the payload size"
                self.in_stride = in_stride
            if out_stride:
                assert out_stride >= n + 33, "--out-stride below the body size"
                self.out_stride = out_stride
            self.d_in = torch.empty(frames * self.in_stride, dtype=torch.uint8, device=dev)
            batch.fill(self.d_in, seed)
            self.flags = torch.zeros(frames, dtype=torch.uint8, device=dev)
            self.flags[::8] = 1
            self.d_out = torch.empty(frames * self.out_stride, dtype=torch.uint8, device=dev)
            self.payload_bytes = frames * n
            # algorithmic bytes per launch: read payload + flag byte, write 33+n body
            self.read_bytes = frames * (n + 1)
            self.write_bytes = frames * (n + 33)
            if cfg == "open4k":
                batch.seal_uniform(self.d_in, self.in_stride, self.d_out, self.out_stride, frames, n, self.subkey,
                                   self.counter0, flags8=self.flags)
                # plaintext slots: the payload stride unless the caller pads them (--plain-stride)
                self.plain_stride = plain_stride or self.in_stride
                self.d_plain = torch.empty(frames * self.plain_stride, dtype=torch.uint8, device=dev)
                self.status = torch.empty(frames, dtype=torch.int16, device=dev)
                # open reads the body + writes payload + 2-byte status (+8 B prev nonce, L2-resident)
                self.read_bytes = frames * (n + 33)
                self.write_bytes = frames * (n + 2)
        else:  # zipf: lengths 64*j, j ~ Zipf(1.2) on 1..1024, seed 42
            rng = np.random.default_rng(42 + rank)
            j = np.empty(0, dtype=np.int64)
            while len(j) < frames:
                z = rng.zipf(1.2, size=frames)
                j = np.concatenate([j, z[z <= 1024]])
            lens = (64 * j[:frames]).astype(np.uint64)
            if fixed_len:  # diagnostic (tools/ab_cfg.py --fixed-len): the segment path on uniform frames
                lens[:] = fixed_len
            desc = np.zeros(frames, dtype=batch.DESC_DTYPE)
            ia = np.uint64(in_align)
            in_len = (lens + ia - np.uint64(1)) // ia * ia
            in_off = np.zeros(frames, dtype=np.uint64)
            in_off[1:] = np.cumsum(in_len[:-1])
            al = np.uint64(out_align)
            out_len = (lens + np.uint64(33) + al - np.uint64(1)) // al * al
            out_off = np.zeros(frames, dtype=np.uint64)
            out_off[1:] = np.cumsum(out_len[:-1])
            desc["in_off"] = in_off
            desc["out_off"] = out_off
            desc["len"] = lens
            desc["counter"] = self.counter0 + np.arange(frames, dtype=np.uint64)
            desc["flags"] = (np.arange(frames) % 8 == 0).astype(np.uint32)
            desc["prev"] = -1
            self.desc_np = desc
            in_bytes = int(in_len.sum())
            out_bytes = int(out_len.sum())
            self.d_in = torch.empty(in_bytes, dtype=torch.uint8, device=dev)
            batch.fill(self.d_in, seed)
            self.d_out = torch.empty(out_bytes, dtype=torch.uint8, device=dev)
            self.d_desc = torch.from_numpy(desc.view(np.uint8)).to(dev)
            pay = int(lens.sum())
            self.payload_bytes = pay
            if cfg in ("zipf", "zipf_open"):
                # long frames split into 64-block segments (one lane each) + Poly1305 combine
                self.plan = batch.SegmentPlan(desc, open_=False, seg_blocks=seg_blocks).to(dev)
                self.read_bytes = pay + 40 * frames + 16 * self.plan.nseg + 16 * self.plan.ncomb
                if cfg == "zipf_open":
                    # the receive side of the same batch: the sealed bodies at the output offset table
                    # opened (tag check, replay floor, flags) into plaintext at the payload offsets
                    batch.seal_segments(self.d_desc, self.plan, self.d_in, self.d_out, self.subkey.view(1, 32))
                    odesc = desc.copy()
                    odesc["in_off"], odesc["out_off"] = desc["out_off"], desc["in_off"]
                    odesc["len"] = desc["len"] + np.uint64(33)
                    odesc["counter"] = desc["counter"] - np.uint64(1)
                    odesc["flags"] = 0x100  # CZ_DESC_CHECK_NONCE
                    self.d_odesc = torch.from_numpy(odesc.view(np.uint8).copy()).to(dev)
                    self.oplan = batch.SegmentPlan(odesc, open_=True, seg_blocks=seg_blocks).to(dev)
                    self.d_plain = torch.empty_like(self.d_in)
                    self.status = torch.empty(frames, dtype=torch.int16, device=dev)
                    self.read_bytes = pay + 33 * frames + 40 * frames + 16 * self.oplan.nseg + 16 * self.oplan.ncomb
                    self.write_bytes = pay + 2 * frames
            else:  # zipf_lane: one lane per frame, longest first
                order = batch.plan_order(desc)
                self.d_order = torch.from_numpy(order.view(np.int32)).to(dev)
                self.read_bytes = pay + 40 * frames + 4 * frames
            if cfg != "zipf_open":
                self.write_bytes = int((lens + np.uint64(33)).sum())
            self.n = None
        torch.cuda.synchronize()

    def step(self):
        if self.cfg == "4k_box":
            batch.seal_uniform_box(self.d_in, self.in_stride, self.d_out, self.out_stride, self.count, self.n,
                                   self.subkey, self.counter0)
        elif self.cfg in ("4k", "4k_dense", "100b"):
            batch.seal_uniform(self.d_in, self.in_stride, self.d_out, self.out_stride, self.count, self.n,
                               self.subkey, self.counter0, flags8=self.flags)
        elif self.cfg == "open4k":
            batch.open_uniform(self.d_out, self.out_stride, self.d_plain, self.plain_stride, self.count, self.n + 33,
                               self.subkey, self.counter0 - 1, self.status)
        elif self.cfg == "zipf":
            batch.seal_segments(self.d_desc, self.plan, self.d_in, self.d_out, self.subkey.view(1, 32))
        elif self.cfg == "zipf_open":
            batch.open_segments(self.d_odesc, self.oplan, self.d_out, self.d_plain, self.subkey.view(1, 32),
                                self.status)
        else:
            batch.seal_batch(self.d_desc, self.count, self.d_in, self.d_out, self.subkey.view(1, 32),
                             order=self.d_order)

    def verify_sample(self):
        """Bit-exact spot check of a few frames against the CPU oracle (test infrastructure)."""
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from cz_testlib import or_curve_encode
        torch.cuda.synchronize()
        if self.cfg in ("4k", "4k_dense", "100b", "4k_box"):
            skip = 33 if self.cfg == "4k_box" else 0
            for i in (0, 1, 7, self.count // 2, self.count - 2, self.count - 1):
                p = self.d_in[i * self.in_stride + skip:i * self.in_stride + skip + self.n].cpu().numpy().tobytes()
                body = self.d_out[i * self.out_stride:i * self.out_stride + self.n + 33].cpu().numpy().tobytes()
                fl = 1 if i % 8 == 0 else 0
                if body != or_curve_encode(p, fl, self.counter0 + i, 0, PRECOM):
                    raise SystemExit(f"parity failure at frame {i}")
        elif self.cfg == "zipf_open":
            st = self.status.cpu().numpy().view(np.uint16)
            if np.any(st & 0xff) or not np.array_equal(st >> 8, self.desc_np["flags"].astype(np.uint16)):
                raise SystemExit("open failures in benchmark batch")
            if not torch.equal(self.d_plain, self.d_in):  # payload lengths are 64-byte multiples: no padding
                raise SystemExit("open round trip mismatch")
        elif self.cfg == "open4k":
            st = self.status.cpu().numpy().view(np.uint16)
            if np.any(st & 0xff):
                raise SystemExit("open failures in benchmark batch")
            got = self.d_plain.view(self.count, self.plain_stride)[:, :self.n]
            if not torch.equal(got, self.d_in.view(self.count, self.in_stride)[:, :self.n]):
                raise SystemExit("open round trip mismatch")
        else:
            longest = int(np.argmax(self.desc_np["len"]))
            for i in (0, 1, longest, self.count - 1):
                d = self.desc_np[i]
                p = self.d_in[int(d["in_off"]):int(d["in_off"]) + int(d["len"])].cpu().numpy().tobytes()
                body = self.d_out[int(d["out_off"]):int(d["out_off"]) + int(d["len"]) + 33].cpu().numpy().tobytes()
                if body != or_curve_encode(p, int(d["flags"]), int(d["counter"]), 0, PRECOM):
                    raise SystemExit(f"parity failure at frame {i}")


def cpu_baseline(wl, target_s):
    """The oracle (oracle/curve_oracle.c, a scalar C restatement of the NaCl path) timed on the
    host: 1 thread, a bounded sample of the same frames.  Reported, not the target."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from cz_testlib import oracle
    lib = oracle()
    n = wl.n if wl.n else 4096
    stride = (n + 15) // 16 * 16
    ostride = (n + 33 + 15) // 16 * 16

    def run(count, threads=1):
        hin = np.frombuffer(np.random.default_rng(1).bytes(count * stride), dtype=np.uint8).copy()
        hout = np.zeros(count * ostride, dtype=np.uint8)
        desc = np.zeros(count, dtype=batch.DESC_DTYPE)
        desc["in_off"] = np.arange(count, dtype=np.uint64) * stride
        desc["out_off"] = np.arange(count, dtype=np.uint64) * ostride
        desc["len"] = n
        desc["counter"] = 3 + np.arange(count, dtype=np.uint64)
        precom = np.frombuffer(PRECOM, dtype=np.uint8).copy()
        t0 = time.perf_counter()
        lib.or_seal_batch(desc.ctypes.data, count, hin.ctypes.data, hout.ctypes.data, precom.ctypes.data, 0, threads)
        return time.perf_counter() - t0

    probe = 256 if n > 1000 else 8192
    dt = run(probe)
    count = int(max(probe, min(probe * target_s / max(dt, 1e-6), 4_000_000)))
    dt = run(count)
    gibs = count * n / dt / 2**30
    # the GPU box's CPU share is 16 cores: the same sample on 16 threads, reported beside it
    dt16 = run(count, 16)
    res = {"value": round(gibs, 4), "unit": "GiB/s", "cores": 1, "kind": "port",
           "value_16_threads": round(count * n / dt16 / 2**30, 4),
           "sample": f"{count} x {n} B frames sealed by oracle/curve_oracle.c (1 thread, {dt:.1f} s), "
                     f"{os.cpu_count()} logical CPUs visible"}
    # an optimised CPU NaCl beside the scalar port: libsodium's crypto_box_afternm of the same
    # box length (0^32 || flags || payload), 1 thread, ~2 s
    sod = _libsodium()
    if sod is not None:
        mlen = n + 33
        m = ctypes.create_string_buffer(mlen)
        c = ctypes.create_string_buffer(mlen)
        nonce = ctypes.create_string_buffer(b"CurveZMQMESSAGEC" + (3).to_bytes(8, "big"), 24)
        k = ctypes.create_string_buffer(PRECOM, 32)
        reps, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < 2.0:
            for _ in range(64):
                sod.crypto_box_afternm(c, m, ctypes.c_ulonglong(mlen), nonce, k)
            reps += 64
        res["libsodium_1core_GiBps"] = round(reps * n / (time.perf_counter() - t0) / 2**30, 4)
    return res


def copy_ceiling(dev, nbytes=1 << 30, chunk=64 << 20, reps=5):
    """PCIe copy ceilings the host-resident lines sit under: pinned H2D alone, D2H alone, and both
    at once (full duplex), nbytes per direction in `chunk`-byte hipMemcpyAsync calls, each
    direction on its own stream (as the 3-stream pipelines issue them).  Median GB/s."""
    hip = ctypes.CDLL("libamdhip64.so")
    vp, sz = ctypes.c_void_p, ctypes.c_size_t
    hip.hipMemcpyAsync.argtypes = [vp, vp, sz, ctypes.c_int, vp]
    hip.hipStreamSynchronize.argtypes = [vp]
    hip.hipHostFree.argtypes = [vp]
    hip.hipFree.argtypes = [vp]
    hip.hipSetDevice(dev.index or 0)
    bufs = [vp() for _ in range(4)]
    for b in bufs[:2]:
        assert hip.hipHostMalloc(ctypes.byref(b), sz(nbytes), 0) == 0, "hipHostMalloc"
    for b in bufs[2:]:
        assert hip.hipMalloc(ctypes.byref(b), sz(nbytes)) == 0, "hipMalloc"
    h_src, h_dst, d_a, d_b = (b.value for b in bufs)
    sa, sb = vp(), vp()
    hip.hipStreamCreateWithFlags(ctypes.byref(sa), 1)
    hip.hipStreamCreateWithFlags(ctypes.byref(sb), 1)

    def timed(h2d, d2h):
        ts = []
        for _ in range(reps + 1):
            t0 = time.perf_counter()
            for off in range(0, nbytes, chunk):
                if h2d:
                    assert hip.hipMemcpyAsync(d_a + off, h_src + off, chunk, 1, sa) == 0
                if d2h:
                    assert hip.hipMemcpyAsync(h_dst + off, d_b + off, chunk, 2, sb) == 0
            hip.hipStreamSynchronize(sa)
            hip.hipStreamSynchronize(sb)
            ts.append(time.perf_counter() - t0)
        return float(np.median(ts[1:]))
    t_h, t_d, t_b = timed(True, False), timed(False, True), timed(True, True)
    hip.hipStreamDestroy(sa)
    hip.hipStreamDestroy(sb)
    for b in bufs[:2]:
        hip.hipHostFree(b)
    for b in bufs[2:]:
        hip.hipFree(b)
    return {"h2d_GBps": round(nbytes / t_h / 1e9, 2), "d2h_GBps": round(nbytes / t_d / 1e9, 2),
            "bidir_GBps_total": round(2 * nbytes / t_b / 1e9, 2), "bytes_per_direction": nbytes,
            "method": f"hipMemcpyAsync of pinned buffers in {chunk >> 20} MiB calls, one stream per direction, "
                      f"median of {reps}"}


def e2e_host(args, dev):
    """End-to-end from pinned host memory (the JNI path): H2D + seal + D2H pipelined over 3
    streams by cz_ctx_seal_uniform, then the reverse open.  Wall clock, payload GiB/s."""
    import ctypes
    lib = _lib.lib()
    frames = min(args.frames, 1 << 18)
    n = 4096
    in_stride, out_stride = 4096, 4224
    pin = lib.cz_host_alloc(frames * in_stride)
    pout = lib.cz_host_alloc(frames * out_stride)
    pback = lib.cz_host_alloc(frames * in_stride)
    pstat = lib.cz_host_alloc(2 * frames)
    if not (pin and pout and pback and pstat):
        raise SystemExit("cz_host_alloc failed: " + _lib.last_error())
    hin = np.ctypeslib.as_array((ctypes.c_uint8 * (frames * in_stride)).from_address(pin))
    hin[:] = np.frombuffer(np.random.default_rng(7).bytes(frames * in_stride), dtype=np.uint8)
    ctx = ctypes.c_void_p()
    _lib.check(lib.cz_ctx_create(ctypes.byref(ctx), dev.index or 0), "cz_ctx_create")
    _lib.check(lib.cz_ctx_set_keys(ctx, PRECOM, 1, _lib.CZ_DIR_C2S), "cz_ctx_set_keys")
    chunk = args.chunk_frames
    res = {}
    for name, fn in (("seal", lambda: lib.cz_ctx_seal_uniform(ctx, frames, n, pin, in_stride, pout, out_stride, 3,
                                                               None, chunk)),
                     ("open", lambda: lib.cz_ctx_open_uniform(ctx, frames, n + 33, pout, out_stride, pback, in_stride,
                                                               2, 1, pstat, chunk))):
        _lib.check(fn(), name)  # warm-up (allocates the per-stream buffers)
        ts = []
        for _ in range(max(args.steps // 4, 3)):
            t0 = time.perf_counter()
            _lib.check(fn(), name)
            ts.append(time.perf_counter() - t0)
        res[name] = float(np.median(ts))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from cz_testlib import or_curve_encode
    hout = np.ctypeslib.as_array((ctypes.c_uint8 * (frames * out_stride)).from_address(pout))
    for i in (0, frames - 1):
        body = hout[i * out_stride:i * out_stride + n + 33].tobytes()
        if body != or_curve_encode(hin[i * in_stride:i * in_stride + n].tobytes(), 0, 3 + i, 0, PRECOM):
            raise SystemExit(f"e2e parity failure at frame {i}")
    hback = np.ctypeslib.as_array((ctypes.c_uint8 * (frames * in_stride)).from_address(pback))
    st = np.ctypeslib.as_array((ctypes.c_uint16 * frames).from_address(pstat))
    if np.any(st & 0xff) or not np.array_equal(hback, hin):
        raise SystemExit("e2e open round trip failed")
    lib.cz_ctx_destroy(ctx)
    for p in (pin, pout, pback, pstat):
        lib.cz_host_free(p)
    pay = frames * n
    ceil = copy_ceiling(dev)
    pcie = frames * (in_stride + out_stride) / res["seal"] / 1e9
    return {"metric": "CURVE seal GiB/s end-to-end from pinned host memory (H2D + seal + D2H), 4 KiB frames",
            "value": round(pay / res["seal"] / 2**30, 3), "unit": "GiB/s", "n_gpus": 1,
            "open_GiBps": round(pay / res["open"] / 2**30, 3),
            "pcie_bytes_per_s": round(pcie, 2),
            "copy_ceiling": ceil, "frac_of_bidir_ceiling": round(pcie / ceil["bidir_GBps_total"], 3),
            "config": {"workload": f"{frames} x 4 KiB frames, pinned host buffers, 3-stream pipeline, "
                                   f"{chunk}-frame chunks", "frames": frames}}


def engine_host(args, dev):
    """Batching engine end-to-end (cz_engine_*): 1024 connections x 256 MESSAGEs of 4 KiB.
    flush_out = descriptors + H2D + segmented seal + V2 pack + D2H into per-connection wire
    streams; flush_in = V2 parse + H2D + unpack + open + D2H + per-connection delivery.
    Wall clock per flush; the Python send/recv loops are timed apart (ctypes overhead)."""
    from jeromq_amd.engine import CurveBatchEngine
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from cz_testlib import or_curve_encode, v2_encode
    nconn, per, n = 1024, 256, 4096
    total = nconn * per * n
    cli = CurveBatchEngine(arena_bytes=total + (1 << 20))
    srv = CurveBatchEngine(arena_bytes=1 << 20)
    keys = [bytes((PRECOM[j] + c) & 0xff for j in range(32)) for c in range(nconn)]
    cc = [cli.add_connection(keys[c]) for c in range(nconn)]
    sc = [srv.add_connection(keys[c], as_server=True) for c in range(nconn)]
    payload = np.random.default_rng(7).integers(0, 256, size=per * n, dtype=np.uint8).tobytes()
    res = {}
    for rep in range(3):          # first round warms allocations and clocks
        t0 = time.perf_counter()
        for c in range(nconn):
            for k in range(per):
                buf = cli.msg_alloc(n)
                ctypes.memmove(buf, payload[k * n:(k + 1) * n], n)
                cli.send(cc[c], buf, more=(k % 8 == 0))
        t_send = time.perf_counter() - t0
        t0 = time.perf_counter()
        cli.flush_out()
        t_out = time.perf_counter() - t0
        wires = [cli.wire_out(cc[c]) for c in range(nconn)]
        t0 = time.perf_counter()
        for c in range(nconn):
            srv.recv(sc[c], wires[c])
        t_recv = time.perf_counter() - t0
        t0 = time.perf_counter()
        srv.flush_in()
        t_in = time.perf_counter() - t0
        res = {"send_loop_s": t_send, "flush_out_s": t_out, "recv_loop_s": t_recv, "flush_in_s": t_in}
    # parity spot checks: connection 5's first frame on the wire, connection 9's last message in
    nonce0 = 3 + 2 * per   # third round
    first = v2_encode(or_curve_encode(payload[:n], 1, nonce0, 0, keys[5]))
    ok = wires[5][:len(first)] == first
    got = srv.messages_in(sc[9])
    ok = ok and len(got) == per and got[-1][0] == payload[(per - 1) * n:per * n]
    ok = ok and all(srv.error(sc[c])[0] == 0 for c in range(nconn))
    msgs = nconn * per
    small = engine_small_flush()
    ceil = copy_ceiling(dev)
    wire_bytes = sum(len(x) for x in wires)
    return {"metric": "CURVE batching engine end-to-end GiB/s (pinned host, 1024 connections, ZMTP v2 wire)",
            "copy_ceiling": ceil,
            "flush_out_pcie_GBps": round((total + wire_bytes) / res["flush_out_s"] / 1e9, 2),
            "value": round(total / res["flush_out_s"] / 2**30, 3), "unit": "GiB/s", "n_gpus": 1,
            "open_GiBps": round(total / res["flush_in_s"] / 2**30, 3),
            "msgs_per_s_out": round(msgs / res["flush_out_s"], 1), "msgs_per_s_in": round(msgs / res["flush_in_s"], 1),
            "timings_s": {k: round(v, 4) for k, v in res.items()}, "verified": bool(ok),
            "small_flush": small,
            "config": {"workload": f"{nconn} connections x {per} x {n} B MESSAGEs per flush", "frames": msgs}}


def engine_small_flush(reps=60):
    """Latency of small engine flushes: one connection, `count` MESSAGEs of `n` bytes per flush;
    median wall clock of flush_out and of flush_in (the wire fed back to a server engine), with the
    delivered payloads checked."""
    from jeromq_amd.engine import CurveBatchEngine
    rows = []
    for count, n in ((1, 100), (1, 4096), (1, 65536), (64, 4096)):
        cli = CurveBatchEngine(arena_bytes=count * n + (1 << 20))
        srv = CurveBatchEngine(arena_bytes=1 << 20)
        cc, sc = cli.add_connection(PRECOM), srv.add_connection(PRECOM, as_server=True)
        payload = np.random.default_rng(n).integers(0, 256, size=count * n, dtype=np.uint8).tobytes()
        t_out, t_in, ok = [], [], True
        for r in range(reps):
            for k in range(count):
                buf = cli.msg_alloc(n)
                ctypes.memmove(buf, payload[k * n:(k + 1) * n], n)
                cli.send(cc, buf)
            t0 = time.perf_counter()
            cli.flush_out()
            t_out.append(time.perf_counter() - t0)
            srv.recv(sc, cli.wire_out(cc))
            t0 = time.perf_counter()
            srv.flush_in()
            t_in.append(time.perf_counter() - t0)
            got = srv.messages_in(sc)
            ok = ok and len(got) == count and all(got[k][0] == payload[k * n:(k + 1) * n] for k in range(count))
        rows.append({"messages": count, "payload_bytes": n, "flush_out_us": round(float(np.median(t_out)) * 1e6, 1),
                     "flush_in_us": round(float(np.median(t_in)) * 1e6, 1), "verified": bool(ok)})
        del cli, srv
    return rows


def _libsodium():
    """libsodium from the image (an optimised CPU NaCl, for comparison only; None if absent)."""
    for path in ("/opt/conda/lib/libsodium.so", "libsodium.so.23", "libsodium.so"):
        try:
            L = ctypes.CDLL(path)
            if L.sodium_init() >= 0:
                return L
        except OSError:
            pass
    return None


def nacl_latency(args, dev):
    """Single-message latency of the jnacl drop-ins (cz_box_afternm / cz_box_open_afternm, the
    Curve.afternm / openAfternm path of INTEGRATION.md section 2: one message per call, host
    buffers in and out), at 100 B / 4 KiB / 64 KiB, beside one CPU core (the oracle port and
    libsodium), and the batch size at which the host-staged batched API (cz_ctx_seal_uniform)
    beats one CPU core per message.  Wall clock through ctypes, median of many calls."""
    lib = _lib.lib()
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from cz_testlib import oracle
    orc = oracle()
    sod = _libsodium()
    k = (ctypes.c_uint8 * 32).from_buffer_copy(PRECOM)
    nonce = (ctypes.c_uint8 * 24).from_buffer_copy(b"CurveZMQMESSAGEC" + (3).to_bytes(8, "big"))

    def med(fn, reps, budget_s=1.5):
        fn()
        ts = []
        t_end = time.perf_counter() + budget_s
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
            if time.perf_counter() > t_end and len(ts) >= 5:
                break
        return float(np.median(ts))
    t_ctypes = med(lambda: lib.cz_version(), 2000)
    rows = []
    for n in (100, 4096, 65536):
        mlen = n + 32
        m = (ctypes.c_uint8 * mlen)()
        m[32:] = list(np.random.default_rng(n).integers(0, 256, size=n, dtype=np.uint8))
        c = (ctypes.c_uint8 * mlen)()
        back = (ctypes.c_uint8 * mlen)()
        t_seal = med(lambda: lib.cz_box_afternm(c, m, mlen, nonce, k), 400)
        t_open = med(lambda: lib.cz_box_open_afternm(back, c, mlen, nonce, k), 400)
        ok = lib.cz_box_afternm(c, m, mlen, nonce, k) == 0 and bytes(c) == orc_seal(orc, bytes(m), nonce, k)
        ok = ok and lib.cz_box_open_afternm(back, c, mlen, nonce, k) == 0 and bytes(back) == bytes(m)
        co, mb, nb = ctypes.create_string_buffer(mlen), bytes(m), bytes(nonce)
        t_or = med(lambda: orc.or_secretbox(co, mb, mlen, nb, PRECOM), 400)
        row = {"payload_bytes": n, "seal_us": round(t_seal * 1e6, 1), "open_us": round(t_open * 1e6, 1),
               "oracle_1core_us": round(t_or * 1e6, 2), "verified": bool(ok)}
        if sod is not None:
            cs = (ctypes.c_uint8 * mlen)()
            t_s = med(lambda: sod.crypto_box_afternm(cs, m, ctypes.c_ulonglong(mlen), nonce, k), 2000)
            row["libsodium_1core_us"] = round(t_s * 1e6, 2)
        rows.append(row)
    # boxes past one pass of k_nacl_one (80 KiB): the segment kernels (CurveZMQ boxes, m[0:32] == 0,
    # the default) against k_nacl_one's multi-pass walk (cz_tune "nacl_one_max"; always taken by a
    # seal whose m[0:32] is not zero, whose MAC key only k_nacl_one derives)
    large = []
    for n in (96 << 10, 256 << 10, 1 << 20, 4 << 20):
        mlen = n + 32
        m = (ctypes.c_uint8 * mlen)()
        m[32:] = list(np.random.default_rng(n).integers(0, 256, size=n, dtype=np.uint8))
        mp = (ctypes.c_uint8 * mlen).from_buffer_copy(bytes(range(1, 33)) + bytes(m)[32:])
        c = (ctypes.c_uint8 * mlen)()
        back = (ctypes.c_uint8 * mlen)()
        row = {"box_bytes": mlen}
        for name, knob in (("segments", 80 << 10), ("one_launch", 1 << 30)):
            old = lib.cz_tune(b"nacl_one_max", knob)
            try:
                row[name + "_seal_us"] = round(med(lambda: lib.cz_box_afternm(c, m, mlen, nonce, k), 50) * 1e6, 1)
                ok = bytes(c) == orc_seal(orc, bytes(m), nonce, k)
                row[name + "_open_us"] = round(med(lambda: lib.cz_box_open_afternm(back, c, mlen, nonce, k), 50) * 1e6, 1)
                row[name + "_verified"] = bool(ok and bytes(back) == bytes(m))
            finally:
                lib.cz_tune(b"nacl_one_max", old)
        row["nonzero_prefix_seal_us"] = round(med(lambda: lib.cz_box_afternm(c, mp, mlen, nonce, k), 50) * 1e6, 1)
        row["nonzero_prefix_verified"] = bytes(c) == orc_seal(orc, bytes(mp), nonce, k)
        large.append(row)
    # the Mechanism mirror (cz_mech_encode / decode), one MESSAGE per call
    from jeromq_amd.mechanism import CurveClientMechanism, CurveServerMechanism, Msg
    mrows = []
    for n in (100, 4096, 65536, 262144):
        cli, srv = CurveClientMechanism(PRECOM), CurveServerMechanism(PRECOM)
        msg = Msg(np.random.default_rng(n).integers(0, 256, size=n, dtype=np.uint8).tobytes())
        t_enc, t_dec, ok = [], [], True
        for _ in range(100):
            t0 = time.perf_counter()
            enc = cli.encode(msg)
            t_enc.append(time.perf_counter() - t0)
            t0 = time.perf_counter()
            dec = srv.decode(enc)
            t_dec.append(time.perf_counter() - t0)
            ok = ok and dec is not None and dec.data == msg.data
        mrows.append({"payload_bytes": n, "encode_us": round(float(np.median(t_enc)) * 1e6, 1),
                      "decode_us": round(float(np.median(t_dec)) * 1e6, 1), "verified": bool(ok)})
    # batched host-staged API at 4 KiB: per-call time for B messages
    ctx = ctypes.c_void_p()
    _lib.check(lib.cz_ctx_create(ctypes.byref(ctx), dev.index or 0), "cz_ctx_create")
    _lib.check(lib.cz_ctx_set_keys(ctx, PRECOM, 1, _lib.CZ_DIR_C2S), "cz_ctx_set_keys")
    bmax = 1 << 16
    pin, pout = lib.cz_host_alloc(bmax * 4096), lib.cz_host_alloc(bmax * 4224)
    batches = []
    for B in (1, 4, 16, 64, 256, 1024, 2048, 4096, 8192, 16384, 65536):
        t = med(lambda: _lib.check(lib.cz_ctx_seal_uniform(ctx, B, 4096, pin, 4096, pout, 4224, 3, None, 0),
                                   "seal"), 100)
        batches.append({"batch": B, "call_us": round(t * 1e6, 1), "per_msg_us": round(t * 1e6 / B, 3),
                        "GiBps": round(B * 4096 / t / 2**30, 3)})
    lib.cz_ctx_destroy(ctx)
    lib.cz_host_free(pin)
    lib.cz_host_free(pout)
    cpu_4k = next(r for r in rows if r["payload_bytes"] == 4096)
    ref_us = cpu_4k.get("libsodium_1core_us", cpu_4k["oracle_1core_us"])
    win = next((b["batch"] for b in batches if b["per_msg_us"] < ref_us), None)
    return {"metric": "jnacl drop-in single-message latency (cz_box_afternm / open), host buffers",
            "value": rows[1]["seal_us"], "unit": "us per 4 KiB message", "higher_is_better": False, "n_gpus": 1,
            "ctypes_call_overhead_us": round(t_ctypes * 1e6, 2), "single_shot": rows, "large_boxes": large,
            "mechanism_single": mrows,
            "batched_4k": batches,
            "batch_beating_one_cpu_core": win,
            "cpu_reference_for_crossover": "libsodium crypto_box_afternm, 1 core" if sod is not None else "oracle, 1 core"}


def orc_seal(orc, m, nonce, k):
    out = ctypes.create_string_buffer(len(m))
    orc.or_secretbox(out, m, len(m), bytes(nonce), bytes(k))
    return out.raw


def beforenm_bench(args, dev):
    """Handshake key agreement: cz_beforenm_batch over 2^18 random key
    pairs per launch (connection churn), timed with HIP events; oracle on 1 host thread beside it."""
    from jeromq_amd import _lib
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from cz_testlib import or_beforenm
    n = 1 << 18
    g = torch.Generator(device="cpu").manual_seed(7)
    pk = torch.randint(0, 256, (32 * n,), dtype=torch.uint8, generator=g).to(dev)
    sk = torch.randint(0, 256, (32 * n,), dtype=torch.uint8, generator=g).to(dev)
    k = torch.empty(32 * n, dtype=torch.uint8, device=dev)
    L = _lib.lib()
    s = torch.cuda.current_stream()

    def step():
        _lib.check(L.cz_beforenm_batch(pk.data_ptr(), sk.data_ptr(), k.data_ptr(), n, ctypes.c_void_p(s.cuda_stream)),
                   "cz_beforenm_batch")
    for _ in range(max(args.warmup, 2)):
        step()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    for a, b in evs:
        a.record(s)
        step()
        b.record(s)
    torch.cuda.synchronize()
    ms = float(np.median([a.elapsed_time(b) for a, b in evs]))
    hp, hs, hk = pk.cpu().numpy().tobytes(), sk.cpu().numpy().tobytes(), k.cpu().numpy().tobytes()
    ok = all(hk[32 * i:32 * i + 32] == or_beforenm(hp[32 * i:32 * i + 32], hs[32 * i:32 * i + 32])
             for i in (0, 1, n // 2, n - 1))
    t0 = time.perf_counter()
    cnt = 0
    while time.perf_counter() - t0 < 2.0:
        or_beforenm(hp[:32], hs[:32])
        cnt += 1
    cpu_rate = cnt / (time.perf_counter() - t0)
    return {"metric": "CURVE handshake beforenm (X25519 + HSalsa20) per second, device batch",
            "value": round(n / (ms / 1e3), 1), "unit": "ops/s", "n_gpus": 1, "steps": args.steps,
            "kernel_ms": round(ms, 4), "batch": n, "verified": bool(ok),
            "cpu_baseline": {"value": round(cpu_rate, 1), "unit": "ops/s", "cores": 1, "kind": "port",
                             "sample": "oracle/curve_oracle.c or_box_beforenm (radix 2^51), 2 s on 1 thread"}}


def load_pmc(key):
    """This config's entry of the committed rocprofv3 PMC summary (profiles/pmc_traffic.json:
    HBM bytes per launch from tools/gpu_traffic.sh, VALU wave-instructions per launch from
    tools/gpu_valu.sh), or {}.  key = tools/pmc_key.py's config + non-default layout options, so
    a layout never borrows another layout's counters."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            return json.load(f).get(key) or {}
    except (OSError, ValueError):
        return {}


# VALU issue roofline.  Every int32 VALU wave-instruction occupies its SIMD for 4 cycles on
# gfx950 (tools/diag/salsa_ub.hip, profiles/r01/ubench_salsa_issue.log: 3.9-4.1 cycles at 3-8
# waves per SIMD, any opcode mix, any order), so the chip issues at most
# 256 CUs x 4 SIMDs x 2.4 GHz / 4 = 614.4 G wave-instructions/s.
VALU_PEAK_G = 256 * 4 * 2.4 / 4


def hbm_copy_ceiling(dev, nbytes=1 << 31, reps=10):
    """Device-to-device copy of nbytes by the library's float4 copy kernel (cz_dev_copy: 16-byte
    loads and stores, the copy the MI355X guide measures at 6.29 TB/s), HIP events on the stream it
    runs on: (read + write bytes) / time, GB/s.  torch's copy_ of the same buffers beside it."""
    src = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    dst = torch.empty_like(src)
    s = torch.cuda.current_stream()
    L = _lib.lib()

    def timed(fn):
        for _ in range(2):
            fn()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        for _ in range(reps):
            fn()
        b.record(s)
        torch.cuda.synchronize()
        return round(2 * nbytes * reps / (a.elapsed_time(b) / 1e3) / 1e9, 1)
    k = None
    if hasattr(L, "cz_dev_copy"):  # (absent only from A/B builds older than it)
        k = timed(lambda: _lib.check(L.cz_dev_copy(dst.data_ptr(), src.data_ptr(), nbytes,
                                                   ctypes.c_void_p(s.cuda_stream)), "cz_dev_copy"))
    t = timed(lambda: dst.copy_(src))
    del src, dst
    return k, t


def pmc_freshness(pmc, lib_path=None):
    """Whether the committed counter entry belongs to the library loaded now: sha256 of the machine
    code of the kernels it was measured on (jeromq_amd.build.kernel_code_sha256, recorded by
    tools/traffic_update.py / valu_update.py) against the same kernels in the loaded library.
    {"traffic_stale": bool | None, "valu_stale": ..., "kernel_sha256": loaded}; None = the entry
    carries no sha (measured before round 6) or no counters."""
    from jeromq_amd.build import kernel_code_sha256
    lib_path = lib_path or _lib.LIB_PATH
    out = {}
    for part, kern_key in (("traffic", "kernels"), ("valu", "valu_kernels")):
        kernels = pmc.get(kern_key) or pmc.get("kernels")
        want = pmc.get(f"{part}_kernel_sha256")
        have = None
        try:
            have = kernel_code_sha256(lib_path, kernels) if kernels else None
        except Exception as e:  # noqa: BLE001 -- a missing tool leaves the question open, never fails the bench
            out[f"{part}_check_error"] = str(e)[:200]
        out[f"{part}_stale"] = None if not want or have is None else want != have
        out[f"{part}_kernel_sha256_loaded"] = have
    return out


def valu_roofline(pmc, kernel_s):
    n = pmc.get("valu_insts_per_launch")
    if not n:
        return None
    g = n / kernel_s / 1e9
    out = {"insts_per_launch": n, "achieved": round(g, 1), "peak": VALU_PEAK_G, "unit": "G wave-instr/s",
           "frac": round(g / VALU_PEAK_G, 4),
           "floor_ms_at_2.4GHz": round(n / (VALU_PEAK_G * 1e9) * 1e3, 4),
           "source": pmc.get("valu_source")}
    clk = pmc.get("stamped_clock_ghz")
    if clk:
        # the issue roof at the clock the kernel really runs at (in-kernel s_memtime stamps, unprofiled):
        # the fraction of that clock's cycles the SIMDs spend issuing VALU
        out["stamped_clock_ghz"] = clk
        out["frac_at_clock"] = round(n * 4 / 1024 / (clk * 1e9) / kernel_s, 4)
        out["clock_source"] = pmc.get("stamped_clock_source")
    return out


def scatter_leg(wl, world, rank, dev):
    """North-star data movement, timed separately: rank 0 holds the whole
    batch, RCCL-scatters each rank its shard over xGMI, every rank seals its shard, and the
    bodies are gathered back to rank 0.  Never folded into `value`; run after the main line is
    out (run_leg), the bytes on data_group() (RCCL), barriers and the verdict on the gloo default."""
    from jeromq_amd import shard
    import torch.distributed as dist
    group = data_group()
    gloo = DATA_BACKEND != "nccl"
    n_in, n_out = wl.d_in.numel(), wl.d_out.numel()
    sdev = torch.device("cpu") if gloo else dev
    full_in = full_out = None
    if rank == 0:
        full_in = torch.empty(world * n_in, dtype=torch.uint8, device=dev)
        for r in range(world):
            batch.fill(full_in[r * n_in:(r + 1) * n_in], shard_plan(r, wl.count, wl.cfg)[1])
        full_out = torch.empty(world * n_out, dtype=torch.uint8, device=sdev)
        torch.cuda.synchronize()
        if gloo:
            full_in = full_in.cpu()
    recv = torch.empty(n_in, dtype=torch.uint8, device=sdev)
    t_sc = shard.timed(lambda: shard.scatter_shards(recv, full_in, group=group), world)
    ok = torch.equal(recv.to(dev), wl.d_in)
    saved = wl.d_in
    wl.d_in = recv.to(dev) if gloo else recv
    t_seal = shard.timed(wl.step, world)
    wl.d_in = saved
    send = wl.d_out.cpu() if gloo else wl.d_out
    t_ga = shard.timed(lambda: shard.gather_shards(send, full_out, group=group), world)
    okt = torch.tensor([1.0 if ok else 0.0], dtype=torch.float64)
    dist.all_reduce(okt, op=dist.ReduceOp.MIN)
    verified = okt.item() == 1.0
    if rank == 0:
        # the last rank's last frame, out of rank 0's gathered buffer, against the oracle
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from cz_testlib import or_curve_encode
        r, i = world - 1, wl.count - 1
        base_in, base_out = r * n_in + i * wl.in_stride, r * n_out + i * wl.out_stride
        p = full_in[base_in:base_in + wl.n].cpu().numpy().tobytes()
        body = full_out[base_out:base_out + wl.n + 33].cpu().numpy().tobytes()
        fl = 1 if i % 8 == 0 else 0
        verified = verified and body == or_curve_encode(p, fl, shard_plan(r, wl.count, wl.cfg)[0] + i, 0, PRECOM)
    moved_out = (world - 1) * n_in
    moved_back = (world - 1) * n_out
    total_payload = world * wl.payload_bytes
    return {"backend": "nccl (RCCL)" if not gloo else "gloo", "scatter_ms": round(t_sc * 1e3, 3), "seal_ms": round(t_seal * 1e3, 3),
            "gather_ms": round(t_ga * 1e3, 3),
            "scatter_GBps": round(moved_out / t_sc / 1e9, 2), "gather_GBps": round(moved_back / t_ga / 1e9, 2),
            "bytes_out_of_rank0": moved_out, "bytes_into_rank0": moved_back,
            "e2e_GiBps": round(total_payload / (t_sc + t_seal + t_ga) / 2**30, 3), "verified": bool(verified)}


def roundtrip_leg(wl, world, steps):
    """BASELINE.json configs[4]: every rank seals its 2^20 x 4 KiB shard and
    opens + tag-verifies the bodies it just sealed (CurveServerMechanism.decode, nonce strictly
    above the previous one), timed separately from `value` with the same barrier + max-over-ranks
    clock.  `verified`: every status is OK and every opened payload equals its input, on all ranks."""
    plain = torch.empty_like(wl.d_in)
    status = torch.empty(wl.count, dtype=torch.int16, device=wl.dev)

    def rt():
        wl.step()
        batch.open_uniform(wl.d_out, wl.out_stride, plain, wl.in_stride, wl.count, wl.n + 33, wl.subkey,
                           wl.counter0 - 1, status)
    for _ in range(3):
        rt()
    torch.cuda.synchronize()
    barrier(world)
    t0 = time.perf_counter()
    for _ in range(steps):
        rt()
    torch.cuda.synchronize()
    barrier(world)
    elapsed = max_over_ranks(world, time.perf_counter() - t0)
    ok = not bool((status & 0xff).any().item()) and torch.equal(plain, wl.d_in)  # low byte: rc, high: flags
    ok = sum_over_ranks(world, 1.0 if ok else 0.0) == world
    total = sum_over_ranks(world, float(wl.payload_bytes)) * steps
    return {"steps": steps, "ms_per_roundtrip": round(elapsed / steps * 1e3, 4),
            "payload_GiBps": round(total / elapsed / 2**30, 3), "verified": bool(ok)}


def jni_host(args):
    """The host path timed THROUGH the JNI shim (north star: the end-to-end rate including the JNI
    pinned-buffer copies): tools/bin/jni_bench (jni/jni_bench.c, built by __graft_entry__.build)
    drives jni/curvezmq_jni.c over the fake JNIEnv -- GpuCurveBatch.sealUniform / openUniform on
    hostAlloc direct buffers at 4 KiB (2^16 .. --frames) and 100 B, the jnacl crypto_box_afternm per
    message, the GpuCurveEngine loop of GpuCurveIoHook over 1024 connections -- each beside the plain
    C-ABI on the same buffers.  Run as a child process: this one never touches the GPU.  `value` =
    the 4 KiB seal at the largest batch through the shim, payload GiB/s (pinned host in and out)."""
    import subprocess
    exe = os.path.join(ROOT, "tools", "bin", "jni_bench")
    if not os.path.exists(exe):
        raise SystemExit(f"{exe} is missing: run __graft_entry__.build() (gcc, the JNI shim over a fake JNIEnv)")
    r = subprocess.run([exe, str(args.frames), str(max(args.steps // 6, 3))], capture_output=True, text=True,
                       timeout=1200)
    sys.stderr.write(r.stderr)
    if r.returncode != 0:
        print(f"jni_bench failed (exit {r.returncode})", file=sys.stderr)
        return r.returncode or 1
    line = json.loads(r.stdout.strip().splitlines()[-1])
    big = max((u for u in line["uniform"] if u["payload_bytes"] == 4096), key=lambda u: u["frames"])
    line.update({"value": big["seal_GiBps"], "unit": "GiB/s", "n_gpus": 1, "higher_is_better": True,
                 "verified": all(u["verified"] for u in line["uniform"]) and all(x["verified"] for x in line["jnacl"])
                 and line["engine"]["verified"],
                 "config": {"workload": f"{big['frames']} x 4 KiB frames, pinned host buffers through "
                                        "GpuCurveBatch.sealUniform (JNI shim, fake JNIEnv)", "frames": big["frames"]}})
    print(json.dumps(line), flush=True)
    return 0 if line["verified"] else 1


def main():
    args = parse()
    if args.config == "jni":
        sys.exit(jni_host(args))
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world, rank, local = setup_dist(args)
    dev = torch.device(f"cuda:{local}")
    if args.config in ("e2e4k", "engine", "beforenm", "nacl"):
        line = {"e2e4k": e2e_host, "engine": engine_host, "beforenm": beforenm_bench,
                "nacl": nacl_latency}[args.config](args, dev)
        if rank == 0:
            print(json.dumps(line), flush=True)
        return
    wl = Workload(args.config, args.frames, rank, dev, out_align=args.out_align, seg_blocks=args.seg_blocks,
                  in_align=args.in_align, plain_stride=args.plain_stride,
                  in_stride=args.in_stride, out_stride=args.out_stride)

    ramp = 0
    t_ramp = time.perf_counter()
    while (time.perf_counter() - t_ramp) * 1e3 < args.ramp_ms:
        for _ in range(4):
            wl.step()
            ramp += 1
        torch.cuda.synchronize()
    for _ in range(args.warmup):
        wl.step()
    torch.cuda.synchronize()
    if not args.no_verify:
        wl.verify_sample()

    stream = torch.cuda.current_stream()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for a, b in evs:
        a.record(stream)
        wl.step()
        b.record(stream)
    torch.cuda.synchronize()
    barrier(world)
    elapsed = time.perf_counter() - t0
    kern_ms = [a.elapsed_time(b) for a, b in evs]
    avg_kernel_s = float(np.mean(kern_ms)) / 1e3

    per_rank, kernel_s = None, [avg_kernel_s]
    if world > 1:
        # every rank's own kernel time and roofline fraction (the driver's 1/2/4/8-GPU runs then
        # carry absolute per-GPU figures with no further code change)
        import torch.distributed as dist
        kd = "cuda" if dist.get_backend() == "nccl" else "cpu"
        mine = torch.tensor([avg_kernel_s], dtype=torch.float64, device=kd)
        allk = [torch.zeros(1, dtype=torch.float64, device=kd) for _ in range(world)]
        dist.all_gather(allk, mine)
        alg = wl.read_bytes + wl.write_bytes
        kernel_s = [float(k.item()) for k in allk]
        per_rank = [{"rank": r, "kernel_ms": round(k * 1e3, 4),
                     "payload_GiBps": round(wl.payload_bytes / k / 2**30, 2),
                     "hbm_frac": round(alg / k / 1e9 / HBM_PEAK_GBS, 4)} for r, k in enumerate(kernel_s)]
    elapsed = max_over_ranks(world, elapsed)
    total_payload = sum_over_ranks(world, float(wl.payload_bytes) * args.steps)
    value = total_payload / elapsed / 2**30
    alg_bytes = wl.read_bytes + wl.write_bytes
    roof_k = multi_rank_roofline(kernel_s, alg_bytes)  # N = 1: this rank's own kernel time
    achieved = roof_k["achieved"]
    slow_kernel_s = max(kernel_s)
    copy_gbs, torch_copy_gbs = hbm_copy_ceiling(dev) if rank == 0 else (None, None)
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from pmc_key import key_from_args
    pmc_key = key_from_args(args)
    pmc = load_pmc(pmc_key)
    traffic = pmc.get("hbm_bytes_per_launch")
    pmc_build = pmc_freshness(pmc)

    want_leg = world > 1 and args.config == "4k" and not args.no_scatter

    rtl = None
    if args.config == "4k" and not args.no_roundtrip:
        rtl = roundtrip_leg(wl, world, min(args.steps, 10))

    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        # at N > 1 too, on rank 0 after every timed leg (the other ranks wait at the barrier below)
        cpu = cpu_baseline(wl, args.cpu_seconds)
        if world > 1:
            cpu["measured"] = f"rank 0 of {world}, after the timed region"
    barrier(world)

    if rank == 0:
        names = {"4k": "1M x 4 KiB frames, seal (configs[1])",
                 "4k_dense": "1M x 4 KiB frames, seal, bodies packed back to back (4129-byte slots)",
                 "4k_box": "1M x 4 KiB frames, seal, input in the reference's box layout (0^32 || flags || payload, "
                           "4224-byte slots)",
                 "100b": "1M x 100 B frames, seal (configs[2])",
                 "zipf": "1M Zipf(1.2) 64 B..64 KiB frames, seal, segmented (configs[3])",
                 "zipf_lane": "1M Zipf(1.2) 64 B..64 KiB frames, seal, lane per frame (configs[3])",
                 "zipf_open": "1M Zipf(1.2) 64 B..64 KiB frames, open+verify of the sealed batch, segmented "
                              "(configs[3], receive side)",
                 "open4k": "1M x 4 KiB frames, open+verify (configs[4] leg)"}
        line = {
            "metric": "CURVE encrypt+MAC GiB/s (device-resident), batched 4 KiB frames, 1/2/4/8 GPU",
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ramp_steps": ramp,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (SplitMix64 payload on device, RFC test keys)",
            "config": {"workload": names[args.config] + (
                           f", input offsets {args.in_align}-byte / output offsets {args.out_align}-byte aligned"
                           if args.config.startswith("zipf") else "") + (
                           f", plaintext slots {wl.plain_stride} B" if args.config == "open4k" else "") + (
                           f", slots in {wl.in_stride} / out {wl.out_stride} B"
                           if args.in_stride or args.out_stride else ""),
                       "frames_per_gpu": wl.count,
                       "payload_bytes_per_gpu": wl.payload_bytes, "parallelism": f"shard{world}",
                       "frames_per_s": round(wl.count * world * args.steps / elapsed, 1)},
            # bound: the roof that binds is VALU issue; achieved / peak / frac are the
            # HBM figures the north star asks for, the VALU roof is in "valu"
            "roofline": {"bound": "valu", "achieved": roof_k["achieved"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": roof_k["frac"],
                         "traffic": traffic,
                         **{k: v for k, v in roof_k.items() if k not in ("achieved", "frac")},
                         # the same bytes against the device-to-device copy rate
                         # measured on this GPU in this process (read + write bytes / time)
                         "hbm_copy_GBps": copy_gbs,  # cz_dev_copy (float4 copy kernel) of 2 GiB, 10 reps
                         "frac_of_copy": round(achieved / copy_gbs, 4) if copy_gbs else None,
                         "torch_copy_GBps": torch_copy_gbs,
                         "pmc_key": pmc_key,
                         "alg_bytes_per_launch": alg_bytes,
                         "valu": valu_roofline(pmc, slow_kernel_s),
                         # traffic / valu are committed rocprofv3 counts (profiles/pmc_traffic.json):
                         # stale when the loaded library's code of the measured kernels differs
                         "pmc_build": pmc_build},
            "cpu_baseline": cpu,
        }
        if rtl is not None:
            line["seal_open_verify"] = rtl
        if want_leg:  # run after this line is out; rank 0 prints its result on an SG_TAG line
            line["scatter_gather"] = {"pending": True, "reported_on": SG_TAG.strip() + " line",
                                      "deadline_s": args.leg_deadline}
        if per_rank is not None:
            import torch.distributed as dist
            assert len(per_rank) == world
            line["per_rank"] = per_rank
            line["dist"] = {"backend": dist.get_backend(), "world_size": world,
                            "gpus_visible": torch.cuda.device_count(),
                            "control_plane": "gloo (barriers, max-over-ranks timing, per-rank figures)",
                            "data_backend": DATA_BACKEND,
                            "rccl": DATA_BACKEND == "nccl"}
        print(json.dumps(line), flush=True)
    if want_leg:
        res = run_leg(lambda: scatter_leg(wl, world, rank, dev), rank, args.leg_deadline)
        if res.get("error"):
            os._exit(0)  # a failed collective can leave the groups unusable: no teardown, the line is out
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


def run_leg(fn, rank, deadline_s):
    """Run an optional leg after the main line: rank 0 prints its result (or error) on an SG_TAG
    line.  A watchdog ends this rank (exit 0: the main line is already out) if the leg has not
    returned within deadline_s -- an RCCL collective that never completes cannot be interrupted
    from Python.  Every rank runs its own watchdog, so a hung peer cannot hold the others."""
    import threading
    done = threading.Event()

    def report(res):
        if rank == 0:
            print(SG_TAG + json.dumps(res), flush=True)

    def watchdog():
        if not done.wait(deadline_s):
            report({"error": f"timeout: the leg did not finish within {deadline_s:.0f} s"})
            sys.stderr.write(f"rank {rank}: leg timed out after {deadline_s:.0f} s, exiting\n")
            sys.stderr.flush()
            os._exit(0)
    threading.Thread(target=watchdog, daemon=True).start()
    try:
        res = fn()
    except Exception as e:  # noqa: BLE001 -- any failure of the optional leg is reported, not fatal
        res = {"error": f"{type(e).__name__}: {e}"[:500]}
    done.set()
    report(res)
    return res


if __name__ == "__main__":
    main()
