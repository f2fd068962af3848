"""GPU, world_size 2 on ONE GPU (gloo; RCCL needs two GPUs, which only the driver's node run has):
the sharded path of SURVEY.md 8(e) with the real gfx950 kernels.

Rank 0 holds the whole batch; scatter_shards hands each rank its frames; every rank seals its
shard with its own counter range (bench.shard_plan); gather_shards brings the bodies back; rank 0
checks EVERY gathered frame against the oracle.  Then bench.py itself at --gpus 2 under
torch.distributed.run (the driver's launch line) must print one verified JSON line with per-rank
figures."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, frames, n, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    sys.path.insert(0, ROOT)
    sys.path.insert(0, HERE)
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        from jeromq_amd import _lib, batch, shard
        dev = torch.device("cuda:0")
        key = torch.tensor(list(bench.PRECOM), dtype=torch.uint8, device=dev).view(1, 32)
        sub = batch.subkeys(key, _lib.CZ_DIR_C2S)[0].contiguous()
        in_stride, out_stride = n, (n + 33 + 127) // 128 * 128
        full_in = full_out = None
        if rank == 0:
            g = torch.empty(world * frames * in_stride, dtype=torch.uint8, device=dev)
            for r in range(world):
                batch.fill(g[r * frames * in_stride:(r + 1) * frames * in_stride], bench.shard_plan(r, frames)[1])
            full_in = g.cpu()
            full_out = torch.empty(world * frames * out_stride, dtype=torch.uint8)
        recv = torch.empty(frames * in_stride, dtype=torch.uint8)
        shard.scatter_shards(recv, full_in)
        d_in = recv.to(dev)
        d_out = torch.empty(frames * out_stride, dtype=torch.uint8, device=dev)
        counter0 = bench.shard_plan(rank, frames)[0]
        batch.seal_uniform(d_in, in_stride, d_out, out_stride, frames, n, sub, counter0)
        torch.cuda.synchronize()
        shard.gather_shards(d_out.cpu(), full_out)
        checked = -1
        if rank == 0:
            from cz_testlib import DESC_DTYPE, oracle_check_full
            total = world * frames
            desc = np.zeros(total, dtype=DESC_DTYPE)
            desc["in_off"] = np.arange(total, dtype=np.uint64) * np.uint64(in_stride)
            desc["out_off"] = np.arange(total, dtype=np.uint64) * np.uint64(out_stride)
            desc["len"] = n
            # rank r's frames carry counters shard_plan(r)[0] + j: consecutive across ranks
            desc["counter"] = 3 + np.arange(total, dtype=np.uint64)
            desc["prev"] = -1
            checked = oracle_check_full(full_in, full_out, desc, bench.PRECOM)
        q.put((rank, checked))
    finally:
        dist.destroy_process_group()


def test_scatter_seal_gather_ws2_full_oracle():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import torch.multiprocessing as mp
    world, frames, n = 2, 8192, 4096
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, frames, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert res[0] == world * frames


def test_bench_ws2_rehearsal():
    """bench.py --gpus 2 as the driver launches it (torch.distributed.run), gloo on one GPU."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = dict(os.environ, CZ_DIST_BACKEND="gloo", TMPDIR="/tmp")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"), "--gpus", "2",
           "--steps", "3", "--warmup", "1", "--ramp-ms", "0", "--frames", "65536", "--cpu-seconds", "1"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["scaling"] == "weak"
    # the leg runs after the main line is out: pending there, its result on the SCATTER_GATHER line
    assert line["scatter_gather"]["pending"]
    sg = [ln for ln in r.stdout.splitlines() if ln.startswith("SCATTER_GATHER ")]
    assert len(sg) == 1 and r.stdout.index(lines[0]) < r.stdout.index(sg[0]), r.stdout[-2000:]
    line["scatter_gather"] = json.loads(sg[0][len("SCATTER_GATHER "):])
    assert line["dist"]["backend"] == "gloo" and line["dist"]["data_backend"] == "gloo"
    # as self-describing as the N = 1 line: slowest-rank roofline with its spread, and the CPU baseline
    roof = line["roofline"]
    assert roof["kernel_ms"] == roof["kernel_ms_max"] == max(p["kernel_ms"] for p in line["per_rank"])
    assert roof["frac_min"] <= roof["frac"] <= roof["frac_max"] and roof["frac"] == roof["frac_min"]
    assert line["cpu_baseline"]["value"] > 0 and "rank 0 of 2" in line["cpu_baseline"]["measured"]
    assert line["scatter_gather"]["verified"] and line["seal_open_verify"]["verified"]
    assert [p["rank"] for p in line["per_rank"]] == [0, 1]
    assert all(p["hbm_frac"] > 0 for p in line["per_rank"])


def test_bench_plain_gpus2_launches_its_own_ranks():
    """`python bench.py --gpus 2` with no launcher (how the driver runs N=1): bench.py starts the two
    ranks itself as a child torch.distributed.run and the line covers both (gloo on one GPU here;
    RCCL on the driver's 8-GPU node)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = dict(os.environ, CZ_DIST_BACKEND="gloo", TMPDIR="/tmp")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
           "--ramp-ms", "0", "--frames", "65536", "--cpu-seconds", "1"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and len(line["per_rank"]) == 2
    assert line["dist"]["world_size"] == 2 and line["dist"]["backend"] == "gloo"
    assert line["scatter_gather"]["verified"] and line["seal_open_verify"]["verified"]
    assert line["launcher"].startswith("bench.py --gpus")
    assert "ranks_exit_status" not in line
