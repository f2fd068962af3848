"""Multi-rank sharding of the batch on CPU with gloo, world_size 2.

The GPU path shards frames across ranks with no collective on the timed path; what
can be checked without a GPU is the shard plan (disjoint, contiguous nonce ranges,
distinct payload streams), the cross-rank timing reduction bench.py uses (max over
ranks / sum of payload), and that each rank's shard seals to the same bytes as the
corresponding slice of the single-rank batch (oracle).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, frames, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        from cz_testlib import or_curve_encode
        counter0, seed = bench.shard_plan(rank, frames)
        # ranks agree on the plan: gather every rank's counter range
        rng = torch.tensor([counter0, counter0 + frames], dtype=torch.int64)
        allr = [torch.zeros(2, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(allr, rng)
        # timing reduction as bench.py does it (slowest rank wins; payload sums)
        t = bench.max_over_ranks(world, 1.0 + rank)
        tot = bench.sum_over_ranks(world, 10.0 * (rank + 1))
        # seal this rank's first 3 frames with the oracle; body nonce must be its counters
        from cz_testlib import splitmix_bytes
        bodies = [or_curve_encode(splitmix_bytes(64, seed + j), 0, counter0 + j, 0, bytes(32)) for j in range(3)]
        nonces = [int.from_bytes(b[8:16], "big") for b in bodies]
        q.put((rank, [tuple(int(v) for v in r) for r in allr], t, tot, nonces, seed))
    finally:
        dist.destroy_process_group()


def test_shard_plan_and_reductions_gloo_ws2():
    world, frames = 2, 1 << 20
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, frames, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        rank, ranges, t, tot, nonces, seed = q.get(timeout=120)
        res[rank] = (ranges, t, tot, nonces, seed)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ranges = res[0][0]
    assert ranges == res[1][0]
    # disjoint, contiguous, starting at the first MESSAGE nonce 3
    assert ranges[0] == (3, 3 + frames) and ranges[1] == (3 + frames, 3 + 2 * frames)
    for r in range(world):
        assert res[r][1] == 2.0           # max over ranks
        assert res[r][2] == 30.0          # sum over ranks
        assert res[r][3] == [ranges[r][0] + j for j in range(3)]
    assert res[0][4] != res[1][4]         # distinct payload streams per rank


def test_shard_equals_slice_of_global_batch():
    """Sealing rank r's shard = sealing frames [r*F, (r+1)*F) of one big batch (same counters)."""
    from cz_testlib import DESC_DTYPE, oracle
    F, n = 8, 100
    rng = np.random.default_rng(0)
    payload = rng.integers(0, 256, size=(2 * F, n), dtype=np.uint8)
    k = bytes(range(32))

    def seal(p, counter0):
        cnt = len(p)
        d = np.zeros(cnt, dtype=DESC_DTYPE)
        d["in_off"] = np.arange(cnt) * n
        d["out_off"] = np.arange(cnt) * (n + 33)
        d["len"] = n
        d["counter"] = counter0 + np.arange(cnt)
        out = np.zeros(cnt * (n + 33), dtype=np.uint8)
        pc = np.ascontiguousarray(p)
        oracle().or_seal_batch(d.ctypes.data, cnt, pc.ctypes.data, out.ctypes.data,
                               np.frombuffer(k, dtype=np.uint8).copy().ctypes.data, 0, 1)
        return out

    import bench
    whole = seal(payload, 3)
    parts = [seal(payload[r * F:(r + 1) * F], bench.shard_plan(r, F)[0]) for r in range(2)]
    assert np.array_equal(np.concatenate(parts), whole)


def _scatter_worker(rank, world, port, F, n, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from cz_testlib import DESC_DTYPE, oracle
        from jeromq_amd import shard
        first, count = shard.frame_range(rank, world, world * F)
        full_in = full_out = None
        if rank == 0:
            rng = np.random.default_rng(5)
            full_in = torch.from_numpy(rng.integers(0, 256, size=world * F * n, dtype=np.uint8))
            full_out = torch.zeros(world * F * (n + 33), dtype=torch.uint8)
        mine = torch.zeros(count * n, dtype=torch.uint8)
        shard.scatter_shards(mine, full_in)
        # seal the shard (oracle stands in for the kernel on CPU) with counters of its range
        d = np.zeros(count, dtype=DESC_DTYPE)
        d["in_off"] = np.arange(count) * n
        d["out_off"] = np.arange(count) * (n + 33)
        d["len"] = n
        d["counter"] = 3 + first + np.arange(count)
        out = np.zeros(count * (n + 33), dtype=np.uint8)
        p = mine.numpy().copy()
        oracle().or_seal_batch(d.ctypes.data, count, p.ctypes.data, out.ctypes.data,
                               np.frombuffer(bytes(range(32)), dtype=np.uint8).copy().ctypes.data, 0, 1)
        shard.gather_shards(torch.from_numpy(out), full_out)
        t = shard.timed(lambda: None, world, device_sync=False)
        q.put((rank, None if full_in is None else (full_in.numpy(), full_out.numpy()), t >= 0))
    finally:
        dist.destroy_process_group()


def test_rccl_style_scatter_seal_gather_gloo_ws2():
    """shard.scatter_shards / gather_shards (the north star's scatter/gather leg) with gloo:
    rank 0's batch, scattered, sealed per shard and gathered back, equals the whole-batch seal."""
    from cz_testlib import DESC_DTYPE, oracle
    world, F, n = 2, 16, 100
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_scatter_worker, args=(r, world, port, F, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        rank, payload, ok = q.get(timeout=120)
        res[rank] = (payload, ok)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    full_in, full_out = res[0][0]
    d = np.zeros(world * F, dtype=DESC_DTYPE)
    d["in_off"] = np.arange(world * F) * n
    d["out_off"] = np.arange(world * F) * (n + 33)
    d["len"] = n
    d["counter"] = 3 + np.arange(world * F)
    want = np.zeros(world * F * (n + 33), dtype=np.uint8)
    fi = np.ascontiguousarray(full_in)
    oracle().or_seal_batch(d.ctypes.data, world * F, fi.ctypes.data, want.ctypes.data,
                           np.frombuffer(bytes(range(32)), dtype=np.uint8).copy().ctypes.data, 0, 1)
    assert np.array_equal(full_out, want)
    assert res[0][1] and res[1][1]


def test_frame_range_and_byte_balance():
    from jeromq_amd import shard
    for total, world in [(10, 3), (1 << 20, 8), (5, 8)]:
        rs = [shard.frame_range(r, world, total) for r in range(world)]
        assert sum(c for _, c in rs) == total
        assert all(rs[i][0] + rs[i][1] == rs[i + 1][0] for i in range(world - 1))
    rng = np.random.default_rng(42)
    lens = 64 * np.clip(rng.zipf(1.2, size=100000), 1, 1024)
    b = shard.balance_by_bytes(lens, 8)
    assert b[0] == 0 and b[-1] == len(lens) and all(b[i] <= b[i + 1] for i in range(8))
    work = [int((lens[b[r]:b[r + 1]] + 33).sum()) for r in range(8)]
    assert max(work) - min(work) <= 2 * (64 * 1024 + 33)   # within ~one max frame of each other
    assert shard.balance_by_bytes([], 4) == [0, 0, 0, 0, 0]


class _FakePopen:
    """Stands in for the child torch.distributed.run: records the command, replays canned stdout."""

    def __init__(self, out, rc=0):
        self.out, self.rc, self.cmd = out, rc, None
        self.pid = -1

    def __call__(self, cmd, **kw):
        self.cmd, self.kw = cmd, kw
        self.stdout = iter(self.out)
        return self

    def wait(self, timeout=None):
        return self.rc


def _rank_line(n, roofline=True, cpu=True):
    import json
    import bench
    line = {"metric": "m", "value": 1.0, "n_gpus": n, "per_rank": [{"rank": r, "kernel_ms": 2.0} for r in range(n)]}
    if roofline:
        line["roofline"] = bench.multi_rank_roofline([2e-3 + 1e-5 * r for r in range(n)], 8.6e9)
    if cpu:
        line["cpu_baseline"] = {"value": 0.5, "unit": "GiB/s", "cores": 1, "kind": "port", "sample": "s"}
    return json.dumps(line) + "\n"


def test_bench_gpus_n_launches_child_ranks_without_touching_gpu(capsys):
    """`python bench.py --gpus N` (no launcher): bench starts torch.distributed.run with N ranks as a
    child process, never initialises the GPU itself, and relays exactly one checked JSON line."""
    import json
    import bench
    fake = _FakePopen(["rank chatter\n", _rank_line(8)])
    rc = bench.launch_ranks(8, ["--gpus", "8", "--steps", "5"], popen=fake)
    assert rc == 0
    assert fake.cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"]
    assert "--nproc-per-node=8" in fake.cmd and "127.0.0.1" in fake.cmd
    assert fake.cmd[-4:] == ["--gpus", "8", "--steps", "5"]
    assert fake.kw["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    assert not torch.cuda.is_initialized()
    out = capsys.readouterr()
    lines = [ln for ln in out.out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1 and json.loads(lines[0])["n_gpus"] == 8
    assert "rank chatter" in out.err


@pytest.mark.parametrize("out,rc", [
    ([_rank_line(1)], 0),                    # ranks timed fewer GPUs than asked
    ([_rank_line(2), _rank_line(2)], 0),     # more than one JSON line
    ([], 0),                                 # no line at all
    ([], 3),                                 # a rank failed before the line: its exit status is passed on
    ([_rank_line(2, roofline=False)], 0),    # N > 1 line without the slowest-rank roofline
    ([_rank_line(2, cpu=False)], 0),         # N > 1 line without the CPU baseline
])
def test_bench_launcher_rejects_bad_rank_output(out, rc, capsys):
    import bench
    got = bench.launch_ranks(2, ["--gpus", "2"], popen=_FakePopen(out, rc))
    assert got == (rc if rc else 1)
    assert not [ln for ln in capsys.readouterr().out.splitlines() if ln.startswith("{")]


def test_multi_rank_roofline_uses_the_slowest_rank():
    """at N > 1, achieved / frac come from the slowest rank's kernel time (it sets
    the job's time), with the per-rank min and max fractions beside it."""
    import bench
    r = bench.multi_rank_roofline([2.0e-3, 2.5e-3, 2.1e-3], 8e9)
    assert r["kernel_ms"] == r["kernel_ms_max"] == 2.5 and r["kernel_ms_min"] == 2.0
    assert r["achieved"] == 3200.0 and r["frac"] == round(3200.0 / bench.HBM_PEAK_GBS, 4) == r["frac_min"]
    assert r["frac_max"] == round(4000.0 / bench.HBM_PEAK_GBS, 4)
    one = bench.multi_rank_roofline([2.0e-3], 8e9)
    assert one["frac"] == one["frac_min"] == one["frac_max"]


def test_bench_refuses_world_size_mismatch(monkeypatch):
    """Under a launcher, WORLD_SIZE must equal --gpus (a mismatch would mislabel the scaling line)."""
    import argparse
    import bench
    monkeypatch.setenv("WORLD_SIZE", "4")
    with pytest.raises(SystemExit, match="WORLD_SIZE=4"):
        bench.setup_dist(argparse.Namespace(gpus=8))
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.delenv("CZ_DIST_BACKEND", raising=False)
    with pytest.raises(SystemExit, match="need 2 GPUs for RCCL"):   # no GPU here: nccl refused, not faked
        bench.setup_dist(argparse.Namespace(gpus=2))


def test_bench_launcher_relays_a_good_line_despite_a_late_rank_failure(capsys):
    """A rank that fails after rank 0's main line is out (in the optional leg) no longer costs the
    scaling line: the line is relayed with the exit status recorded."""
    import json
    import bench
    rc = bench.launch_ranks(2, ["--gpus", "2"], popen=_FakePopen([_rank_line(2)], 3))
    assert rc == 0
    line = json.loads([ln for ln in capsys.readouterr().out.splitlines() if ln.startswith("{")][0])
    assert line["ranks_exit_status"] == 3


# --- the N > 1 line survives its optional RCCL scatter/gather leg -------------
# Stand-in children are real processes (python -c) in their own session, as torch.distributed.run
# is: they print a rank-0 main line, then (a) hang, (b) report a failed leg, or (c) report a good one.

def _main_line_pending(n):
    import json
    line = json.loads(_rank_line(n))
    line["scatter_gather"] = {"pending": True}
    return json.dumps(line)


def _stand_in(script):
    import sys
    return [sys.executable, "-c", script]


def _alive(pid):
    try:
        with open(f"/proc/{pid}/status") as f:
            return not any(ln.startswith("State:") and "Z" in ln.split()[1] for ln in f)
    except OSError:
        return False


def test_launcher_kills_ranks_that_hang_in_the_leg(tmp_path, capsys):
    import json
    import time
    import bench
    pidfile = tmp_path / "pids"
    script = f"""
import subprocess, sys, time, os
kid = subprocess.Popen([sys.executable, "-c", "import time; time.sleep(600)"])   # a 'rank'
open({str(pidfile)!r}, "w").write(f"{{os.getpid()}} {{kid.pid}}")
print('rank chatter', flush=True)
print({_main_line_pending(2)!r}, flush=True)
time.sleep(600)
"""
    t0 = time.monotonic()
    rc = bench.launch_ranks(2, ["--gpus", "2"], cmd=_stand_in(script), leg_deadline_s=2.0)
    took = time.monotonic() - t0
    assert rc == 0 and took < 60
    out = capsys.readouterr()
    lines = [ln for ln in out.out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and "timeout" in line["scatter_gather"]["error"]
    assert "killing their process group" in out.err
    parent, kid = (int(x) for x in pidfile.read_text().split())
    deadline = time.monotonic() + 10
    while (_alive(parent) or _alive(kid)) and time.monotonic() < deadline:
        time.sleep(0.1)
    assert not _alive(parent) and not _alive(kid), "stand-in ranks survived the launcher's kill"


def test_launcher_records_a_failed_leg(capsys):
    import json
    import bench
    script = f"""
print({_main_line_pending(2)!r}, flush=True)
print('SCATTER_GATHER {{"error": "DistBackendError: RCCL init failed"}}', flush=True)
raise SystemExit(1)
"""
    rc = bench.launch_ranks(2, ["--gpus", "2"], cmd=_stand_in(script), leg_deadline_s=60.0)
    assert rc == 0
    line = json.loads([ln for ln in capsys.readouterr().out.splitlines() if ln.startswith("{")][0])
    assert line["scatter_gather"] == {"error": "DistBackendError: RCCL init failed"}
    assert line["ranks_exit_status"] == 1


def test_launcher_merges_a_good_leg(capsys):
    import json
    import bench
    script = f"""
print({_main_line_pending(2)!r}, flush=True)
print('leg chatter', flush=True)
print('SCATTER_GATHER {{"backend": "nccl (RCCL)", "verified": true, "e2e_GiBps": 9.5}}', flush=True)
"""
    rc = bench.launch_ranks(2, ["--gpus", "2"], cmd=_stand_in(script), leg_deadline_s=60.0)
    assert rc == 0
    out = capsys.readouterr()
    lines = [ln for ln in out.out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    line = json.loads(lines[0])
    assert line["scatter_gather"] == {"backend": "nccl (RCCL)", "verified": True, "e2e_GiBps": 9.5}
    assert "ranks_exit_status" not in line and "leg chatter" in out.err


def test_launcher_reports_a_leg_that_never_reported():
    """ranks that exit cleanly after a pending main line without a leg line: an error, not a hang"""
    import bench
    import io
    import contextlib
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        rc = bench.launch_ranks(2, ["--gpus", "2"], cmd=_stand_in(f"print({_main_line_pending(2)!r})"))
    import json
    line = json.loads(buf.getvalue().splitlines()[-1])
    assert rc == 0 and "without reporting" in line["scatter_gather"]["error"]


@pytest.mark.parametrize("body,expect", [
    ("import time; time.sleep(120)", "timeout"),              # a collective that never returns
    ("1 / 0", "ZeroDivisionError"),                           # a leg that raises
    ("{'verified': True}", None),                             # a good leg
])
def test_rank_side_leg_watchdog(body, expect):
    """bench.run_leg on rank 0: the leg's result, its exception, or (watchdog) a timeout is printed on
    the SCATTER_GATHER line and the rank exits 0 -- within seconds, whatever the leg does."""
    import json
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    code = (f"import sys; sys.path.insert(0, {os.path.dirname(here)!r}); import bench\n"
            f"def leg():\n    return eval(compile({body!r}, 'leg', 'exec' if 'import' in {body!r} else 'eval'))\n"
            "r = bench.run_leg(leg, 0, 2.0)\nprint('returned', flush=True)\n")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=90)
    assert r.returncode == 0, r.stderr[-2000:]
    sg = [ln for ln in r.stdout.splitlines() if ln.startswith("SCATTER_GATHER ")]
    assert len(sg) == 1, r.stdout
    res = json.loads(sg[0][len("SCATTER_GATHER "):])
    if expect is None:
        assert res == {"verified": True} and "returned" in r.stdout
    else:
        assert expect in res["error"]
        assert ("returned" in r.stdout) == (expect != "timeout")
