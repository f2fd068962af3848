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
