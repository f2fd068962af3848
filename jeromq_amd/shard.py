"""Sharding a frame batch across the GPUs of one node.

Frames are independent given (subkey, counter), so a batch splits into
contiguous frame ranges with no data-path collective: each rank seals its range
with explicit counters.  The only data movement is the optional scatter of a
batch that arrives on one GPU (rank 0) and the gather of the sealed bodies back,
which the north star names as "a trivial RCCL scatter/gather over xGMI": here
torch.distributed's scatter/gather, which on ROCm's "nccl" backend is RCCL
(grouped point-to-point sends over xGMI).  It is timed separately from the
kernel scaling curve (8(e): at 8 GPUs it moves 7/8 of the batch out of rank 0).

The reference has no multi-device notion: JeroMQ encrypts on its IO threads,
one connection at a time (StreamEngine.java:809,1061).
"""
import numpy as np
import torch
import torch.distributed as dist


def frame_range(rank, world, total_frames):
    """Contiguous range [first, first+count) of rank's frames (uniform frames: by count)."""
    base, extra = divmod(total_frames, world)
    first = rank * base + min(rank, extra)
    return first, base + (1 if rank < extra else 0)


def balance_by_bytes(lens, world):
    """Contiguous frame ranges with near-equal payload bytes (ragged batches, 8(e):
    "balance by sum of bytes, not frame count").  Returns world+1 boundaries b with
    rank r owning frames [b[r], b[r+1])."""
    lens = np.asarray(lens, dtype=np.int64)
    if world <= 1 or len(lens) == 0:
        return [0, len(lens)] + [len(lens)] * max(world - 1, 0)
    csum = np.concatenate([[0], np.cumsum(lens + 33)])  # work ~ body bytes
    targets = csum[-1] * np.arange(1, world) / world
    cuts = np.searchsorted(csum, targets, side="left")
    b = [0] + [int(c) for c in cuts] + [len(lens)]
    for i in range(1, len(b)):  # monotone even for empty shards
        b[i] = max(b[i], b[i - 1])
    return b


def scatter_shards(shard, full=None, src=0, group=None):
    """Rank `src` holds `full` (world * shard.numel() bytes, rank r's shard at r*shard.numel());
    every rank receives its shard into `shard`.  Collective: every rank calls it.  group: the
    process group that carries the bytes (an RCCL group for device tensors; None = the default)."""
    world = dist.get_world_size(group)
    if dist.get_rank() == src:
        if full is None or full.numel() != world * shard.numel():
            raise ValueError("scatter_shards: full must hold world * shard bytes on the source rank")
        parts = list(full.view(world, -1).unbind(0))
        dist.scatter(shard, scatter_list=parts, src=src, group=group)
    else:
        dist.scatter(shard, src=src, group=group)


def gather_shards(shard, full=None, dst=0, group=None):
    """Inverse of scatter_shards: rank `dst` receives every rank's shard into `full`."""
    world = dist.get_world_size(group)
    if dist.get_rank() == dst:
        if full is None or full.numel() != world * shard.numel():
            raise ValueError("gather_shards: full must hold world * shard bytes on the destination rank")
        parts = list(full.view(world, -1).unbind(0))
        dist.gather(shard, gather_list=parts, dst=dst, group=group)
    else:
        dist.gather(shard, dst=dst, group=group)


def timed(fn, world, device_sync=True):
    """Run fn between barriers of the default group; return the slowest rank's wall time in
    seconds (the reduction on the default group's device: host for gloo)."""
    import time
    dist.barrier()
    if device_sync and torch.cuda.is_available():
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    if device_sync and torch.cuda.is_available():
        torch.cuda.synchronize()
    dist.barrier()
    dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64,
                      device="cuda" if dist.get_backend() == "nccl" else "cpu")
    dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    return float(dt.item())
