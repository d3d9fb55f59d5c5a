"""Multi-GPU sharding of a packet batch: one process per GPU, no data-path
collective.

QUIC packets are independent, so a batch of N packets is split into contiguous descriptor
ranges, one per rank; every rank protects / opens its own range in its own HBM. Uniform
batches split by count; mixed-length batches split at byte quantiles of the prefix sum of the
packet lengths, so every rank gets about sum(L) / world wire bytes. The only
cross-rank traffic is control: a barrier around the timed region and the reduction of the
timing and counters (max of elapsed, sums of bytes and failures) — done here with
torch.distributed, which is RCCL ("nccl") on the GPU box and gloo in the CPU tests.
"""
from dataclasses import dataclass

import numpy as np


def shard_range(n_total, rank, world):
    """Contiguous [lo, hi) descriptor range of `rank` (sizes differ by at most one)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, extra = divmod(n_total, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def shard_range_bytes(lengths, rank, world):
    """Contiguous [lo, hi) descriptor range of `rank` holding about sum(lengths) / world bytes.

    Rank r's range starts at the first packet whose byte prefix reaches r * total / world, so
    each rank's byte count differs from the ideal share by less than one packet length."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    L = np.asarray(lengths, dtype=np.int64)
    if len(L) == 0:
        return 0, 0
    prefix = np.concatenate(([0], np.cumsum(L)))  # prefix[i] = bytes before packet i
    total = int(prefix[-1])

    def cut(r):
        if r <= 0:
            return 0
        if r >= world:
            return len(L)
        return int(np.searchsorted(prefix, (total * r) // world, side="left"))

    return cut(rank), cut(rank + 1)


def shard_batch(arena, desc, rank, world, balance="count"):
    """This rank's slice of a host batch: (arena bytes, descriptors rebased to that slice).

    balance="count" splits the descriptors evenly, "bytes" at byte quantiles of their lengths.
    The slice spans the byte range covered by the rank's descriptors (they need not be sorted),
    so every packet of the shard keeps its bytes and nothing of other shards is copied."""
    if balance == "count":
        lo, hi = shard_range(len(desc), rank, world)
    elif balance == "bytes":
        lo, hi = shard_range_bytes(desc["len"], rank, world)
    else:
        raise ValueError("balance must be 'count' or 'bytes'")
    d = desc[lo:hi].copy()
    if len(d) == 0:
        return arena[:0].copy(), d
    start = int(d["offset"].min())
    end = int((d["offset"].astype(np.int64) + d["len"].astype(np.int64)).max())
    start &= ~15  # keep the arena's 16-B chunk alignment (the staging works in 16-B chunks)
    d["offset"] -= start
    return arena[start:end].copy(), d


def tag_checksum(arena, desc):
    """Checksum of the 16-B tags of a sealed batch: the sum of their little-endian 16-bit words.

    Sums of per-shard checksums equal the checksum of the whole batch (a size-independent
    parity property of sharding: a checksum of checksums); exact in float64 up to 2^34 packets."""
    if len(desc) == 0:
        return 0
    end = desc["offset"].astype(np.int64) + desc["len"].astype(np.int64)
    idx = end[:, None] - 16 + np.arange(16)[None, :]
    tags = arena[idx].astype(np.int64)
    return int((tags[:, 0::2] + (tags[:, 1::2] << 8)).sum())


def reduce_checksum(value, dist=None, device=None):
    """Whole-job sum of per-rank tag checksums."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return int(value)
    import torch
    if dist.get_backend() != "nccl":
        device = "cpu"
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return int(t[0])


@dataclass
class Totals:
    elapsed: float   # max over ranks (seconds)
    wire_bytes: int  # sum over ranks
    failures: int    # sum over ranks


def reduce_totals(elapsed, wire_bytes, failures, dist=None, device=None):
    """Whole-job totals of one timed run: max elapsed, summed bytes and failures."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return Totals(float(elapsed), int(wire_bytes), int(failures))
    import torch
    if dist.get_backend() != "nccl":
        device = "cpu"  # gloo reduces host tensors
    t_max = torch.tensor([float(elapsed)], dtype=torch.float64, device=device)
    t_sum = torch.tensor([float(wire_bytes), float(failures)], dtype=torch.float64, device=device)
    dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
    dist.all_reduce(t_sum, op=dist.ReduceOp.SUM)
    return Totals(float(t_max[0]), int(t_sum[0]), int(t_sum[1]))
