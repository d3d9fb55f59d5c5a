"""Multi-GPU sharding of a packet batch: one process per GPU, no data-path
collective.

QUIC packets are independent, so a batch of N packets is split into contiguous descriptor
ranges, one per rank; every rank protects / opens its own range in its own HBM. The only
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


def shard_batch(arena, desc, rank, world):
    """This rank's slice of a host batch: (arena bytes, descriptors rebased to that slice).

    The slice spans the byte range covered by the rank's descriptors (they need not be sorted),
    so every packet of the shard keeps its bytes and nothing of other shards is copied."""
    lo, hi = shard_range(len(desc), rank, world)
    d = desc[lo:hi].copy()
    if len(d) == 0:
        return arena[:0].copy(), d
    start = int(d["offset"].min())
    end = int((d["offset"].astype(np.int64) + d["len"].astype(np.int64)).max())
    start &= ~15  # keep the arena's 16-B chunk alignment (the staging works in 16-B chunks)
    d["offset"] -= start
    return arena[start:end].copy(), d


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
