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


def tag_checksum_torch(arena, offsets, lens):
    """tag_checksum() on torch tensors (device-resident arena, int64 offsets / lens of the packets
    to cover): the same sum of the tags' little-endian 16-bit words, computed where the arena
    lives (the bench's arena never leaves HBM)."""
    import torch
    if offsets.numel() == 0:
        return 0
    end = offsets.to(torch.int64) + lens.to(torch.int64)
    idx = (end - 16)[:, None] + torch.arange(16, device=end.device, dtype=torch.int64)[None, :]
    tags = arena[idx.reshape(-1)].to(torch.int64).reshape(-1, 16)
    return int((tags[:, 0::2] + (tags[:, 1::2] << 8)).sum().item())


def keys_to_bytes(rows):
    """Serialise key rows (mq_key_material, 88 B each) for a broadcast."""
    import ctypes
    return b"".join(ctypes.string_at(ctypes.addressof(r), ctypes.sizeof(r)) for r in rows)


def keys_from_bytes(blob):
    from . import _lib
    import ctypes
    sz = ctypes.sizeof(_lib.KeyMaterial)
    if len(blob) % sz:
        raise ValueError("key blob is not a whole number of mq_key_material rows")
    return [_lib.KeyMaterial.from_buffer_copy(blob[k:k + sz]) for k in range(0, len(blob), sz)]


def broadcast_keys(rows, dist=None, device=None):
    """Rank 0's key rows on every rank (torch.distributed broadcast: RCCL over xGMI on the GPU box,
    a device tensor; gloo in the CPU tests, a host tensor). Non-zero ranks pass rows=None."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return list(rows)
    import torch
    if dist.get_backend() != "nccl":
        device = "cpu"
    n = torch.tensor([len(keys_to_bytes(rows)) if dist.get_rank() == 0 else 0], dtype=torch.int64, device=device)
    dist.broadcast(n, src=0)
    if dist.get_rank() == 0:
        buf = torch.frombuffer(bytearray(keys_to_bytes(rows)), dtype=torch.uint8).to(device)
    else:
        buf = torch.empty(int(n.item()), dtype=torch.uint8, device=device)
    dist.broadcast(buf, src=0)
    return keys_from_bytes(buf.cpu().numpy().tobytes())


def reduce_sums(values, dist=None, device=None):
    """Whole-job sums of integer counters (failures, tag checksums) — exact int64 all-reduce."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return [int(v) for v in values]
    import torch
    if dist.get_backend() != "nccl":
        device = "cpu"
    t = torch.tensor([int(v) for v in values], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return [int(x) for x in t.cpu().tolist()]


def sample_indices(n_total, target=4096):
    """The fixed sample of global packet indices a sharded run checks against the oracle: every
    stride-th packet, stride = max(1, n_total // target)."""
    stride = max(1, n_total // target)
    return np.arange(0, n_total, stride, dtype=np.int64)


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
