"""N>1 path on CPU (gloo, world_size 2): sharding of a batch across ranks and the whole-job
reductions bench.py uses (packets are independent, no data-path collective).

Each rank seals + opens its own shard with the CPU oracle (the checker) and the ranks' results,
gathered, must equal the single-process result on the whole batch — i.e. sharding changes
nothing about the bytes, and the reductions give max-elapsed / summed bytes and failures.
"""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

from milli_quic_amd import shard, workload  # noqa: E402


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _span(w, rank, world, balance):
    if balance == "bytes":
        return shard.shard_range_bytes(w.seal_desc["len"], rank, world)
    return shard.shard_range(w.n, rank, world)


def _worker(rank, world, port, n, out_dir, balance):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle
    w = workload.config_e(n, seed=0xABCD)  # every rank builds the same global batch
    arena, desc = shard.shard_batch(w.arena, w.seal_desc, rank, world, balance=balance)
    st = oracle.batch_seal(w.keys, arena, desc, w.suite_hint, threads=2)
    csum = shard.reduce_checksum(shard.tag_checksum(arena, desc), dist)
    lo, hi = _span(w, rank, world, balance)
    odesc = w.open_desc[lo:hi].copy()
    odesc["offset"] = desc["offset"]
    sealed = arena.copy()
    st2, pn = oracle.batch_open(w.keys, arena, odesc, w.suite_hint, threads=2)
    tot = shard.reduce_totals(0.5 + rank, int(desc["len"].astype(np.int64).sum()),
                              int((st != 0).sum() + (st2 != 0).sum()), dist)
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), sealed=sealed, desc=desc, st=st, st2=st2, pn=pn,
             tot=np.array([tot.elapsed, tot.wire_bytes, tot.failures], dtype=np.float64),
             csum=np.array([csum], dtype=np.int64))
    dist.barrier()
    dist.destroy_process_group()


def test_shard_range_covers_batch():
    for n in (0, 1, 7, 1000, 1 << 20):
        for world in (1, 2, 3, 8):
            spans = [shard.shard_range(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [hi - lo for lo, hi in spans]
            assert max(sizes) - min(sizes) <= 1


def test_reduce_totals_single_process():
    t = shard.reduce_totals(1.5, 100, 2)
    assert (t.elapsed, t.wire_bytes, t.failures) == (1.5, 100, 2)


def test_shard_range_bytes_balances_bytes():
    rng = np.random.default_rng(7)
    for n in (0, 1, 5, 1000, 20000):
        L = rng.integers(64, 1351, size=n)
        for world in (1, 2, 3, 8):
            spans = [shard.shard_range_bytes(L, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            if n >= world * 10:
                share = L.sum() / world
                for lo, hi in spans:  # within one packet of the ideal share at either end
                    assert abs(int(L[lo:hi].sum()) - share) <= 2 * L.max()


@pytest.mark.parametrize("balance", ["count", "bytes"])
def test_two_rank_gloo_shards_match_single_process(tmp_path, balance):
    n, world = 3000, 2
    mp.spawn(_worker, args=(world, _free_port(), n, str(tmp_path), balance), nprocs=world, join=True)
    from oracle import oracle
    w = workload.config_e(n, seed=0xABCD)
    whole = w.arena.copy()
    st_all = oracle.batch_seal(w.keys, whole, w.seal_desc.copy(), w.suite_hint, threads=2)
    assert (st_all == 0).all()
    whole_csum = shard.tag_checksum(whole, w.seal_desc)
    total_wire = 0
    for r in range(world):
        z = np.load(tmp_path / f"r{r}.npz")
        assert int(z["csum"][0]) == whole_csum  # checksum of the shards' checksums
        lo, hi = _span(w, r, world, balance)
        assert (z["st"] == 0).all() and (z["st2"] == 0).all()
        assert (z["pn"] == w.pns[lo:hi]).all()
        for k in range(hi - lo):  # every sealed packet of the shard equals the whole-batch seal
            o, ln = int(z["desc"]["offset"][k]), int(z["desc"]["len"][k])
            go = int(w.seal_desc["offset"][lo + k])
            assert z["sealed"][o:o + ln].tobytes() == whole[go:go + ln].tobytes()
        total_wire += int(z["desc"]["len"].astype(np.int64).sum())
        elapsed, wire, fails = z["tot"]
        assert elapsed == 1.5 and fails == 0  # max over ranks (0.5, 1.5); summed failures
    assert int(wire) == total_wire == int(w.seal_desc["len"].astype(np.int64).sum())


def test_config_e_ranges_are_slices_of_the_global_batch():
    """workload.config_e(n, lo=, hi=) and config_e_at(): a shard or a sample of the mixed batch is
    built on its own and equals its part of the whole (bench.py's sharded config E)."""
    from milli_quic_amd import workload
    n = 3000
    whole = workload.config_e(n, seed=11)
    L = whole.seal_desc["len"].astype(np.int64)
    parts = [shard.shard_range_bytes(L, r, 3) for r in range(3)]
    assert parts[0][0] == 0 and parts[-1][1] == n
    for (lo, hi) in parts:
        r = workload.config_e(n, seed=11, lo=lo, hi=hi)
        base = int(whole.seal_desc["offset"][lo]) & ~15
        assert r.n == hi - lo and (r.pns == whole.pns[lo:hi]).all()
        for f in ("len", "key_id", "pn", "pn_offset", "pn_len", "flags"):
            assert (r.seal_desc[f] == whole.seal_desc[f][lo:hi]).all()
        assert (r.seal_desc["offset"].astype(np.int64) == whole.seal_desc["offset"][lo:hi].astype(np.int64) - base).all()
        assert r.arena.tobytes() == whole.arena[base:base + len(r.arena)].tobytes()
    g = np.array([0, 1, 977, n - 1])
    s = workload.config_e_at(g, n, seed=11)
    for k, i in enumerate(g):
        o, ln = int(whole.seal_desc["offset"][i]), int(L[i])
        so = int(s.seal_desc["offset"][k])
        assert s.arena[so:so + ln].tobytes() == whole.arena[o:o + ln].tobytes()
        assert s.seal_desc["key_id"][k] == whole.seal_desc["key_id"][i]
