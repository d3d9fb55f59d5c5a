"""One rank of bench.py's N-rank path on CPU (gloo), launched by bench.launch_ranks exactly as
`python bench.py --gpus N` launches the GPU ranks (tests/test_bench_launch.py).

It runs bench.py's own distributed pieces — rank setup, RCCL/gloo key broadcast, the global-batch
shard (config D: contiguous; config E: byte quantiles), the sampled global indices, the checksum
all-reduce, and rank 0's oracle check — with the CPU oracle standing in for the device seal (this
is test code: the bench itself seals on the GPU). Rank 0 writes what it saw to $MQ_TEST_OUT as
JSON; every rank writes its shard's range and wire bytes next to it."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import bench  # noqa: E402
from milli_quic_amd import shard  # noqa: E402
from oracle import oracle  # noqa: E402


def main():
    args = bench.parse(sys.argv[1:])
    rank, world, _ = bench.init_dist("gloo")
    dd = dist if world > 1 else None
    keys = bench.rank_keys(args.config, args.keys, dd, "cpu")
    w, first = bench.build_shard(args.config, args.packets, rank, world, keys)
    oracle.load()
    st = oracle.batch_seal(w.keys, w.arena, w.seal_desc, w.suite_hint, threads=2)
    st2, pn = oracle.batch_open(w.keys, w.arena, w.open_desc, w.suite_hint, threads=2)
    fails = int((st != 0).sum() + (st2 != 0).sum()) + int((pn != w.pns).sum())
    arena = torch.from_numpy(w.arena)
    offs = torch.from_numpy(w.seal_desc["offset"].astype(np.int64))
    lens = torch.from_numpy(w.seal_desc["len"].astype(np.int64))
    g, local = bench.sample_for_rank(args.packets * world, first, w.n)
    ls = torch.from_numpy(local.astype(np.int64))
    csum = shard.tag_checksum_torch(arena, offs, lens)
    s_csum = shard.tag_checksum_torch(arena, offs[ls], lens[ls])
    if os.environ.get("MQ_TEST_CORRUPT_RANK") == str(rank):  # a wrong result on one rank
        s_csum += 1
    pn_ok = bool((pn == w.pns).all())
    parity = bench.parity_check(args.config, args.packets * world, g, keys, fails, csum, s_csum, pn_ok, dd)
    tot = shard.reduce_totals(0.25 * (rank + 1), w.wire_bytes, 0, dd)
    if rank == 0:
        o_fail, o_csum = bench.oracle_sample_checksum(args.config, args.packets * world, g, keys)
        with open(os.environ["MQ_TEST_OUT"], "w") as f:
            json.dump({"world": world, "fails": parity["failures"], "csum": parity["tag_checksum"],
                       "sample_csum": parity["sample_tag_checksum"], "oracle_sample_csum": o_csum,
                       "oracle_fail": o_fail, "n_sample": int(len(g)), "parity": parity,
                       "elapsed": tot.elapsed, "wire": tot.wire_bytes, "key_rows": len(w.keys),
                       "first_pn": int(w.pns[0])}, f)
    with open(os.environ["MQ_TEST_OUT"] + f".match{rank}", "w") as f:
        f.write("1" if parity["match"] else "0")
    with open(os.environ["MQ_TEST_OUT"] + f".shard{rank}", "w") as f:
        json.dump({"first": int(first), "n": int(w.n), "wire": int(w.wire_bytes), "csum": int(csum)}, f)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
