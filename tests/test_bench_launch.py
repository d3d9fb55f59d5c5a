"""bench.py's N-GPU path on CPU (world 2, gloo): `bench.launch_ranks` starts the ranks as
`python bench.py --gpus N` does (torch.distributed.run in a child process), and the ranks run
bench.py's key broadcast, global-batch sharding (config D: rank s = packets [s n, (s+1) n) of one
batch), checksum all-reduce and rank 0's sampled oracle check (tests/dist_bench_worker.py; the
oracle stands in for the device seal there)."""
import json
import os

import numpy as np
import pytest

pytest.importorskip("torch")

import bench  # noqa: E402
from milli_quic_amd import _lib, shard, workload  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.parametrize("keys", [1, 5])
def test_launch_two_ranks_sharded_global_batch(tmp_path, orc, keys):
    out = tmp_path / "r0.json"
    os.environ["MQ_TEST_OUT"] = str(out)
    n = 1500
    rc = bench.launch_ranks(2, ["--gpus", "2", "--packets", str(n), "--keys", str(keys)],
                            script=os.path.join(HERE, "dist_bench_worker.py"))
    assert rc == 0
    r = json.loads(out.read_text())
    assert r["world"] == 2 and r["fails"] == 0 and r["key_rows"] == keys
    assert r["first_pn"] == workload.PN0  # rank 0 holds global packets 0..n-1
    # the sampled global indices span both ranks; the ranks' reduced checksum equals the oracle's
    assert r["n_sample"] == len(shard.sample_indices(2 * n)) and r["oracle_fail"] == 0
    assert r["sample_csum"] == r["oracle_sample_csum"]
    # the two shards are exactly the single-process global batch of 2n packets
    w = workload.uniform(2 * n, 2, keys=workload.uniform_keys(2, keys))
    st = orc.batch_seal(w.keys, w.arena, w.seal_desc, w.suite_hint, threads=4)
    assert (st == 0).all()
    assert r["csum"] == shard.tag_checksum(w.arena, w.seal_desc)
    assert r["wire"] == 2 * n * 1200 and r["elapsed"] == 0.5  # summed bytes, max of elapsed
    assert r["parity"]["match"] and all((tmp_path / f"r0.json.match{k}").read_text() == "1" for k in (0, 1))


@pytest.mark.parametrize("corrupt", [None, 1])
def test_launch_two_ranks_config_e(tmp_path, orc, corrupt):
    # config E over N ranks is ONE global mixed batch of N x n packets split at
    # byte quantiles of the packet lengths; rank 0's oracle checks the global sample
    # the ranks all-reduce, so a correct 2-rank run matches and a wrong result on rank 1 does not
    out = tmp_path / "r0.json"
    os.environ["MQ_TEST_OUT"] = str(out)
    if corrupt is None:
        os.environ.pop("MQ_TEST_CORRUPT_RANK", None)
    else:
        os.environ["MQ_TEST_CORRUPT_RANK"] = str(corrupt)
    n = 700
    try:
        rc = bench.launch_ranks(2, ["--gpus", "2", "--packets", str(n), "--config", "e"],
                                script=os.path.join(HERE, "dist_bench_worker.py"))
    finally:
        os.environ.pop("MQ_TEST_CORRUPT_RANK", None)
    assert rc == 0
    r = json.loads(out.read_text())
    assert r["world"] == 2 and r["fails"] == 0 and r["oracle_fail"] == 0
    p = r["parity"]
    assert p["match"] == (corrupt is None)
    assert (p["sample_tag_checksum"] == r["oracle_sample_csum"]) == (corrupt is None)
    # every rank reaches the same verdict
    assert {(tmp_path / f"r0.json.match{k}").read_text() for k in (0, 1)} == {"1" if corrupt is None else "0"}
    # the shards tile the global batch at its byte median, and hold exactly its packets
    sh = [json.loads((tmp_path / f"r0.json.shard{k}").read_text()) for k in (0, 1)]
    w = workload.config_e(2 * n)
    assert sh[0]["first"] == 0 and sh[1]["first"] == sh[0]["n"] and sh[0]["n"] + sh[1]["n"] == 2 * n
    L = w.seal_desc["len"].astype(np.int64)
    assert sh[0]["wire"] == int(L[:sh[0]["n"]].sum()) and sh[1]["wire"] == int(L[sh[0]["n"]:].sum())
    assert abs(sh[0]["wire"] - sh[1]["wire"]) <= 2 * int(L.max())  # byte-balanced, not count-balanced
    assert shard.shard_range_bytes(L, 1, 2) == (sh[1]["first"], 2 * n)
    st = orc.batch_seal(w.keys, w.arena, w.seal_desc, w.suite_hint, threads=4)
    assert (st == 0).all()
    if corrupt is None:
        assert sh[0]["csum"] + sh[1]["csum"] == shard.tag_checksum(w.arena, w.seal_desc)


def test_sample_indices_and_shard_positions():
    for n, world in ((1 << 20, 8), (1000, 3), (5, 2)):
        g = shard.sample_indices(n * world)
        got = []
        for rank in range(world):
            gs, local = bench.sample_for_rank(n * world, rank * n, n)
            assert (gs == g).all() and ((local >= 0) & (local < n)).all()
            got.append(local + rank * n)
        assert (np.concatenate(got) == g).all()
    assert len(shard.sample_indices(8 << 20)) == 4096


def test_roofline_seal_composite_traffic():
    """roofline.kernel / traffic name the seal composite the bench's event time covers: the tile
    kernel ("1" variant for a one-row key table; both suites' tiles apply header protection
    themselves since r03), or for partitioned batches the partition launches and the tile kernels
    mq_host.cpp picks; the PMC traffic is the sum of those kernels' per-launch HBM bytes from
    profiles/pmc_traffic_<cfg>.json."""
    assert bench.seal_kernels("b", 1) == ("mq_chacha_seal1_kernel",)  # HP inside the tile (r03)
    assert bench.seal_kernels("b", 1024) == ("mq_chacha_seal_kernel",)
    # single-key AES: 4 lanes per 1200-B packet, 2 per 64-B packet, 8 over 1536 B (r06 narrow tiles)
    assert bench.seal_kernels("c", 1) == ("mq_aes_seal1n_kernel",)
    assert bench.seal_kernels("c", 1, 1 << 20, None, 64 << 20) == ("mq_aes_seal1n2_kernel",)
    assert bench.seal_kernels("c", 1, 1 << 20, None, 2048 << 20) == ("mq_aes_seal1_kernel",)
    # the hot AES key's segment on the slice kernel (4 lanes per packet) beside the multi-key kernel
    hot = ("mq_aes_sealsn_kernel", "mq_aes_seal_kernel")
    assert bench.seal_kernels("e", 4098) == bench.PARTITION + hot + ("mq_chacha_seal_lgrid_kernel",)
    # config E's table has one non-AES row: its ChaCha20 list runs on the single-key kernel
    assert bench.seal_kernels("e", 4098, 1 << 20, 1) == bench.PARTITION + hot + ("mq_chacha_seal_lgrid1_kernel",)
    # 1024 keys over 2^20 packets (>= 512 per row): the key-segmented kernel runs list 0 (r03);
    # 4096 keys: the hot split and the multi-key kernel
    assert bench.seal_kernels("c", 1024) == bench.PARTITION + ("mq_aes_sealsn_kernel", "mq_aes_seal_kernel")
    assert bench.seal_kernels("c", 4096) == bench.PARTITION + hot + ("mq_aes_seal_kernel",)
    with _lib.option("MQ_AES_NARROW", 0), _lib.option("MQ_AES_HOT_SEG", 0):
        assert bench.seal_kernels("c", 1) == ("mq_aes_seal1_kernel",)
        assert bench.seal_kernels("c", 4096) == bench.PARTITION + ("mq_aes_seal1_kernel", "mq_aes_seal_kernel",
                                                                   "mq_aes_seal_kernel")
    assert bench.kernel_key("void mq_mixed_hp_kernel(mq::KeyRow const*, unsigned int)") == "mq_mixed_hp_kernel"
    for cfg in ("b", "c"):
        ks = bench.seal_kernels(cfg, 1)
        with open(os.path.join(HERE, "..", "profiles", f"pmc_traffic_{cfg}.json")) as f:
            d = {k.split("(")[0]: v["hbm_bytes_per_launch"] for k, v in json.load(f)["kernels"].items()}
        assert bench.load_traffic(cfg, ks) == int(sum(d[k] for k in ks))
