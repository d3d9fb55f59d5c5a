"""configs[3] — 8M x 1200-B ChaCha20-Poly1305, one global batch sharded over 8 GPUs — on the HIP path.

bench.py's own config-D code (rank_keys, build_shard, sample_for_rank) builds shards s = 0 and
s = 7 of the 8 x 2^20 global batch (rank 7 holds global indices 7 x 2^20 .. 8 x 2^20 - 1: PNs up
to 0x107FFFFF) on this one GPU; each is sealed and opened on the device as the bench does, and
every byte of that shard's members of the fixed global sample (shard.sample_indices) must equal
the oracle sealing exactly those global packets (workload.uniform_at). The per-GPU device model
(mq_device_init per thread, key tables bound to their device, side streams per caller stream) is
exercised alongside."""
import ctypes
import threading

import numpy as np
import pytest

torch = pytest.importorskip("torch")

import bench  # noqa: E402
from milli_quic_amd import _lib, batch, shard, workload  # noqa: E402
from milli_quic_amd.batch import KeyTable  # noqa: E402

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
N, WORLD = 1 << 20, 8


@pytest.fixture(scope="module", autouse=True)
def _device(mqlib):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    assert mqlib.mq_device_init(0) == 0


def to_dev(a):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8)).to(DEV)


@pytest.mark.parametrize("rank,keys", [(0, 1), (7, 1), (7, 1024)])
def test_config_d_shard_vs_oracle(orc, rank, keys):
    k = bench.rank_keys("b", keys, None, DEV)
    w, first = bench.build_shard("b", N, rank, WORLD, k)
    assert first == rank * N
    assert int(w.pns[0]) == workload.PN0 + rank * N and int(w.pns[-1]) == workload.PN0 + (rank + 1) * N - 1
    kt = KeyTable(w.keys)
    a, sd, od = to_dev(w.arena), to_dev(w.seal_desc), to_dev(w.open_desc)
    st = torch.full((N,), 0xEE, dtype=torch.uint8, device=DEV)
    pn = torch.zeros(N, dtype=torch.int64, device=DEV)
    ws = torch.empty(max(batch.workspace_bytes(N), 256), dtype=torch.uint8, device=DEV)
    batch.seal(kt, a, sd, st, w.suite_hint, ws)
    torch.cuda.synchronize()
    assert int((st != 0).sum()) == 0
    g, local = bench.sample_for_rank(N * WORLD, first, N)
    assert len(g) == 4096 and len(local) == 4096 // WORLD
    mine = g[(g >= rank * N) & (g < (rank + 1) * N)]
    sw = workload.uniform_at(mine, w.suite_hint, keys=w.keys)
    o_st = orc.batch_seal(sw.keys, sw.arena, sw.seal_desc, sw.suite_hint, threads=8)
    assert (o_st == 0).all()
    sealed = a.cpu().numpy().reshape(N, 1200)
    assert sealed[local].tobytes() == sw.arena.tobytes()
    # this shard's share of the sampled-tag checksum the bench all-reduces
    offs = torch.from_numpy(w.seal_desc["offset"].astype(np.int64)).to(DEV)
    lens = torch.from_numpy(w.seal_desc["len"].astype(np.int64)).to(DEV)
    ls = torch.from_numpy(local.astype(np.int64)).to(DEV)
    assert shard.tag_checksum_torch(a, offs[ls], lens[ls]) == shard.tag_checksum(sw.arena, sw.seal_desc)
    batch.open_(kt, a, od, st, pn, w.suite_hint, ws)
    torch.cuda.synchronize()
    assert int((st != 0).sum()) == 0
    assert (pn.cpu().numpy().view(np.uint64) == w.pns).all()
    back = a.cpu().numpy().reshape(N, 1200)[:, :1184]
    assert back.tobytes() == w.arena.reshape(N, 1200)[:, :1184].tobytes()


def test_device_selection_is_per_thread(mqlib):
    # the thread's selection survives a failed one; the library hands the caller's HIP device back
    # after every call (it runs each call on its object's device under a guard)
    assert mqlib.mq_device_current() == 0
    n_dev = torch.cuda.device_count()
    assert mqlib.mq_device_init(n_dev) == _lib.MQ_ERR_NO_DEVICE and mqlib.mq_device_current() == 0
    w = workload.config_b(64)
    kt = KeyTable(w.keys)
    assert mqlib.mq_keytable_device(kt.handle) == 0
    seen = {}

    def other():  # a thread that selected nothing follows its current HIP device (0)
        seen["cur"] = mqlib.mq_device_current()
        seen["init"] = mqlib.mq_device_init(0)

    t = threading.Thread(target=other)
    t.start()
    t.join()
    assert seen == {"cur": 0, "init": 0}
    a = to_dev(w.arena)
    st = torch.zeros(w.n, dtype=torch.uint8, device=DEV)
    batch.seal(kt, a, to_dev(w.seal_desc), st, w.suite_hint)
    torch.cuda.synchronize()
    assert int((st != 0).sum()) == 0 and torch.cuda.current_device() == 0


def test_mixed_batches_on_two_streams(orc):
    # two caller streams pipelining mixed batches concurrently: each stream forks its own side
    # streams (no false dependency through a shared one), results equal the oracle; then the
    # streams' side-stream sets are released
    ws_list, outs = [], []
    streams = [torch.cuda.Stream(device=DEV) for _ in range(2)]
    loads = [workload.config_e(6000, seed=21 + k) for k in range(2)]
    for _ in range(3):  # several rounds: the side streams are reused per caller stream
        outs = []
        for s, w in zip(streams, loads):
            with torch.cuda.stream(s):
                kt = KeyTable(w.keys)
                a = to_dev(w.arena)
                st = torch.full((w.n,), 0xEE, dtype=torch.uint8, device=DEV)
                ws = torch.empty(max(batch.workspace_bytes(w.n), 256), dtype=torch.uint8, device=DEV)
                batch.seal(kt, a, to_dev(w.seal_desc), st, w.suite_hint, ws, s.cuda_stream)
                outs.append((w, kt, a, st, ws))
        torch.cuda.synchronize()
        for (w, kt, a, st, ws) in outs:
            ref = w.arena.copy()
            o_st = orc.batch_seal(w.keys, ref, w.seal_desc, w.suite_hint, threads=8)
            assert (o_st == 0).all() and (st.cpu().numpy() == 0).all()
            assert a.cpu().numpy().tobytes() == ref.tobytes()
    lib = _lib.load()
    for s in streams:
        lib.mq_stream_release(ctypes.c_void_p(s.cuda_stream))
    torch.cuda.synchronize()
