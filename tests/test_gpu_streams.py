"""Batch calls on stream handles that do not name one stream: hipStreamPerThread from
several host threads at once, and a stream under graph capture. The persistent AES kernels' dynamic
tile schedule keeps one slot of device words per stream handle; such launches must take the static
stride (mq_host.cpp sched_slot), or two kernels sharing a slot skip or repeat tiles. Every byte and
status is compared with the oracle (reference composites: transmit.rs:625-755, recv.rs:340-421)."""
import threading

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from milli_quic_amd import _lib, batch, workload  # noqa: E402
from milli_quic_amd.batch import KeyTable  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
PER_THREAD = 2  # hipStreamPerThread


@pytest.fixture(scope="module", autouse=True)
def _device(mqlib):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    assert mqlib.mq_device_init(0) == 0


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).copy()).to(DEV)


def test_per_thread_stream_from_two_threads(orc):
    # AES over 3 keys: partition + key-uniform persistent tiles, both with schedule slots normally
    ws_all = [workload.uniform(1 << 15, _lib.MQ_SUITE_AES128GCM, n_keys=3, start=k << 15) for k in range(2)]
    refs = []
    for w in ws_all:
        ref = w.arena.copy()
        assert (orc.batch_seal(w.keys, ref, w.seal_desc, w.suite_hint, threads=8) == 0).all()
        refs.append(ref)
    out, errs = [None, None], []

    def worker(k):
        try:
            lib = _lib.load()
            assert lib.mq_device_init(0) == 0
            torch.cuda.set_device(0)
            w = ws_all[k]
            kt = KeyTable(w.keys)
            a, sd, od = _dev(w.arena), _dev(w.seal_desc), _dev(w.open_desc)
            st = torch.full((w.n,), 0xEE, dtype=torch.uint8, device=DEV)
            pn = torch.zeros(w.n, dtype=torch.int64, device=DEV)
            ws = torch.empty(batch.workspace_bytes(w.n), dtype=torch.uint8, device=DEV)
            torch.cuda.synchronize()
            bad = 0
            # overlapping seal/open rounds of the two threads; torch's own ops run on its stream,
            # so every hand-over between the two goes through a device-wide synchronize
            for _ in range(4):
                batch.seal(kt, a, sd, st, w.suite_hint, ws, stream=PER_THREAD)
                torch.cuda.synchronize()
                bad += int((st != 0).sum())
                batch.open_(kt, a, od, st, pn, w.suite_hint, ws, stream=PER_THREAD)
                torch.cuda.synchronize()
                bad += int((st != 0).sum())
            batch.seal(kt, a, sd, st, w.suite_hint, ws, stream=PER_THREAD)
            torch.cuda.synchronize()
            out[k] = (a.cpu().numpy(), st.cpu().numpy(), bad)
        except Exception as e:  # noqa: BLE001 - reported below
            errs.append(e)

    th = [threading.Thread(target=worker, args=(k,)) for k in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs
    for k in range(2):
        arena, st, bad = out[k]
        assert (st == 0).all() and bad == 0
        assert arena.tobytes() == refs[k].tobytes()


def test_graph_capture_single_key(orc):
    w = workload.config_c(1 << 14)
    ref = w.arena.copy()
    assert (orc.batch_seal(w.keys, ref, w.seal_desc, w.suite_hint, threads=8) == 0).all()
    kt = KeyTable(w.keys)
    a, sd, od = _dev(w.arena), _dev(w.seal_desc), _dev(w.open_desc)
    st = torch.full((w.n,), 0xEE, dtype=torch.uint8, device=DEV)
    pn = torch.zeros(w.n, dtype=torch.int64, device=DEV)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):  # captured on torch's capture stream: no schedule slot
        batch.seal(kt, a, sd, st, w.suite_hint, None)
    g.replay()
    torch.cuda.synchronize()
    assert (st.cpu().numpy() == 0).all()
    assert a.cpu().numpy().tobytes() == ref.tobytes()
    # open (the plaintext is back; the tag room keeps the tag), then seal again by replaying the
    # graph: the same sealed bytes
    batch.open_(kt, a, od, st, pn, w.suite_hint, None)
    torch.cuda.synchronize()
    assert (st.cpu().numpy() == 0).all()
    body = w.arena.reshape(w.n, 1200)[:, :1184].tobytes()
    assert a.cpu().numpy().reshape(w.n, 1200)[:, :1184].tobytes() == body
    g.replay()
    torch.cuda.synchronize()
    assert a.cpu().numpy().tobytes() == ref.tobytes()
