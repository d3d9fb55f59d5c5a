"""Receive composite over raw datagrams on the GPU: mq_batch_recv against the
oracle's restatement of Connection::recv (recv.rs:189-510, 953-1025) — every packet record,
the updated connection table and every arena byte equal."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from milli_quic_amd import _lib, recv  # noqa: E402
from milli_quic_amd.batch import KeyTable  # noqa: E402

from recv_traffic import assemble, build_pn_jump, build_traffic  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _device(mqlib):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    assert mqlib.mq_device_init(0) == 0


def t(a):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1).copy()).to(DEV)


def gpu_recv(keys, conns, arena, dgrams, max_pkts):
    kt = KeyTable(keys)
    c, a = t(conns), t(arena)
    pk = torch.zeros(max_pkts * recv.PKT_DTYPE.itemsize, dtype=torch.uint8, device=DEV)
    n = torch.zeros(1, dtype=torch.int32, device=DEV)
    ws = torch.empty(recv.workspace_bytes(len(dgrams), max_pkts, len(conns)), dtype=torch.uint8, device=DEV)
    recv.recv(kt, c, a, t(dgrams), pk, n, ws)
    torch.cuda.synchronize()
    cnt = int(n.cpu()[0])
    return (pk.cpu().numpy().view(recv.PKT_DTYPE)[:min(cnt, max_pkts)], cnt, c.cpu().numpy().view(recv.CONN_DTYPE),
            a.cpu().numpy())


@pytest.mark.parametrize("seed,n_conns,n_app,tamper_flip", [(3, 6, 20, False), (11, 64, 60, False),
                                                            (5, 16, 30, True), (13, 4, 300, False),
                                                            (17, 3, 450, True), (19, 300, 12, False)])
def test_recv_vs_oracle(orc, seed, n_conns, n_app, tamper_flip):
    # tamper_flip: the first packet after a key-phase flip fails to open, so the
    # walk's speculation (it rotated there) is wrong; the next packet must be reported as the
    # reference's next-generation open (key_gen 2) and rotate the connection. The 300- / 450-packet
    # runs span several of the walk's 64-packet chunks (r04): chunks decided in parallel, chunks
    # replayed sequentially (PN-window crossings, the key update, tampered packets), and the later
    # walks' settled prefixes ending at a failed packet. 300 connections: the record sort takes two
    # 8-bit digit passes (r04's own stable radix sort)
    keys, conns, scripts = build_traffic(orc, seed=seed, n_conns=n_conns, n_app=n_app, tamper_flip=tamper_flip)
    arena, dgrams = assemble(orc, keys, conns, scripts, seed=seed)
    oc, oa = conns.copy(), arena.copy()
    o_pk, o_n = orc.batch_recv(keys, oc, oa, dgrams, 1 << 16)
    g_pk, g_n, gc, ga = gpu_recv(keys, conns, arena, dgrams, 1 << 16)
    assert g_n == o_n
    for f in recv.PKT_DTYPE.names:
        assert (g_pk[f] == o_pk[f]).all(), (f, np.nonzero(g_pk[f] != o_pk[f])[0][:10])
    assert gc.tobytes() == oc.tobytes()
    assert ga.tobytes() == oa.tobytes()


def test_recv_max_pkts_truncates(orc):
    keys, conns, scripts = build_traffic(orc, seed=5, n_conns=4, n_app=12)
    arena, dgrams = assemble(orc, keys, conns, scripts, seed=5, extras=False)
    o_pk, o_n = orc.batch_recv(keys, conns.copy(), arena.copy(), dgrams, 1 << 12)
    g_pk, g_n, _, _ = gpu_recv(keys, conns, arena, dgrams, 7)  # only the first 7 records are kept
    assert g_n == o_n and len(g_pk) == 7


def test_recv_speculation_opened_reference_fails(orc):
    # packets that open only under the batch's speculation (a PN decoded against a
    # corrupted packet's PN the reference never accepts) are MQ_ERR_CRYPTO, as in the reference,
    # and are re-sealed under the inputs that opened them: every arena byte equals the oracle's,
    # whose failed packets are never touched
    keys, conns, arena, dgrams = build_pn_jump(orc)
    oc, oa = conns.copy(), arena.copy()
    o_pk, o_n = orc.batch_recv(keys, oc, oa, dgrams, 1 << 10)
    st = o_pk["status"][:o_n]
    assert list(st[:7]) == [0, 0, 1, 1, 1, 0, 0] and list(st[7:14]) == [0, 0, 1, 1, 1, 0, 0]
    g_pk, g_n, gc, ga = gpu_recv(keys, conns, arena, dgrams, 1 << 10)
    assert g_n == o_n
    for f in recv.PKT_DTYPE.names:
        assert (g_pk[f] == o_pk[f][:o_n]).all(), (f, g_pk[f], o_pk[f][:o_n])
    assert gc.tobytes() == oc.tobytes()
    assert ga.tobytes() == oa.tobytes()
    # the failed packets' bytes are exactly as received
    for k in np.nonzero(st != 0)[0]:
        o, L = int(g_pk["offset"][k]), int(g_pk["len"][k])
        assert ga[o:o + L].tobytes() == arena[o:o + L].tobytes()


from recv_traffic import long_runs  # noqa: E402


@pytest.mark.parametrize("n_conns,n_per_conn,interleave", [(1, 16384, False), (4, 16384, True), (4, 16384, False),
                                                           (64, 2048, True), (2, 3000, True)])
def test_recv_long_runs_vs_oracle(orc, n_conns, n_per_conn, interleave):
    # runs longer than the walk's segment (r05: kSeg packets per wave, chained starts verified,
    # fallback to the sequential walk): PN gaps (some beyond a 1-byte window), in-window
    # reordering, a key update whose first packet overtakes the last old-phase one (previous-key
    # open), tampered packets — every record, the connection table and every arena byte vs the oracle.
    # The old-phase packet that arrives after the rotation is the reference's next-generation
    # attempt after an update in the same batch: MQ_ERR_DEFERRED in both (recv.rs:476-509)
    keys, conns, arena, dgrams = long_runs(orc, n_conns, n_per_conn, seed=n_conns * 7 + n_per_conn,
                                           interleave=interleave)
    oc, oa = conns.copy(), arena.copy()
    o_pk, o_n = orc.batch_recv(keys, oc, oa, dgrams, len(dgrams), threads=8)
    assert (o_pk["status"] == 0).sum() > 0.98 * o_n and (oc["key_updates"] == 1).all()
    assert (o_pk["status"] == _lib.MQ_ERR_CRYPTO).sum() > 0 and (o_pk["status"] == _lib.MQ_ERR_DEFERRED).sum() > 0
    g_pk, g_n, gc, ga = gpu_recv(keys, conns, arena, dgrams, len(dgrams))
    assert g_n == o_n
    for f in recv.PKT_DTYPE.names:
        assert (g_pk[f] == o_pk[f]).all(), (f, np.nonzero(g_pk[f] != o_pk[f])[0][:10])
    assert gc.tobytes() == oc.tobytes()
    assert ga.tobytes() == oa.tobytes()


def full_size_traffic(orc, n, n_conns, L=1200):
    """The bench's receive shape (tools/bench_aux.py): n one-packet datagrams of L bytes over
    n_conns connections (round robin), ChaCha20 1-RTT keys per connection, PNs 0x10000000 + i //
    n_conns, built by the oracle's send composite."""
    from milli_quic_amd import _lib, send, workload
    fl = L - 29
    w = workload.uniform(64, _lib.MQ_SUITE_CHACHA20, n_keys=n_conns)
    sc = send.make_conns([workload.DCID8] * n_conns, [b""] * n_conns, [[k, k, k] for k in range(n_conns)])
    req = np.zeros(n, dtype=send.REQ_DTYPE)
    i = np.arange(n, dtype=np.uint64)
    req["frames_offset"], req["out_offset"] = i * np.uint64(fl), i * np.uint64(L)
    req["pn"] = np.uint64(0x10000000) + i // np.uint64(n_conns)
    req["largest_acked"] = req["pn"] - np.uint64(1 << 24)
    req["frame_len"], req["out_cap"], req["level"] = fl, L, send.APPLICATION
    req["conn"] = (i % np.uint64(n_conns)).astype(np.uint32)
    frames = workload.splitmix_bytes(n * fl, seed=3)
    arena = np.zeros(n * L, dtype=np.uint8)
    st, ln = orc.batch_protect(w.keys, sc, frames, arena, req, _lib.MQ_SUITE_CHACHA20)
    assert (st == 0).all() and (ln == L).all()
    rc = np.zeros(n_conns, dtype=recv.CONN_DTYPE)
    rc["app_row"][:, 1] = np.arange(n_conns)
    rc["dcid_len"], rc["flags"] = 8, recv.HAS_APP
    dg = np.zeros(n, dtype=recv.DGRAM_DTYPE)
    dg["offset"], dg["len"], dg["conn"] = i * np.uint64(L), L, req["conn"]
    return w.keys, rc, arena, dg


@pytest.mark.parametrize("n_conns", [4096, 4, 1])
def test_recv_full_size_vs_oracle(orc, n_conns):
    # the benchmarked receive shape at full size: 2^20 datagrams over 4096
    # connections, and the same packets over 4 and 1 connections (runs of 2^18 / 2^20 packets: the
    # segmented walk) — every record, the connection table and every arena byte vs the oracle on
    # 16 threads
    n = 1 << 20
    keys, conns, arena, dgrams = full_size_traffic(orc, n, n_conns)
    g_pk, g_n, gc, ga = gpu_recv(keys, conns, arena, dgrams, n)
    oc = conns.copy()
    o_pk, o_n = orc.batch_recv(keys, oc, arena, dgrams, n, threads=16)  # arena opened in place
    assert g_n == o_n == n and (o_pk["status"] == 0).all()
    for f in recv.PKT_DTYPE.names:
        assert (g_pk[f] == o_pk[f]).all(), (f, np.nonzero(g_pk[f] != o_pk[f])[0][:10])
    assert gc.tobytes() == oc.tobytes()
    assert np.array_equal(ga, arena)
