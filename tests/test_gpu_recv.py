"""Receive composite over raw datagrams on the GPU: mq_batch_recv against the
oracle's restatement of Connection::recv (recv.rs:189-510, 953-1025) — every packet record,
the updated connection table and every arena byte equal."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from milli_quic_amd import recv  # noqa: E402
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
