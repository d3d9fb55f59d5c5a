"""Send composite from frames on the GPU: mq_batch_protect bit-exact against
the oracle (statuses, packet lengths / `needed`, every output byte), RFC 9001 A.5 rebuilt from its
PING frame, and a full-size 2^20-packet 1-RTT batch whose packets open through the receive path."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from milli_quic_amd import _lib, batch, send, workload  # noqa: E402
from milli_quic_amd.batch import KeyTable  # noqa: E402

from test_send import A5_PN, a5_key, random_batch  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _device(mqlib):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    assert mqlib.mq_device_init(0) == 0


def t(a):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1).copy()).to(DEV)


def gpu_protect(keys, conns, frames, out, req, hint):
    kt = KeyTable(keys)
    n = len(req)
    o = t(out)
    st = torch.full((n,), 0xEE, dtype=torch.uint8, device=DEV)
    ln = torch.zeros(n, dtype=torch.int32, device=DEV)
    ws = torch.empty(send.workspace_bytes(n), dtype=torch.uint8, device=DEV)
    send.protect(kt, t(conns), t(frames), o, t(req), st, ln, hint, ws)
    torch.cuda.synchronize()
    return o.cpu().numpy(), st.cpu().numpy(), ln.cpu().numpy().view(np.uint32)


def test_a5_from_frames(ref_fixtures):
    conns = send.make_conns([b""], [b""], [[0, 0, 0]])
    req = np.zeros(1, dtype=send.REQ_DTYPE)
    req["pn"], req["largest_acked"], req["frame_len"], req["out_cap"] = A5_PN, A5_PN - (1 << 15), 1, 64
    req["level"] = send.APPLICATION
    out, st, ln = gpu_protect([a5_key()], conns, np.array([1], dtype=np.uint8), np.zeros(64, dtype=np.uint8), req,
                              _lib.MQ_SUITE_CHACHA20)
    assert st[0] == 0 and ln[0] == 21 and out[:21].tobytes().hex() == ref_fixtures["rfc9001"]["a5_packet"]


@pytest.mark.parametrize("seed", [1, 7])
def test_protect_vs_oracle(orc, seed):
    keys, conns, frames, req, out = random_batch(3000, seed)
    req["conn"][20] = 999                        # bad connection row
    req["frames_offset"][21] = frames.size       # frames out of range
    g_out, g_st, g_ln = gpu_protect(keys, conns, frames, out, req, _lib.MQ_SUITE_MIXED)
    o_out = out.copy()
    o_st, o_ln = orc.batch_protect(keys, conns, frames, o_out, req, _lib.MQ_SUITE_MIXED)
    assert (g_st == o_st).all(), np.nonzero(g_st != o_st)
    assert (g_ln == o_ln).all()
    assert g_out.tobytes() == o_out.tobytes()


def chacha_heavy_batch(n, seed):
    """random_batch with most requests 1-RTT on the ChaCha20 row (the fused protect kernel's
    case), the rest Initial / Handshake or 1-RTT on the AES row (suite errors under the hint)."""
    keys, conns, frames, req, out = random_batch(n, seed)
    conns["key_row"][2:, 2] = 0
    rng = np.random.default_rng(seed + 100)
    req["level"] = np.where(rng.random(n) < 0.85, send.APPLICATION, req["level"])
    return keys, conns, frames, req, out


@pytest.mark.parametrize("hint", [_lib.MQ_SUITE_CHACHA20, _lib.MQ_SUITE_AES128GCM])
@pytest.mark.parametrize("seed", [2, 9])
def test_protect_suite_hint_vs_oracle(orc, seed, hint):
    # a single-suite hint: rows of the other suite fail with MQ_ERR_SUITE before anything is
    # written (orc_batch_protect); ChaCha20 runs the fused build + seal kernel, unaligned output
    # slots and packets past the LDS image budget (direct path) included
    keys, conns, frames, req, out = chacha_heavy_batch(3000, seed)
    g_out, g_st, g_ln = gpu_protect(keys, conns, frames, out, req, hint)
    o_out = out.copy()
    o_st, o_ln = orc.batch_protect(keys, conns, frames, o_out, req, hint)
    assert (g_st == o_st).all(), np.nonzero(g_st != o_st)
    assert (g_ln == o_ln).all(), np.nonzero(g_ln != o_ln)
    assert g_out.tobytes() == o_out.tobytes()
    assert (o_st == 0).sum() > (1000 if hint == _lib.MQ_SUITE_CHACHA20 else 100)


def test_protect_fused_matches_two_kernel():
    # the fused ChaCha20 kernel and the build-then-seal composite (MQ_PROTECT_FUSED 0) agree byte
    # for byte, statuses and lengths included
    keys, conns, frames, req, out = chacha_heavy_batch(5000, 4)
    a = gpu_protect(keys, conns, frames, out, req, _lib.MQ_SUITE_CHACHA20)
    with _lib.option("MQ_PROTECT_FUSED", 0):
        b = gpu_protect(keys, conns, frames, out, req, _lib.MQ_SUITE_CHACHA20)
    for x, y in zip(a, b):
        assert x.tobytes() == y.tobytes()


def test_full_size_protect_then_open():
    # 2^20 1-RTT packets of 1171-byte frames (config B's payload), ChaCha20; the built packets
    # are exactly config B's wire format and open through mq_batch_open
    n, fl = 1 << 20, 1171
    w = workload.config_b(64)
    conns = send.make_conns([workload.DCID8], [b""], [[0, 0, 0]])
    req = np.zeros(n, dtype=send.REQ_DTYPE)
    req["frames_offset"] = np.arange(n, dtype=np.uint64) * np.uint64(fl)
    req["out_offset"] = np.arange(n, dtype=np.uint64) * np.uint64(1200)
    req["pn"] = 0x10000000 + np.arange(n, dtype=np.uint64)
    req["largest_acked"] = req["pn"] - np.uint64(1 << 24)   # 4-byte PN, as config B
    req["frame_len"], req["out_cap"], req["level"] = fl, 1200, send.APPLICATION
    frames = workload.splitmix_bytes(n * fl, seed=3)
    kt = KeyTable(w.keys)
    out = torch.zeros(n * 1200, dtype=torch.uint8, device=DEV)
    st = torch.full((n,), 0xEE, dtype=torch.uint8, device=DEV)
    ln = torch.zeros(n, dtype=torch.int32, device=DEV)
    ws = torch.empty(send.workspace_bytes(n), dtype=torch.uint8, device=DEV)
    send.protect(kt, t(conns), t(frames), out, t(req), st, ln, _lib.MQ_SUITE_CHACHA20, ws)
    torch.cuda.synchronize()
    assert int((st != 0).sum()) == 0 and int((ln != 1200).sum()) == 0
    od = w.open_desc[:1].repeat(n)
    od["offset"] = req["out_offset"]
    od["pn"] = req["pn"] - np.uint64(1)
    pn = torch.zeros(n, dtype=torch.int64, device=DEV)
    batch.open_(kt, out, t(od), st, pn, _lib.MQ_SUITE_CHACHA20)
    torch.cuda.synchronize()
    assert int((st != 0).sum()) == 0 and (pn.cpu().numpy().view(np.uint64) == req["pn"]).all()
    back = out.cpu().numpy().reshape(n, 1200)[:, 13:1184]
    assert back.tobytes() == frames.tobytes()
