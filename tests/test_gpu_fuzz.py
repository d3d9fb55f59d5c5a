"""Randomised differential tests of the batch API against the oracle (GPU vs CPU restatement).

Each seeded batch mixes everything a descriptor can say at once: short and long QUIC headers
(pn_offset 1..320: AAD up to 21 GHASH blocks), plain AEAD rows (MQ_PKT_NO_HP), TLS records,
packets of 21 B to 5.2 kB (past 4080 B the AES counters exceed 255: no CTR cache; past 2048 B the
receive composite's limit, recv.rs:356-360, with and without MQ_PKT_NO_RECV_LIMIT), arbitrary byte alignments and gaps, both suites on several key rows plus
out-of-range and empty (suite 0) key ids, PNs near 2^62 (ProtocolViolation on open), lengths too
short for the sample or the tag, and tampered ciphertexts. The bar is the oracle's: identical
status for every packet, identical bytes in the whole arena (failed packets untouched, gap bytes
untouched), identical decoded PNs — under the mixed hint (device partition) and under each
single-suite hint (the other suite's rows: MQ_ERR_SUITE).
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from milli_quic_amd import _lib, batch, workload  # noqa: E402
from milli_quic_amd.batch import KeyTable, make_descs  # noqa: E402
from milli_quic_amd.key_schedule import make_key_material  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _device(mqlib):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    assert mqlib.mq_device_init(0) == 0


def _keys(rng):
    rows = []
    for suite in (_lib.MQ_SUITE_CHACHA20, _lib.MQ_SUITE_AES128GCM, _lib.MQ_SUITE_CHACHA20,
                  _lib.MQ_SUITE_AES128GCM, _lib.MQ_SUITE_AES128GCM):
        klen = 32 if suite == _lib.MQ_SUITE_CHACHA20 else 16
        rows.append(make_key_material(suite, rng.bytes(klen), rng.bytes(12), rng.bytes(klen)))
    rows.append(_lib.KeyMaterial())  # suite 0: every packet on it fails per packet
    return rows


def random_batch(seed, n):
    """(keys, arena, seal descriptors, open descriptors) of one fuzz batch."""
    rng = np.random.default_rng(seed)
    keys = _keys(rng)
    kind = rng.choice(4, size=n, p=[0.45, 0.3, 0.1, 0.15])  # short, long, plain AEAD, TLS record
    lens = np.zeros(n, dtype=np.int64)
    pn_off = np.zeros(n, dtype=np.int64)
    pn_len = rng.integers(1, 5, size=n)
    flags = np.zeros(n, dtype=np.uint8)
    reserved = np.zeros(n, dtype=np.uint32)
    for i in range(n):
        if kind[i] == 0:
            pn_off[i] = 1 + int(rng.integers(0, 21))
        elif kind[i] == 1:
            # long headers; some as long as an Initial with a token (AAD over 144 B)
            pn_off[i] = int(rng.integers(7, 61)) if rng.random() < 0.9 else int(rng.integers(61, 320))
            flags[i] = _lib.MQ_PKT_LONG_HEADER
        elif kind[i] == 2:
            pn_off[i] = int(rng.integers(0, 40))
            pn_len[i] = int(rng.integers(0, 5))
            flags[i] = _lib.MQ_PKT_NO_HP
        else:
            pn_off[i], pn_len[i] = 5, 0
            flags[i] = _lib.MQ_PKT_TLS_RECORD
            reserved[i] = int(rng.choice([20, 21, 22, 23]))
        lo = int(pn_off[i] + pn_len[i] + 16)
        r = rng.random()
        if r < 0.04:
            lens[i] = int(rng.integers(max(1, lo - 8), lo + 4))        # around the minimum
        elif r < 0.12:
            lens[i] = int(rng.integers(2040, 2600))                   # around the receive limit
        elif r < 0.14:
            lens[i] = int(rng.integers(4060, 5200))                   # counters past 255 (no CTR cache)
        else:
            lens[i] = int(rng.integers(lo, 1400))
        if kind[i] != 3 and rng.random() < 0.2:
            flags[i] |= _lib.MQ_PKT_NO_RECV_LIMIT
    lens = np.maximum(lens, 1)
    lens = np.maximum(lens, np.where((kind == 1) & (pn_off > 60), pn_off + pn_len + 40, 0))
    gaps = rng.integers(0, 40, size=n)
    offs = np.zeros(n, dtype=np.int64)
    offs[1:] = np.cumsum(lens[:-1] + gaps[:-1])
    offs += int(rng.integers(0, 16))
    arena = workload.splitmix_bytes(int(offs[-1] + lens[-1]) + 64, seed=seed)
    pns = rng.integers(0, 1 << 40, size=n).astype(np.uint64)
    near = rng.random(n) < 0.03
    pns[near] = np.uint64((1 << 62) - 1) - rng.integers(0, 3, size=int(near.sum())).astype(np.uint64)
    for i in range(n):  # first byte and PN bytes of the QUIC headers, as the sender writes them
        o = int(offs[i])
        if kind[i] in (0, 1) and lens[i] > pn_off[i] + pn_len[i]:
            arena[o] = (0xC0 if kind[i] == 1 else 0x40) | (int(pn_len[i]) - 1)
            for j in range(int(pn_len[i])):
                arena[o + int(pn_off[i]) + j] = (int(pns[i]) >> (8 * (int(pn_len[i]) - 1 - j))) & 0xFF
    key_id = rng.integers(0, 5, size=n).astype(np.uint32)
    bad = rng.random(n)
    key_id[bad < 0.03] = 5                     # empty row
    key_id[(bad >= 0.03) & (bad < 0.05)] = 77  # out of range
    seal = make_descs(offs.astype(np.uint64), lens.astype(np.uint32), key_id, pns, pn_off.astype(np.uint16),
                      pn_len.astype(np.uint8), flags)
    seal["reserved"] = reserved
    opn = seal.copy()
    quic = (kind == 0) | (kind == 1)
    opn["pn"][quic] = pns[quic] - np.uint64(1)       # open: largest PN of the space
    opn["pn_len"][quic] = 0
    opn["reserved"] = 0
    top = quic & (rng.random(n) < 0.03)              # largest PN at 2^62 - 1: decode_pn can overflow
    opn["pn"][top] = np.uint64((1 << 62) - 1)
    # TLS records open with len = 5 + the header's length field (= the sealed length)
    return keys, arena, seal, opn


def gpu(keys, arena, desc, hint, open_):
    kt = KeyTable(keys)
    n = len(desc)
    a = torch.from_numpy(arena.copy()).to(DEV)
    d = torch.from_numpy(desc.view(np.uint8).copy()).to(DEV)
    st = torch.full((n,), 0xEE, dtype=torch.uint8, device=DEV)
    pn = torch.zeros(n, dtype=torch.int64, device=DEV)
    ws = torch.full((max(batch.workspace_bytes(n), 256),), 0x5A, dtype=torch.uint8, device=DEV)
    if open_:
        batch.open_(kt, a, d, st, pn, hint, ws)
    else:
        batch.seal(kt, a, d, st, hint, ws)
    torch.cuda.synchronize()
    return a.cpu().numpy(), st.cpu().numpy(), pn.cpu().numpy().view(np.uint64)


def oracle(orc, keys, arena, desc, hint, open_):
    a = arena.copy()
    if open_:
        st, pn = orc.batch_open(keys, a, desc, hint, threads=8)
        return a, st, pn
    return a, orc.batch_seal(keys, a, desc, hint, threads=8), None


@pytest.mark.parametrize("seed", [101, 202, 303, 404])
def test_fuzz_batches_vs_oracle(orc, seed):
    keys, arena, seal, opn = random_batch(seed, 3000)
    for hint in (_lib.MQ_SUITE_MIXED, _lib.MQ_SUITE_AES128GCM, _lib.MQ_SUITE_CHACHA20):
        g_out, g_st, _ = gpu(keys, arena, seal, hint, False)
        o_out, o_st, _ = oracle(orc, keys, arena, seal, hint, False)
        assert (g_st == o_st).all(), (hint, np.nonzero(g_st != o_st)[0][:10])
        assert g_out.tobytes() == o_out.tobytes(), hint
        if hint == _lib.MQ_SUITE_MIXED:
            assert (o_st == 0).sum() > 2000 and len(set(o_st.tolist())) >= 4  # a real mix of outcomes
        # tamper a few sealed packets, then open
        rng = np.random.default_rng(seed + hint)
        bad = o_out.copy()
        for v in rng.choice(len(seal), size=60, replace=False):
            o, ln = int(seal["offset"][v]), int(seal["len"][v])
            bad[o + int(rng.integers(0, ln))] ^= 1 << int(rng.integers(0, 8))
        g_back, g_st, g_pn = gpu(keys, bad, opn, hint, True)
        o_back, o_st, o_pn = oracle(orc, keys, bad, opn, hint, True)
        assert (g_st == o_st).all(), (hint, np.nonzero(g_st != o_st)[0][:10])
        assert g_back.tobytes() == o_back.tobytes(), hint
        ok = o_st == 0
        quic = (opn["flags"] & _lib.MQ_PKT_NO_HP) == 0
        assert (g_pn[ok & quic] == o_pn[ok & quic]).all(), hint


@pytest.mark.parametrize("first_row", ["chacha", "empty"])
def test_fuzz_single_non_aes_row(orc, first_row):
    # r04: a key table whose only non-AES row is row 0 runs the mixed batch's second list on the
    # single-key ChaCha kernels (key material of that row in SGPRs). Every other row is AES; the
    # batch's out-of-range key ids land in the same list and must still fail alone, and an empty
    # (suite 0) row 0 must fail its packets with MQ_ERR_SUITE
    keys, arena, seal, opn = random_batch(505 if first_row == "chacha" else 606, 3000)
    rng = np.random.default_rng(7)
    for r in range(1, len(keys)):
        keys[r] = make_key_material(_lib.MQ_SUITE_AES128GCM, rng.bytes(16), rng.bytes(12), rng.bytes(16))
    if first_row == "empty":
        keys[0] = _lib.KeyMaterial()
    g_out, g_st, _ = gpu(keys, arena, seal, _lib.MQ_SUITE_MIXED, False)
    o_out, o_st, _ = oracle(orc, keys, arena, seal, _lib.MQ_SUITE_MIXED, False)
    assert (g_st == o_st).all(), np.nonzero(g_st != o_st)[0][:10]
    assert g_out.tobytes() == o_out.tobytes()
    on0 = seal["key_id"] == 0
    assert on0.sum() > 300 and (o_st[on0] == 0).any() == (first_row == "chacha")
    g_back, g_st, g_pn = gpu(keys, o_out, opn, _lib.MQ_SUITE_MIXED, True)
    o_back, o_st, o_pn = oracle(orc, keys, o_out, opn, _lib.MQ_SUITE_MIXED, True)
    assert (g_st == o_st).all(), np.nonzero(g_st != o_st)[0][:10]
    assert g_back.tobytes() == o_back.tobytes()
    ok = (o_st == 0) & ((opn["flags"] & _lib.MQ_PKT_NO_HP) == 0)
    assert (g_pn[ok] == o_pn[ok]).all()
