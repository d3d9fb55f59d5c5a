"""Narrow ChaCha20-Poly1305 tiles (r05: G lanes per packet, 64 / G packets per wave) against the
oracle, byte for byte: flat batches of short packets (the narrow kernel, mq_chacha.hip
chacha_narrow_flat) over random lengths, both header forms, 1..4-byte packet numbers, several key
rows, packed back to back at every alignment; the same batches forced through the octet kernel
(MQ_CC_NARROW 0) must give the same bytes, and long packets forced through the narrow kernel
(MQ_CC_NARROW 1: G = 8 rounds, direct rounds over the LDS budget) as well. Tampered packets, bad
key ids and a packet ending exactly at an arena end that is not 16-B aligned are included.
Reference composites: transmit.rs:625-755 (seal + header protection), recv.rs:340-421 /
953-1025 (header protection removal, decode_pn, open); rustcrypto.rs:111-165, 197-220."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from milli_quic_amd import _lib, batch, workload  # noqa: E402
from milli_quic_amd.batch import KeyTable, make_descs  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
CHACHA = _lib.MQ_SUITE_CHACHA20


@pytest.fixture(scope="module", autouse=True)
def _device(mqlib):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    assert mqlib.mq_device_init(0) == 0


def _Env(v):
    """MQ_CC_NARROW for the calls inside the block (mq_debug_option; None: the product choice)."""
    return _lib.option("MQ_CC_NARROW", v)


def to_dev(a):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).copy()).to(DEV)


def gpu_run(keys, arena, desc, open_=False, use_ws=True, hint=CHACHA):
    kt = KeyTable(keys)
    n = len(desc)
    a, d = to_dev(arena), to_dev(desc)
    st = torch.full((max(n, 1),), 0xEE, dtype=torch.uint8, device=DEV)
    pn = torch.zeros(max(n, 1), dtype=torch.int64, device=DEV)
    ws = torch.full((max(batch.workspace_bytes(n), 256),), 0xA5, dtype=torch.uint8, device=DEV) if use_ws else None
    if open_:
        batch.open_(kt, a, d, st, pn, hint, ws)
    else:
        batch.seal(kt, a, d, st, hint, ws)
    torch.cuda.synchronize()
    return a.cpu().numpy(), st.cpu().numpy()[:n], pn.cpu().numpy().view(np.uint64)[:n]


def oracle_run(orc, keys, arena, desc, open_=False, hint=CHACHA):
    a = arena.copy()
    if open_:
        st, pn = orc.batch_open(keys, a, desc, hint, threads=8)
        return a, st, pn
    return a, orc.batch_seal(keys, a, desc, hint, threads=8), None


def short_batch(n, lmin, lmax, n_keys=1, seed=1, long_frac=0.2, lead=0, suite=CHACHA):
    """n packets (ChaCha20, or `suite`) of random lengths in [lmin, lmax] packed back to back after `lead` bytes:
    short headers (DCID 8) or long ones (26-B Initial layout), pn_len 1..4, key row i mod n_keys.
    The arena ends exactly at the last packet (its length is usually not a multiple of 16)."""
    rng = np.random.default_rng(seed)
    keys = workload.uniform_keys(suite, n_keys)
    pn_len = rng.integers(1, 5, size=n).astype(np.uint8)
    long_h = rng.random(n) < long_frac
    pn_off = np.where(long_h, workload.LONG_HDR, workload.SHORT_HDR).astype(np.int64)
    L = rng.integers(lmin, lmax + 1, size=n).astype(np.int64)
    L = np.maximum(L, pn_off + 20)  # the header-protection sample fits
    offs = lead + np.concatenate([[0], np.cumsum(L[:-1])]).astype(np.int64)
    arena = workload.splitmix_bytes(int(offs[-1] + L[-1]), seed=seed)
    pns = (np.uint64(1 << 20) + rng.integers(0, 1 << 30, size=n).astype(np.uint64))
    for i in range(n):
        o, pl = int(offs[i]), int(pn_len[i])
        arena[o] = (0xC0 if long_h[i] else 0x40) | (pl - 1)
        po = int(pn_off[i])
        for b in range(pl):
            arena[o + po + b] = (int(pns[i]) >> (8 * (pl - 1 - b))) & 0xFF
    kid = (np.arange(n) % n_keys).astype(np.uint32)
    flags = np.where(long_h, _lib.MQ_PKT_LONG_HEADER, 0).astype(np.uint8)
    sd = make_descs(offs.astype(np.uint64), L.astype(np.uint32), kid, pns, pn_off.astype(np.uint16), pn_len, flags)
    od = make_descs(offs.astype(np.uint64), L.astype(np.uint32), kid, pns - np.uint64(1), pn_off.astype(np.uint16), 0,
                    flags)
    return keys, arena, sd, od, pns


def roundtrip_vs_oracle(orc, keys, arena, sd, od, pns, modes=(None, "0", "1"), hint=CHACHA, env=_Env):
    o_out, o_st, _ = oracle_run(orc, keys, arena, sd, hint=hint)
    o_back, o_st2, o_pn = oracle_run(orc, keys, o_out, od, open_=True, hint=hint)
    assert (o_st == 0).all() and (o_st2 == 0).all()
    for mode in modes:
        with env(mode):
            for use_ws in (True, False):
                g_out, g_st, _ = gpu_run(keys, arena, sd, use_ws=use_ws, hint=hint)
                assert (g_st == o_st).all(), (mode, use_ws, np.nonzero(g_st != o_st)[0][:8])
                assert g_out.tobytes() == o_out.tobytes(), (mode, use_ws)
                g_back, g_st, g_pn = gpu_run(keys, o_out, od, open_=True, use_ws=use_ws, hint=hint)
                assert (g_st == o_st2).all(), (mode, use_ws)
                assert g_back.tobytes() == o_back.tobytes(), (mode, use_ws)
                assert (g_pn == o_pn).all() and (g_pn == pns).all(), (mode, use_ws)


@pytest.mark.parametrize("lmin,lmax,n,n_keys", [
    (21, 90, 3001, 1),     # G = 1 (one round of 64 packets per wave), a ragged last wave
    (21, 140, 2000, 3),    # G = 1 / 2 by wave, three key rows
    (130, 290, 1500, 1),   # G = 2
    (290, 600, 1200, 2),   # G = 4
    (21, 640, 4000, 1),    # every G, waves of mixed sizes
])
def test_narrow_flat_vs_oracle(orc, lmin, lmax, n, n_keys):
    keys, arena, sd, od, pns = short_batch(n, lmin, lmax, n_keys, seed=lmin * 7 + lmax)
    roundtrip_vs_oracle(orc, keys, arena, sd, od, pns)


@pytest.mark.parametrize("lead", [0, 5, 13])
def test_narrow_uniform_alignments(orc, lead):
    # uniform 64-B / 256-B batches (the len_sweep shapes) shifted by `lead` bytes: every packet at
    # a fixed misalignment, the arena's last chunk partial
    for L in (64, 256):
        w = workload.uniform(777, CHACHA, L=L, pn_len=1 + L % 4)
        arena = np.concatenate([np.full(lead, 0x5A, np.uint8), w.arena])
        sd, od = w.seal_desc.copy(), w.open_desc.copy()
        sd["offset"] += lead
        od["offset"] += lead
        roundtrip_vs_oracle(orc, w.keys, arena, sd, od, w.pns, modes=(None, "0"))


def test_narrow_forced_on_long_packets(orc):
    # MQ_CC_NARROW=1 on packets up to 2048 B: waves choose G = 8 rounds (the octet layout without
    # the pool), rounds over the LDS budget run on HBM (direct)
    keys, arena, sd, od, pns = short_batch(700, 21, 2048, 2, seed=99)
    roundtrip_vs_oracle(orc, keys, arena, sd, od, pns, modes=("1",))


def test_narrow_failures_match_oracle(orc):
    keys, arena, sd, od, pns = short_batch(2500, 21, 400, 2, seed=5)
    sealed, st, _ = oracle_run(orc, keys, arena, sd)
    assert (st == 0).all()
    rng = np.random.default_rng(8)
    bad = sealed.copy()
    for v in rng.choice(len(sd), size=300, replace=False):  # one flipped bit anywhere in the packet
        o, L = int(sd["offset"][v]), int(sd["len"][v])
        bad[o + int(rng.integers(0, L))] ^= 1 << int(rng.integers(0, 8))
    od = od.copy()
    od["key_id"][3] = 77                   # key id out of range
    od["len"][4] = 24                      # sample out of range -> Crypto
    od["offset"][6] = len(bad) - 10        # past the arena end
    od["pn"][9] = (1 << 62) - 2            # decode_pn above 2^62 - 1 -> ProtocolViolation
    o_out, o_st, o_pn = oracle_run(orc, keys, bad, od, open_=True)
    assert (o_st != 0).sum() >= 250
    for mode in (None, "0"):
        with _Env(mode):
            for use_ws in (True, False):
                g_out, g_st, g_pn = gpu_run(keys, bad, od, open_=True, use_ws=use_ws)
                assert (g_st == o_st).all(), (mode, use_ws, np.nonzero(g_st != o_st)[0][:8])
                assert g_out.tobytes() == o_out.tobytes(), (mode, use_ws)
                ok = o_st == 0
                assert (g_pn[ok] == o_pn[ok]).all()
    sd = sd.copy()
    sd["pn_len"][3] = 0
    sd["len"][9] = 20
    sd["key_id"][10] = 1 << 20
    o_out, o_st, _ = oracle_run(orc, keys, arena, sd)
    g_out, g_st, _ = gpu_run(keys, arena, sd)
    assert (g_st == o_st).all() and g_out.tobytes() == o_out.tobytes()


@pytest.mark.parametrize("n", [1, 2, 63, 64, 65, 255, 257])
def test_narrow_counts(orc, n):
    # waves with one packet, exactly full waves, a partial last wave and a partial workgroup
    keys, arena, sd, od, pns = short_batch(n, 21, 200, 1, seed=n)
    roundtrip_vs_oracle(orc, keys, arena, sd, od, pns, modes=(None,))


@pytest.mark.parametrize("lmin,lmax,n", [(21, 150, 30000), (64, 700, 30000), (21, 2000, 20000), (64, 1350, 4097)])
@pytest.mark.parametrize("grid", [None, "1"])
def test_mixed_batches_narrow_regions(orc, lmin, lmax, n, grid):
    # mixed batches (MQ_SUITE_MIXED: the device partition) whose ChaCha20 list has narrow regions
    # (mq_partition.hip: classes of G = 4, 2, 1 after the octet classes; workgroups with and
    # without octet tiles, region boundaries inside a workgroup); grid "1" forces the persistent
    # list kernels, which walk the same list as octet tiles
    w = workload.config_e(n, seed=lmin * 31 + lmax, lmin=lmin, lmax=lmax)
    hint = _lib.MQ_SUITE_MIXED
    with _lib.option("MQ_CC_LIST", grid):
        g_out, g_st, _ = gpu_run(w.keys, w.arena, w.seal_desc, hint=hint)
        o_out, o_st, _ = oracle_run(orc, w.keys, w.arena, w.seal_desc, hint=hint)
        assert (o_st == 0).all() and (g_st == o_st).all()
        assert g_out.tobytes() == o_out.tobytes()
        g_back, g_st, g_pn = gpu_run(w.keys, g_out, w.open_desc, open_=True, hint=hint)
        o_back, o_st, o_pn = oracle_run(orc, w.keys, o_out, w.open_desc, open_=True, hint=hint)
        assert (g_st == 0).all() and (g_st == o_st).all() and (g_pn == o_pn).all()
        assert g_back.tobytes() == o_back.tobytes()


def _EnvLong(v):
    """MQ_CC_LONG for the calls inside the block (mq_debug_option)."""
    return _lib.option("MQ_CC_LONG", v)


@pytest.mark.parametrize("lmin,lmax,n", [(1150, 1600, 3000), (1600, 1950, 3001), (1500, 2600, 2000), (21, 2600, 2500)])
@pytest.mark.parametrize("mode", [None, "0", "1", "2"])
def test_long_images_vs_oracle(orc, lmin, lmax, n, mode):
    # flat ChaCha20 batches of long packets (r05): the 13-KiB (12 waves per CU) and 20-KiB (8 per CU)
    # image kernels, picked by the arena's bytes per packet or forced (MQ_CC_LONG); tiles over the
    # image budget take the direct path inside them. Open over 2048 B with MQ_PKT_NO_RECV_LIMIT.
    keys, arena, sd, od, pns = short_batch(n, lmin, lmax, 2, seed=lmax + n)
    od = od.copy()
    od["flags"] |= _lib.MQ_PKT_NO_RECV_LIMIT
    with _EnvLong(mode):
        roundtrip_vs_oracle(orc, keys, arena, sd, od, pns, modes=(None,))


@pytest.mark.parametrize("mode", [None, "1", "2"])
def test_long_images_single_key_vs_oracle(orc, mode):
    # the single-key (key material in SGPRs) long-image kernels, 1600-1950-B packets, a partial
    # last workgroup
    keys, arena, sd, od, pns = short_batch(4093, 1600, 1950, 1, seed=77)
    with _EnvLong(mode):
        roundtrip_vs_oracle(orc, keys, arena, sd, od, pns, modes=(None,))


@pytest.mark.parametrize("hinted", [False, True])
def test_subrange_batch_len_hint(orc, hinted):
    # a batch over part of a larger arena (descriptors of 4000 packets out of 24 000
    # 1200-B packets) — with MQ_BATCH_LEN_HINT it runs the 10-KiB octet kernel of a tight arena,
    # without it the 20-KiB one; same bytes either way, only the packets of the batch touched
    w = workload.config_b(24000)
    lo, hi = 9000, 13000
    assert batch.flat_kind(len(w.arena), hi - lo, CHACHA | (_lib.MQ_BATCH_LEN_HINT(1200) if hinted else 0)) == \
        (1 if hinted else 3)
    hint = CHACHA | (_lib.MQ_BATCH_LEN_HINT(1200) if hinted else 0)
    sd, od = w.seal_desc[lo:hi], w.open_desc[lo:hi]
    o_out, o_st, _ = oracle_run(orc, w.keys, w.arena, sd)
    assert (o_st == 0).all()
    g_out, g_st, _ = gpu_run(w.keys, w.arena, sd, hint=hint)
    assert (g_st == 0).all() and g_out.tobytes() == o_out.tobytes()
    assert g_out[:1200 * lo].tobytes() == w.arena[:1200 * lo].tobytes()
    g_back, g_st, g_pn = gpu_run(w.keys, g_out, od, open_=True, hint=hint)
    assert (g_st == 0).all() and (g_pn == w.pns[lo:hi]).all()
    v = g_back.reshape(-1, 1200)[lo:hi, :1184]
    assert v.tobytes() == w.arena.reshape(-1, 1200)[lo:hi, :1184].tobytes()


# ---- narrow AES-128-GCM tiles (r06, VERDICT r04 #1 "both suites"): single-key tiles of 16 packets on
# 4 lanes each or 32 on 2 (mq_aes.hip AesStream G = 4 / 2, the H^G Horner multiplier, the
# header-protection block in the free slot nblk once a packet has 4 CTR blocks); MQ_AES_NARROW
# 0 / 1 / 2 forces 8 / 4 / 2 lanes per packet. Reference: rustcrypto.rs:38-94 (seal /
# open), :175-186 (header protection), transmit.rs:625-755, recv.rs:340-421.
AES = _lib.MQ_SUITE_AES128GCM


def _EnvAes(v):
    """MQ_AES_NARROW for the calls inside the block (mq_debug_option)."""
    return _lib.option("MQ_AES_NARROW", v)


@pytest.mark.parametrize("lmin,lmax,n", [
    (21, 90, 3001),      # nblk < 4 (the late HP block) and >= 4 (HP in slot nblk), a ragged last tile
    (64, 64, 2048),      # uniform 64 B (the len_sweep shape)
    (90, 300, 1500),     # several iterations per tile, AAD of 1-2 blocks
    (21, 640, 4000),     # lean iterations beside short packets in one wave
])
def test_aes_narrow_flat_vs_oracle(orc, lmin, lmax, n):
    keys, arena, sd, od, pns = short_batch(n, lmin, lmax, 1, seed=lmin * 5 + lmax, suite=AES)
    roundtrip_vs_oracle(orc, keys, arena, sd, od, pns, modes=(None, "0", "1", "2"), hint=AES, env=_EnvAes)


@pytest.mark.parametrize("lead", [0, 5, 13])
def test_aes_narrow_uniform_alignments(orc, lead):
    for L in (64, 256, 448):
        w = workload.uniform(555, AES, L=L, pn_len=1 + L % 4)
        arena = np.concatenate([np.full(lead, 0x5A, np.uint8), w.arena])
        sd, od = w.seal_desc.copy(), w.open_desc.copy()
        sd["offset"] += lead
        od["offset"] += lead
        roundtrip_vs_oracle(orc, w.keys, arena, sd, od, w.pns, modes=(None, "0", "1", "2"), hint=AES, env=_EnvAes)


def test_aes_narrow_forced_on_long_packets(orc):
    # MQ_AES_NARROW=1 on packets up to 4500 B: counters past 255 (no CTR cache), long AAD, many
    # lean iterations; open over 2048 B with MQ_PKT_NO_RECV_LIMIT
    keys, arena, sd, od, pns = short_batch(900, 21, 4500, 1, seed=123, long_frac=0.5, suite=AES)
    od = od.copy()
    od["flags"] |= _lib.MQ_PKT_NO_RECV_LIMIT
    roundtrip_vs_oracle(orc, keys, arena, sd, od, pns, modes=("1", "2"), hint=AES, env=_EnvAes)


def test_aes_narrow_failures_match_oracle(orc):
    keys, arena, sd, od, pns = short_batch(2500, 21, 400, 1, seed=6, suite=AES)
    sealed, st, _ = oracle_run(orc, keys, arena, sd, hint=AES)
    assert (st == 0).all()
    rng = np.random.default_rng(9)
    bad = sealed.copy()
    for v in rng.choice(len(sd), size=300, replace=False):  # one flipped bit anywhere in the packet
        o, L = int(sd["offset"][v]), int(sd["len"][v])
        bad[o + int(rng.integers(0, L))] ^= 1 << int(rng.integers(0, 8))
    od = od.copy()
    od["key_id"][3] = 77                   # key id out of range
    od["len"][4] = 24                      # sample out of range -> Crypto
    od["offset"][6] = len(bad) - 10        # past the arena end
    od["pn"][9] = (1 << 62) - 2            # decode_pn above 2^62 - 1 -> ProtocolViolation
    o_out, o_st, o_pn = oracle_run(orc, keys, bad, od, open_=True, hint=AES)
    assert (o_st != 0).sum() >= 250
    for mode in (None, "0", "1", "2"):
        with _EnvAes(mode):
            for use_ws in (True, False):
                g_out, g_st, g_pn = gpu_run(keys, bad, od, open_=True, use_ws=use_ws, hint=AES)
                assert (g_st == o_st).all(), (mode, use_ws, np.nonzero(g_st != o_st)[0][:8])
                assert g_out.tobytes() == o_out.tobytes(), (mode, use_ws)
                ok = o_st == 0
                assert (g_pn[ok] == o_pn[ok]).all()
    sd = sd.copy()
    sd["pn_len"][3] = 0
    sd["len"][9] = 20
    sd["key_id"][10] = 1 << 20
    o_out, o_st, _ = oracle_run(orc, keys, arena, sd, hint=AES)
    for mode in (None, "1", "2"):
        with _EnvAes(mode):
            g_out, g_st, _ = gpu_run(keys, arena, sd, hint=AES)
            assert (g_st == o_st).all() and g_out.tobytes() == o_out.tobytes()


@pytest.mark.parametrize("n", [1, 2, 15, 16, 17, 191, 192, 193, 3073])
def test_aes_narrow_counts(orc, n):
    # tiles with one packet, exactly full tiles / workgroups (12 waves x 16 packets), partial ones
    keys, arena, sd, od, pns = short_batch(n, 21, 200, 1, seed=n + 1000, suite=AES)
    roundtrip_vs_oracle(orc, keys, arena, sd, od, pns, modes=(None, "1", "2"), hint=AES, env=_EnvAes)


@pytest.mark.parametrize("cfg,n,n_keys", [("c", 40000, 16), ("c", 20000, 3), ("e", 20000, 0)])
def test_aes_narrow_partitioned_vs_oracle(orc, cfg, n, n_keys):
    # partitioned AES (mixed hint): the hot key's segment on the narrow single-key kernel, the
    # key-segmented kernels with narrow tiles inside every segment (segments start at any multiple
    # of 8 entries), the multi-key octet kernel after the hot split; MQ_AES_NARROW 0 / 1 / 2 = 8 / 4
    # / 2 lanes per packet
    w = workload.config_c(n, n_keys=n_keys) if cfg == "c" else workload.config_e(n, seed=3)
    hint = _lib.MQ_SUITE_MIXED
    o_out, o_st, _ = oracle_run(orc, w.keys, w.arena, w.seal_desc, hint=hint)
    o_back, o_st2, o_pn = oracle_run(orc, w.keys, o_out, w.open_desc, open_=True, hint=hint)
    assert (o_st == 0).all() and (o_st2 == 0).all()
    for mode in (None, "0", "1", "2"):
        with _EnvAes(mode):
            g_out, g_st, _ = gpu_run(w.keys, w.arena, w.seal_desc, hint=hint)
            assert (g_st == o_st).all() and g_out.tobytes() == o_out.tobytes(), mode
            g_back, g_st, g_pn = gpu_run(w.keys, o_out, w.open_desc, open_=True, hint=hint)
            assert (g_st == o_st2).all() and (g_pn == o_pn).all(), mode
            assert g_back.tobytes() == o_back.tobytes(), mode


@pytest.mark.parametrize("hinted", [False, True])
def test_aes_subrange_batch_len_hint(orc, hinted):
    # a flat AES batch over part of a larger arena: with MQ_BATCH_LEN_HINT(1200) it runs 4 lanes per
    # packet (the narrow kernels of a tight arena), without it the arena's 7200 B per descriptor pick
    # the octet kernels; same bytes either way, only the batch's packets touched
    w = workload.config_c(24000)
    lo, hi = 9000, 13000
    hint = AES | (_lib.MQ_BATCH_LEN_HINT(1200) if hinted else 0)
    assert batch.aes_flat_kind(len(w.arena), hi - lo, hint) == (4 if hinted else 8)
    sd, od = w.seal_desc[lo:hi], w.open_desc[lo:hi]
    o_out, o_st, _ = oracle_run(orc, w.keys, w.arena, sd, hint=AES)
    assert (o_st == 0).all()
    g_out, g_st, _ = gpu_run(w.keys, w.arena, sd, hint=hint)
    assert (g_st == 0).all() and g_out.tobytes() == o_out.tobytes()
    assert g_out[:1200 * lo].tobytes() == w.arena[:1200 * lo].tobytes()
    g_back, g_st, g_pn = gpu_run(w.keys, g_out, od, open_=True, hint=hint)
    assert (g_st == 0).all() and (g_pn == w.pns[lo:hi]).all()
    v = g_back.reshape(-1, 1200)[lo:hi, :1184]
    assert v.tobytes() == w.arena.reshape(-1, 1200)[lo:hi, :1184].tobytes()
