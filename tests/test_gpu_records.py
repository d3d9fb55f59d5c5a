"""TLS 1.3 record layer on the GPU: the per-record trait calls and the batched
record seal/open, bit-exact against RFC 8448 §3 (tests/golden/tls_records.json) and the oracle."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from milli_quic_amd import _lib, batch, crypto, tls_record, workload  # noqa: E402
from milli_quic_amd.batch import KeyTable  # noqa: E402
from milli_quic_amd.key_schedule import make_key_material  # noqa: E402

from conftest import load_golden  # noqa: E402
from test_tls_records import km_of, pack  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _device(mqlib):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    assert mqlib.mq_device_init(0) == 0


@pytest.fixture(scope="module")
def records():
    return load_golden("tls_records.json")["records"]


def to_dev(a):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).copy()).to(DEV)


def gpu_records(keys, arena, desc, hint, open_):
    kt = KeyTable(keys)
    n = len(desc)
    a, d = to_dev(arena), to_dev(desc)
    st = torch.full((n,), 0xEE, dtype=torch.uint8, device=DEV)
    info = torch.zeros(n, dtype=torch.int64, device=DEV)
    ws = torch.empty(max(batch.workspace_bytes(n), 256), dtype=torch.uint8, device=DEV)
    if open_:
        batch.open_records(kt, a, d, st, info, hint, ws)
    else:
        batch.seal_records(kt, a, d, st, hint, ws)
    torch.cuda.synchronize()
    return a.cpu().numpy(), st.cpu().numpy(), info.cpu().numpy().view(np.uint64)


def test_per_record_api_rfc8448(records):
    for r in records:
        aead = crypto.Aes128GcmProvider().aead(bytes.fromhex(r["key"]))
        nonce = tls_record.build_nonce(bytes.fromhex(r["iv"]), r["seq"])
        p = bytes.fromhex(r["payload"])
        buf = bytearray(p) + bytearray(17)
        n = tls_record.seal_record(aead, nonce, buf, len(p), r["inner_type"])
        rec = bytes.fromhex(r["record"])
        assert n == len(p) + 17 and bytes(buf) == rec[5:], r["source"]
        assert tls_record.encode_record_header(23, n) == rec[:5]
        dl, ct = tls_record.open_record(aead, nonce, buf, n, rec[:5])
        assert (dl, ct) == (len(p), r["inner_type"]) and bytes(buf[:dl]) == p
    aead = crypto.ChaCha20Provider().aead(bytes(32))
    with pytest.raises(crypto.BufferTooSmall) as e:     # record.rs:97-99
        tls_record.seal_record(aead, bytes(12), bytearray(20), 4, 23)
    assert e.value.needed == 21
    buf = bytearray(3 + 17)                              # all-zero plaintext -> Error::Tls
    n = tls_record.seal_record(aead, bytes(12), buf, 3, 0)
    with pytest.raises(crypto.TlsError):
        tls_record.open_record(aead, bytes(12), buf, n, tls_record.encode_record_header(23, n))


@pytest.mark.parametrize("align", [1, 16])
def test_batch_rfc8448_records(records, align):
    keys = [km_of(r) for r in records]
    lens = [len(r["record"]) // 2 for r in records]
    arena, offs = pack(records, "payload", align)
    sd = tls_record.record_descs(offs, lens, range(len(records)), [r["seq"] for r in records],
                                 [r["inner_type"] for r in records])
    out, st, _ = gpu_records(keys, arena, sd, _lib.MQ_SUITE_AES128GCM, open_=False)
    assert (st == 0).all(), st
    want, _ = pack(records, "record", align)
    assert out.tobytes() == want.tobytes()  # records exact, gap bytes untouched
    od = tls_record.record_descs(offs, lens, range(len(records)), [r["seq"] for r in records])
    back, st, info = gpu_records(keys, out, od, _lib.MQ_SUITE_AES128GCM, open_=True)
    assert (st == 0).all()
    dl, ct = tls_record.unpack_info(info)
    for i, (o, r) in enumerate(zip(offs, records)):
        p = bytes.fromhex(r["payload"])
        assert dl[i] == len(p) and ct[i] == r["inner_type"]
        assert back[int(o) + 5:int(o) + 5 + len(p)].tobytes() == p


@pytest.mark.parametrize("suite", [1, 2])
def test_random_records_vs_oracle(orc, suite):
    # record sizes 0..16384 data bytes (the largest take the direct, non-LDS path), mixed with
    # malformed rows; statuses, bytes and (data_len, type) equal to the oracle
    rng = np.random.default_rng(100 + suite)
    n = 600
    data = rng.integers(0, 1400, size=n)
    data[:6] = [0, 1, 15, 16, 16384, 16383]
    lens = (data + 5 + 1 + 16).astype(np.int64)
    offs = np.zeros(n, dtype=np.int64)
    offs[1:] = np.cumsum(lens[:-1] + rng.integers(0, 9, size=n - 1))
    total = int(offs[-1] + lens[-1]) + 64
    arena = workload.splitmix_bytes(total, seed=suite)
    keys = [make_key_material(suite, bytes(rng.integers(0, 256, 32, dtype=np.uint8)),
                              bytes(rng.integers(0, 256, 12, dtype=np.uint8)), bytes(32)) for _ in range(4)]
    kid = (np.arange(n) % 4).astype(np.uint32)
    seq = rng.integers(0, 1 << 40, size=n).astype(np.uint64)
    types = rng.choice([20, 21, 22, 23], size=n).astype(np.uint32)
    types[7] = 0                                 # seals fine, fails the inner-type scan on open
    sd = tls_record.record_descs(offs.astype(np.uint64), lens, kid, seq, types)
    sd["pn_offset"][8] = 4                       # invalid descriptor
    sd["len"][9] = 21                            # no room for the type byte
    g_out, g_st, _ = gpu_records(keys, arena, sd, suite, open_=False)
    o_out = arena.copy()
    o_st = orc.batch_seal(keys, o_out, sd, suite, threads=8)
    assert (g_st == o_st).all() and o_st[10:].max() == 0
    assert g_out.tobytes() == o_out.tobytes()
    od = tls_record.record_descs(offs.astype(np.uint64), lens, kid, seq)
    bad = o_out.copy()
    for v in rng.choice(np.arange(20, n), size=40, replace=False):  # corrupt some records
        bad[int(offs[v]) + int(rng.integers(0, lens[v]))] ^= 0x40
    g_back, g_st, g_info = gpu_records(keys, bad, od, suite, open_=True)
    o_back = bad.copy()
    o_st, o_info = orc.batch_open(keys, o_back, od, suite, threads=8)
    assert (g_st == o_st).all() and o_st[7] == _lib.MQ_ERR_TLS
    assert g_back.tobytes() == o_back.tobytes()
    ok = o_st == 0
    assert (g_info[ok] == o_info[ok]).all()


# find_inner_content_type mirrors (reference tcp_tls/connection.rs:1019-1038): the inner
# plaintexts basic [41 42 43 17], padded [41 16 00 00] and all-zero [00 00 00 00]
INNER_CASES = [(bytes([0x41, 0x42, 0x43, 23]), (3, 23)), (bytes([0x41, 22, 0, 0]), (1, 22)), (bytes(4), None)]


@pytest.mark.parametrize("suite,klen", [(1, 16), (2, 32)])
def test_find_inner_content_type_mirrors(suite, klen):
    key, iv = bytes(range(klen)), bytes(range(100, 112))
    prov = crypto.Aes128GcmProvider() if suite == 1 else crypto.ChaCha20Provider()
    aead = prov.aead(key)
    recs = []
    for k, (inner, want) in enumerate(INNER_CASES):
        nonce = tls_record.build_nonce(iv, k)
        hdr = tls_record.encode_record_header(23, len(inner) + 16)
        buf = bytearray(inner) + bytearray(16)
        assert aead.seal_in_place(nonce, hdr, buf, len(inner)) == len(inner) + 16
        recs.append(hdr + bytes(buf))
        # per record (mq_record_open)
        b = bytearray(buf)
        if want is None:
            with pytest.raises(crypto.TlsError):          # find_inner_content_type_empty
                tls_record.open_record(aead, nonce, b, len(b), hdr)
            assert bytes(b[:4]) == inner                   # plaintext in place, as the reference
        else:
            assert tls_record.open_record(aead, nonce, b, len(b), hdr) == want
    # batch (mq_batch_open_records), one record each, unaligned
    offs = np.array([0, 27, 61], dtype=np.uint64)
    arena = np.zeros(128, dtype=np.uint8)
    for o, r in zip(offs, recs):
        arena[int(o):int(o) + len(r)] = np.frombuffer(r, dtype=np.uint8)
    km = make_key_material(suite, key, iv, bytes(32))
    od = tls_record.record_descs(offs, [len(r) for r in recs], [0, 0, 0], [0, 1, 2])
    back, st, info = gpu_records([km], arena, od, suite, open_=True)
    dl, ct = tls_record.unpack_info(info)
    assert list(st) == [0, 0, _lib.MQ_ERR_TLS]
    assert (int(dl[0]), int(ct[0])) == (3, 23) and (int(dl[1]), int(ct[1])) == (1, 22)
    for (inner, _), o in zip(INNER_CASES, offs):
        assert back[int(o) + 5:int(o) + 9].tobytes() == inner
