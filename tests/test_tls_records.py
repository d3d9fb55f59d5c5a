"""TLS 1.3 record layer — CPU side: the oracle pinned to RFC 8448 §3 records
(tests/golden/tls_records.json, extracted from the reference's rfc/rfc8448.txt by
gen_tls_records.py), mirrors of the reference's record-layer unit tests (src/tcp_tls/record.rs:145-186,
src/tcp_tls/connection.rs:1019-1038) and the descriptor rules. GPU parity is in test_gpu_records.py."""
import numpy as np
import pytest

from milli_quic_amd import _lib, tls_record
from milli_quic_amd.crypto import BufferTooSmall, TlsError
from milli_quic_amd.key_schedule import make_key_material

from conftest import load_golden


@pytest.fixture(scope="module")
def records():
    return load_golden("tls_records.json")["records"]


def km_of(r):
    return make_key_material(r["suite"], bytes.fromhex(r["key"]), bytes.fromhex(r["iv"]), bytes(16))


def pack(recs, field, align=1):
    """Records back to back at `align`; seal input = header room + payload + type + tag room."""
    offs, pos = [], 0
    for r in recs:
        pos = (pos + align - 1) // align * align
        offs.append(pos)
        pos += len(r["record"]) // 2
    arena = np.full(pos + 32, 0x5A, dtype=np.uint8)
    for o, r in zip(offs, recs):
        if field == "record":
            b = bytes.fromhex(r["record"])
        else:  # unsealed: 5 junk header bytes, payload, junk type byte, zero tag room
            b = b"\xEE" * 5 + bytes.fromhex(r["payload"]) + b"\xEE" + bytes(16)
        arena[o:o + len(b)] = np.frombuffer(b, dtype=np.uint8)
    return arena, np.array(offs, dtype=np.uint64)


def test_header_codec_and_nonce_mirrors():
    # record.rs:150-158 record_header_roundtrip
    assert tls_record.decode_record_header(tls_record.encode_record_header(tls_record.HANDSHAKE, 42)) == (22, 0x0303, 42)
    with pytest.raises(TlsError):                       # :176-179 decode_invalid_content_type
        tls_record.decode_record_header(bytes([0xFF, 3, 3, 0, 1]))
    with pytest.raises(BufferTooSmall):                 # :181-185 decode_too_short
        tls_record.decode_record_header(bytes([0x17, 3, 3, 0]))


def test_nonce_construction(mqlib):
    # record.rs:160-173 nonce_construction
    assert tls_record.build_nonce(bytes(12), 0) == bytes(12)
    n1 = tls_record.build_nonce(bytes(12), 1)
    assert n1[11] == 1 and n1[10] == 0
    assert tls_record.build_nonce(bytes([0xFF] * 12), 0) == bytes([0xFF] * 12)


def test_oracle_seals_rfc8448_records(orc, records):
    arena, offs = pack(records, "payload", align=1)
    lens = [len(r["record"]) // 2 for r in records]
    d = tls_record.record_descs(offs, lens, range(len(records)), [r["seq"] for r in records],
                                [r["inner_type"] for r in records])
    st = orc.batch_seal([km_of(r) for r in records], arena, d, _lib.MQ_SUITE_AES128GCM)
    assert (st == 0).all()
    for o, r in zip(offs, records):
        assert arena[int(o):int(o) + len(r["record"]) // 2].tobytes().hex() == r["record"], r["source"]


def test_oracle_opens_rfc8448_records(orc, records):
    arena, offs = pack(records, "record", align=16)
    lens = [len(r["record"]) // 2 for r in records]
    d = tls_record.record_descs(offs, lens, range(len(records)), [r["seq"] for r in records])
    st, info = orc.batch_open([km_of(r) for r in records], arena, d, _lib.MQ_SUITE_AES128GCM)
    assert (st == 0).all()
    dl, ct = tls_record.unpack_info(info)
    for i, (o, r) in enumerate(zip(offs, records)):
        p = bytes.fromhex(r["payload"])
        assert dl[i] == len(p) and ct[i] == r["inner_type"]
        assert arena[int(o) + 5:int(o) + 5 + len(p)].tobytes() == p


def test_oracle_record_errors(orc, records):
    r = records[3]
    rec = bytes.fromhex(r["record"])
    base = np.frombuffer(rec, dtype=np.uint8).copy()
    # tampered ciphertext -> Crypto, buffer untouched
    bad = base.copy()
    bad[9] ^= 1
    d = tls_record.record_descs([0], [len(rec)], [0], [r["seq"]])
    st, _ = orc.batch_open([km_of(r)], bad, d, _lib.MQ_SUITE_AES128GCM)
    assert st[0] == _lib.MQ_ERR_CRYPTO and bad[10:].tobytes() == rec[10:]
    # wrong sequence number -> Crypto
    st, _ = orc.batch_open([km_of(r)], base.copy(), tls_record.record_descs([0], [len(rec)], [0], [r["seq"] + 1]),
                           _lib.MQ_SUITE_AES128GCM)
    assert st[0] == _lib.MQ_ERR_CRYPTO
    # descriptor rules: pn_offset must be 5; seal needs room for the type byte and the tag
    d2 = d.copy()
    d2["pn_offset"] = 4
    assert orc.batch_open([km_of(r)], base.copy(), d2, _lib.MQ_SUITE_AES128GCM)[0][0] == _lib.MQ_ERR_INVALID_ARG
    small = tls_record.record_descs([0], [21], [0], [0], [0x17])
    assert orc.batch_seal([km_of(r)], base.copy(), small, _lib.MQ_SUITE_AES128GCM)[0] == _lib.MQ_ERR_BUFFER_TOO_SMALL
    short = tls_record.record_descs([0], [20], [0], [0])
    assert orc.batch_open([km_of(r)], base.copy(), short, _lib.MQ_SUITE_AES128GCM)[0][0] == _lib.MQ_ERR_CRYPTO


@pytest.mark.parametrize("suite", [1, 2])
def test_oracle_inner_content_type_rules(orc, suite):
    # connection.rs:1019-1038: type after data, zero padding skipped, all-zero -> Error::Tls,
    # and a byte outside 20..23 -> Error::Tls (record.rs:16-24)
    key = bytes(range(32 if suite == 2 else 16))
    km = make_key_material(suite, key, bytes(range(12)), bytes(32))
    cases = [(b"ABC", 0x17, b""), (b"A", 0x16, b"\x00\x00"), (b"", 0x00, b"\x00\x00\x00"), (b"xy", 0x30, b"")]
    for data, ctype, pad in cases:
        # seal data || type || pad as the "plaintext" of a record whose inner type byte is pad's last
        # byte (or the type itself when there is no padding)
        body = data + bytes([ctype]) + pad
        total = 5 + len(body) + 16
        a = np.zeros(total, dtype=np.uint8)
        a[5:5 + len(body) - 1] = np.frombuffer(body[:-1], dtype=np.uint8)
        sd = tls_record.record_descs([0], [total], [0], [7], [body[-1]])
        assert orc.batch_seal([km], a, sd, suite)[0] == 0
        st, info = orc.batch_open([km], a, tls_record.record_descs([0], [total], [0], [7]), suite)
        if ctype in (0x16, 0x17):
            dl, ct = tls_record.unpack_info(info)
            assert st[0] == 0 and dl[0] == len(data) and ct[0] == ctype
        else:
            assert st[0] == _lib.MQ_ERR_TLS
            assert a[5:5 + len(body)].tobytes() == body  # plaintext is in place (as the reference)
