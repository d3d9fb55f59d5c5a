"""Pin the CPU oracle before trusting it (no GPU needed).

The reference's own tests never pin AEAD/HP output bytes; what pins them:
  * RFC 9001 Appendix A (A.1 keys, A.2/A.3 AES-128-GCM Initial packets, A.5 ChaCha20 short
    header) as shipped in the reference tree (rfc/rfc9001.txt:2319-2553);
  * the reference's captured curl --http3 Initial (src/connection/mod.rs:2210), which its test
    server_processes_curl_initial_packet must open (:2233-2311);
  * RFC 8439 §2.8.2;
  * OpenSSL-generated vectors (tests/golden/gen_golden.c) over edge lengths.
"""
import numpy as np
import pytest

from milli_quic_amd import _lib
from milli_quic_amd.batch import make_descs

from helpers import curl_desc_and_keys

A1 = {
    "initial_secret": "7db5df06e7a69e432496adedb00851923595221596ae2ae9fb8115c1e9ed0a44",
}


def test_aead_vectors_seal_open(orc, aead_vectors):
    for c in aead_vectors:
        key, nonce, aad, pt = (bytes.fromhex(c[k]) for k in ("key", "nonce", "aad", "pt"))
        rc, ct, _ = orc.aead_seal(c["suite"], key, nonce, aad, pt)
        assert rc == 0
        assert ct.hex() == c["ct_tag"], (c["suite"], len(pt))
        rc, back = orc.aead_open(c["suite"], key, nonce, aad, ct)
        assert rc == 0 and back == pt


def test_rfc8439_tag_literal(orc, aead_vectors):
    c = [v for v in aead_vectors if v.get("name") == "rfc8439-2.8.2"][0]
    # RFC 8439 §2.8.2: Tag 1a:e1:0b:59:4f:09:e2:6a:7e:90:2e:cb:d0:60:06:91
    assert c["ct_tag"][-32:] == "1ae10b594f09e26a7e902ecbd0600691"
    rc, ct, _ = orc.aead_seal(2, bytes.fromhex(c["key"]), bytes.fromhex(c["nonce"]), bytes.fromhex(c["aad"]),
                              bytes.fromhex(c["pt"]))
    assert ct.hex()[-32:] == "1ae10b594f09e26a7e902ecbd0600691"


def test_aead_tamper_and_errors(orc):
    key, nonce = bytes([0x42] * 32), bytes(12)
    rc, ct, _ = orc.aead_seal(2, key, nonce, b"aad", b"secret")
    bad = bytearray(ct)
    bad[0] ^= 0xFF
    rc, after = orc.aead_open(2, key, nonce, b"aad", bytes(bad))
    assert rc == _lib.MQ_ERR_CRYPTO and after == bytes(bad)  # buffer left as received
    assert orc.aead_seal(2, key, bytes(11), b"", b"x")[0] == _lib.MQ_ERR_CRYPTO
    rc, _, needed = orc.aead_seal(2, key, nonce, b"", b"abcdef", buf_len=10)
    assert rc == _lib.MQ_ERR_BUFFER_TOO_SMALL and needed == 22
    assert orc.aead_open(1, bytes(16), nonce, b"", bytes(15))[0] == _lib.MQ_ERR_CRYPTO


def test_hp_vectors(orc, hp_vectors):
    for c in hp_vectors:
        rc, m = orc.hp_mask(c["suite"], bytes.fromhex(c["hp"]), bytes.fromhex(c["sample"]))
        assert rc == 0 and m.hex() == c["mask"]
    assert orc.hp_mask(1, bytes(16), bytes(15))[0] == _lib.MQ_ERR_INVALID_ARG


def test_rfc9001_a1_keys(orc, ref_fixtures):
    a1 = ref_fixtures["rfc9001"]["a1"]
    c, s = orc.derive_initial_secrets(bytes.fromhex(ref_fixtures["rfc9001"]["dcid"]))
    assert c.hex() == a1["client_initial_secret"] and s.hex() == a1["server_initial_secret"]
    for side, sec in (("client", c), ("server", s)):
        assert orc.hkdf_expand_label(sec, b"quic key", b"", 16)[1].hex() == a1[f"{side}_key"]
        assert orc.hkdf_expand_label(sec, b"quic iv", b"", 12)[1].hex() == a1[f"{side}_iv"]
        assert orc.hkdf_expand_label(sec, b"quic hp", b"", 16)[1].hex() == a1[f"{side}_hp"]
    a5 = ref_fixtures["rfc9001"]["a5"]
    assert orc.hkdf_expand_label(bytes.fromhex(a5["secret"]), b"quic ku", b"", 32)[1].hex().endswith(a5["ku"])
    # info > 80 bytes -> Error::Crypto (key_schedule.rs:37-39)
    assert orc.hkdf_expand_label(bytes(32), b"x" * 80, b"", 16)[0] == _lib.MQ_ERR_CRYPTO


def _km(p):
    km = _lib.KeyMaterial()
    km.suite = p["suite"]
    for name in ("key", "iv", "hp"):
        b = bytes.fromhex(p[name])
        getattr(km, name)[: len(b)] = list(b)
    return km


def _one(p, protected):
    data = bytes.fromhex(p["protected" if protected else "unprotected"])
    arena = np.frombuffer(data, dtype=np.uint8).copy()
    flags = _lib.MQ_PKT_LONG_HEADER if p["long_header"] else 0
    seal = make_descs([0], [p["len"]], [0], [p["pn"]], [p["pn_offset"]], [p["pn_len"]], [flags])
    opn = make_descs([0], [p["len"]], [0], [p["largest_pn"]], [p["pn_offset"]], [0], [flags])
    return arena, seal, opn


def test_packet_vectors_protect_unprotect(orc, packet_vectors):
    for p in packet_vectors:
        arena, seal, opn = _one(p, protected=False)
        st = orc.batch_seal([_km(p)], arena, seal, _lib.MQ_SUITE_MIXED)
        assert st[0] == 0 and arena.tobytes().hex() == p["protected"], p["name"]
        st, pn = orc.batch_open([_km(p)], arena, opn, _lib.MQ_SUITE_MIXED)
        assert st[0] == 0 and int(pn[0]) == p["pn"], p["name"]
        # after open: header unmasked, payload decrypted, tag bytes untouched
        assert arena.tobytes()[:-16].hex() == p["unprotected"][:-32], p["name"]


def test_rfc9001_packets_match_rfc_text(packet_vectors, ref_fixtures):
    by = {p["name"]: p for p in packet_vectors}
    assert by["rfc9001-A.2"]["protected"] == ref_fixtures["rfc9001"]["a2_protected"]
    assert by["rfc9001-A.3"]["protected"] == ref_fixtures["rfc9001"]["a3_protected"]
    assert by["rfc9001-A.5"]["protected"] == ref_fixtures["rfc9001"]["a5_packet"]


def test_curl_initial_opens(orc, ref_fixtures):
    data, dcid, pn_offset, length, client = curl_desc_and_keys(orc, ref_fixtures, orc.derive_initial_secrets)
    assert len(data) == 1200 and len(dcid) == 20 and pn_offset == 52
    km = _lib.KeyMaterial()
    km.suite = _lib.MQ_SUITE_AES128GCM
    km.key[:16] = list(orc.hkdf_expand_label(client, b"quic key", b"", 16)[1])
    km.iv[:12] = list(orc.hkdf_expand_label(client, b"quic iv", b"", 12)[1])
    km.hp[:16] = list(orc.hkdf_expand_label(client, b"quic hp", b"", 16)[1])
    arena = np.frombuffer(data, dtype=np.uint8).copy()
    opn = make_descs([0], [pn_offset + length], [0], [0], [pn_offset], [0], [_lib.MQ_PKT_LONG_HEADER])
    st, pn = orc.batch_open([km], arena, opn, _lib.MQ_SUITE_AES128GCM)
    assert st[0] == 0 and int(pn[0]) == 0
    pn_len = (arena[0] & 3) + 1
    assert pn_len == 1 and arena[pn_offset + pn_len] == 0x06  # first frame: CRYPTO


def test_decode_pn_rfc9000_a3(orc):
    # RFC 9000 A.3 example: largest 0xa82f30ea, truncated 0x9b32 (2 bytes) -> 0xa82f9b32
    assert orc.decode_pn(0x9B32, 2, 0xA82F30EA) == 0xA82F9B32
    rng = np.random.default_rng(7)
    from milli_quic_amd.packet import decode_pn
    for _ in range(2000):
        largest = int(rng.integers(0, 1 << 40))
        pn_len = int(rng.integers(1, 5))
        trunc = int(rng.integers(0, 1 << (8 * pn_len)))
        assert orc.decode_pn(trunc, pn_len, largest) == decode_pn(trunc, pn_len, largest)


@pytest.mark.parametrize("suite", [_lib.MQ_SUITE_AES128GCM, _lib.MQ_SUITE_CHACHA20])
def test_receive_limit_2048(orc, suite):
    # recv.rs:356-360 / :962-965: the receive composite copies the packet into a 2048-B stack
    # buffer and returns Err(BufferTooSmall { needed: len }) above that, before any crypto; the
    # packet stays as received. MQ_PKT_NO_RECV_LIMIT lifts it (documented divergence).
    from milli_quic_amd import workload
    for L, flags in ((2048, 0), (2049, 0), (3000, 0), (2049, _lib.MQ_PKT_NO_RECV_LIMIT)):
        w = workload.uniform(4, suite, L=L)
        st = orc.batch_seal(w.keys, w.arena, w.seal_desc, suite)
        assert (st == 0).all()  # the send side has no such limit (transmit.rs:625-755)
        sealed = w.arena.copy()
        od = w.open_desc.copy()
        od["flags"] |= flags
        st, pn = orc.batch_open(w.keys, w.arena, od, suite)
        if L > 2048 and not flags:
            assert (st == _lib.MQ_ERR_BUFFER_TOO_SMALL).all() and w.arena.tobytes() == sealed.tobytes()
        else:
            assert (st == 0).all() and (pn == w.pns).all()
    # records (MQ_PKT_TLS_RECORD) and plain AEAD rows (MQ_PKT_NO_HP) are not QUIC receive
    # composites: no limit
    w = workload.uniform(2, suite, L=3000)
    sd, od = w.seal_desc.copy(), w.open_desc.copy()
    for d in (sd, od):
        d["flags"] = _lib.MQ_PKT_NO_HP
        d["pn_len"] = 4
    od["pn"] = sd["pn"]  # plain AEAD: the descriptor's pn is the nonce's pn
    assert (orc.batch_seal(w.keys, w.arena, sd, suite) == 0).all()
    assert (orc.batch_open(w.keys, w.arena, od, suite)[0] == 0).all()
