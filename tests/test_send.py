"""Send composite from frames — CPU side: the oracle's restatement of
build_and_encrypt_initial_packet / build_and_encrypt_packet (src/connection/transmit.rs:499-755)
pinned to RFC 9001 A.5 and to the header codecs (packet.py, pinned to RFC 9001 A.2 in
test_abi.py), and its packets open through the pinned receive composite. GPU parity:
test_gpu_send.py."""
import numpy as np
import pytest

from milli_quic_amd import _lib, packet, send
from milli_quic_amd.batch import make_descs
from milli_quic_amd.key_schedule import key_material, make_key_material
from milli_quic_amd.workload import A1_SERVER_SECRET, A5_SECRET

A5_PN = 654360564


def a5_key():
    return key_material(_lib.MQ_SUITE_CHACHA20, A5_SECRET)


def test_rfc9001_a5_from_frames(orc, ref_fixtures):
    # A.5: short header, empty DCID, key phase 0, 3-byte PN (largest_acked 2^15 behind), PING frame
    conns = send.make_conns([b""], [b""], [[0, 0, 0]])
    req = np.zeros(1, dtype=send.REQ_DTYPE)
    req["pn"], req["largest_acked"], req["frame_len"], req["out_cap"] = A5_PN, A5_PN - (1 << 15), 1, 64
    req["level"] = send.APPLICATION
    out = np.zeros(64, dtype=np.uint8)
    st, ln = orc.batch_protect([a5_key()], conns, np.array([1], dtype=np.uint8), out, req, _lib.MQ_SUITE_MIXED)
    assert st[0] == 0 and ln[0] == 21
    assert out[:21].tobytes().hex() == ref_fixtures["rfc9001"]["a5_packet"]


def random_batch(n, seed, n_conns=16):
    """Requests over all levels, CID lengths 0..20, frame lengths 0..1400, PN distances that give
    every PN length, pad_to_min on most Initials; frames random; output slots sized generously,
    with a few too small. Key rows: 0 ChaCha 1-RTT, 1 AES 1-RTT, 2 AES (Initial/Handshake)."""
    rng = np.random.default_rng(seed)
    keys = [key_material(_lib.MQ_SUITE_CHACHA20, A5_SECRET), key_material(_lib.MQ_SUITE_AES128GCM, A1_SERVER_SECRET),
            make_key_material(_lib.MQ_SUITE_AES128GCM, bytes(range(16)), bytes(range(12)), bytes(range(16, 32)))]
    dl = rng.integers(0, 21, size=n_conns)
    sl = rng.integers(0, 21, size=n_conns)
    dl[:2], sl[:2] = [20, 0], [20, 0]
    conns = send.make_conns([rng.bytes(int(x)) for x in dl], [rng.bytes(int(x)) for x in sl],
                            [[2, 2, int(k)] for k in rng.integers(0, 2, size=n_conns)], 0)
    conns["key_phase"] = rng.integers(0, 2, size=n_conns)
    req = np.zeros(n, dtype=send.REQ_DTYPE)
    req["level"] = rng.choice(3, size=n, p=[0.25, 0.25, 0.5])
    req["flags"] = np.where(rng.random(n) < 0.8, send.PAD_TO_MIN, 0)
    fl = rng.integers(0, 1400, size=n)
    fl[:8] = [0, 1, 2, 3, 4, 30, 31, 1100]
    req["frame_len"] = fl
    req["conn"] = rng.integers(0, n_conns, size=n)
    pn_dist = np.array([1, 100, 200, 40000, 1 << 24])[rng.integers(0, 5, size=n)]
    la = rng.integers(0, 1 << 40, size=n).astype(np.uint64)
    req["largest_acked"] = la
    req["pn"] = la + pn_dist.astype(np.uint64)
    req["frames_offset"] = np.concatenate([[0], np.cumsum(fl[:-1])]).astype(np.uint64)
    frames = rng.integers(0, 256, size=int(fl.sum()) + 8, dtype=np.uint8)
    cap = np.array([send.max_packet_len(int(f), int(lv), True) for f, lv in zip(fl, req["level"])])
    if n > 14:
        cap[10:14] = [5, 20, 40, 100]  # too small: header / PN / payload BufferTooSmall
    req["out_cap"] = cap
    req["out_offset"] = np.concatenate([[0], np.cumsum(cap[:-1] + rng.integers(0, 5, size=n - 1))]).astype(np.uint64)
    out = np.full(int(req["out_offset"][-1]) + int(cap[-1]) + 64, 0xA5, dtype=np.uint8)
    return keys, conns, frames, req, out


def expected_header(c, r, pn_len, pad):
    """The header bytes from the independent packet.py codec (long_header.rs / short_header.rs)."""
    dcid, scid = bytes(c["dcid"][:c["dcid_len"]]), bytes(c["scid"][:c["scid_len"]])
    body = pn_len + int(r["frame_len"]) + pad + 16
    if r["level"] == send.INITIAL:
        return packet.initial_header(dcid, scid, b"", pn_len, body)[0]
    if r["level"] == send.HANDSHAKE:
        return packet.handshake_header(dcid, scid, pn_len, body)[0]
    return packet.short_header(dcid, pn_len, int(c["key_phase"]))[0]


def test_oracle_send_roundtrip(orc):
    keys, conns, frames, req, out = random_batch(400, seed=1)
    st, ln = orc.batch_protect(keys, conns, frames, out, req, _lib.MQ_SUITE_MIXED)
    assert (st[10:14] == _lib.MQ_ERR_BUFFER_TOO_SMALL).all() and (np.delete(st, range(10, 14)) == 0).all()
    for i in range(len(req)):
        r, c = req[i], conns[req[i]["conn"]]
        o = int(r["out_offset"])
        if st[i] != 0:
            assert (out[o:o + int(r["out_cap"])] == 0xA5).all()  # failed packets write nothing
            continue
        pn_len = packet.pn_length(int(r["pn"]), int(r["largest_acked"]))
        L = int(ln[i])
        fl = int(r["frame_len"])
        if r["level"] == send.INITIAL:  # transmit.rs:537-543: padding sized with the unpadded header
            total0 = len(expected_header(c, r, pn_len, 0)) + pn_len + fl + 16
            pad = 1200 - total0 if (r["flags"] & send.PAD_TO_MIN and total0 < 1200) else 0
        else:                           # :644-649
            pad = max(0, (20 - pn_len) - fl - 16)
        if r["level"] == send.INITIAL and r["flags"] & send.PAD_TO_MIN:
            assert L >= 1200
        hdr = expected_header(c, r, pn_len, pad)
        assert L == len(hdr) + pn_len + int(r["frame_len"]) + pad + 16
        # open with the (pinned) receive composite: header + PN + frames + PADDING come back
        pkt = out[o:o + L].copy()
        flags = _lib.MQ_PKT_LONG_HEADER if r["level"] != send.APPLICATION else 0
        d = make_descs([0], [L], [int(c["key_row"][r["level"]])], [int(r["largest_acked"])], [len(hdr)], [0], [flags])
        s2, pn = orc.batch_open(keys, pkt, d, _lib.MQ_SUITE_MIXED)
        assert s2[0] == 0 and int(pn[0]) == int(r["pn"])
        f0 = int(r["frames_offset"])
        want = hdr + int(r["pn"]).to_bytes(8, "big")[8 - pn_len:] + frames[f0:f0 + int(r["frame_len"])].tobytes() + bytes(pad)
        assert pkt[:L - 16].tobytes() == want, i


def test_oracle_send_edges(orc):
    keys, conns, _, req, out = random_batch(8, seed=2)
    frames = np.arange(2048, dtype=np.uint32).astype(np.uint8)
    r = req[:1].copy()
    r["level"], r["flags"], r["conn"], r["frames_offset"] = send.INITIAL, send.PAD_TO_MIN, 1, 0  # 0-length CIDs
    r["pn"], r["largest_acked"] = 5, 4                                   # 1-byte PN
    for fl, total in ((0, 1201), (30, 1201), (1100, 1200), (1300, 10 + 1 + 1300 + 16)):
        # a padded Initial whose Length varint grows from 1 to 2 bytes comes out 1201 bytes long,
        # exactly as transmit.rs:537-558 (padding sized with the first header) builds it
        r["frame_len"], r["out_cap"] = fl, 1400
        st, ln = orc.batch_protect(keys, conns, frames, out, r, _lib.MQ_SUITE_MIXED)
        assert st[0] == 0 and ln[0] == total, (fl, ln[0])
    r["out_cap"] = 1000                                                  # needed = whole packet
    st, ln = orc.batch_protect(keys, conns, frames, out, r, _lib.MQ_SUITE_MIXED)
    assert st[0] == _lib.MQ_ERR_BUFFER_TOO_SMALL and ln[0] == 1327
    r["out_cap"], r["frame_len"] = 3, 10                                 # needed = header length
    st, ln = orc.batch_protect(keys, conns, frames, out, r, _lib.MQ_SUITE_MIXED)
    assert st[0] == _lib.MQ_ERR_BUFFER_TOO_SMALL and ln[0] == 1 + 4 + 1 + 1 + 1 + 2
    r["conn"] = 99                                                       # bad connection row
    assert orc.batch_protect(keys, conns, frames, out, r, _lib.MQ_SUITE_MIXED)[0][0] == _lib.MQ_ERR_INVALID_ARG
    r["conn"], r["level"] = 1, send.INITIAL
    c2 = conns.copy()
    c2["key_row"][1, 0] = 0                                              # ChaCha row for Initial
    assert orc.batch_protect(keys, c2, frames, out, r, _lib.MQ_SUITE_MIXED)[0][0] == _lib.MQ_ERR_SUITE
