"""Receive composite over raw datagrams — CPU side: the oracle's restatement
of Connection::recv (src/connection/recv.rs:189-510, 953-1025) without frame dispatch, checked on
traffic built by the (pinned) send composite: every untampered packet opens with its PN, the
skipped packet types are skipped, the per-connection state (largest PN, key phase, rotation)
advances as the reference's does. GPU parity: test_gpu_recv.py."""
import numpy as np

from milli_quic_amd import _lib, recv

from recv_traffic import assemble, build_traffic


import pytest


@pytest.mark.parametrize("tamper_flip", [False, True])
def test_oracle_recv_traffic(orc, tamper_flip):
    # tamper_flip: the first packet of the new key phase fails; the next one confirms the
    # update (recv.rs:476-509), so the rotation still happens exactly once
    keys, conns, scripts = build_traffic(orc, seed=3, n_conns=6, n_app=20, tamper_flip=tamper_flip)
    arena, dgrams = assemble(orc, keys, conns, scripts, seed=3)
    c2 = conns.copy()
    a2 = arena.copy()
    pk, n = orc.batch_recv(keys, c2, a2, dgrams, 4096)
    assert n == len(pk)
    ok = pk["status"] == 0
    # every scripted packet appears once; tampered ones fail with Error::Crypto
    n_script = sum(len(p) for _, _, dgs in scripts for p in dgs)
    tampered = sum(1 for _, _, dgs in scripts for p in dgs for part in p if part[5])
    assert ok.sum() == n_script - tampered
    assert (pk["status"][pk["dgram"] < len(dgrams) - 6] != _lib.MQ_ERR_CRYPTO).sum() >= n_script - tampered
    # state: one key update per connection, phase flipped, next generation consumed
    assert (c2["key_updates"] == 1).all() and (c2["key_phase"] == 1).all()
    assert ((c2["flags"] & recv.HAS_PREV) != 0).all() and ((c2["flags"] & recv.HAS_NEXT) == 0).all()
    for c, (_, rows, dgs) in enumerate(scripts):
        app = [part[3] for p in dgs for part in p if part[1] == 2 and not part[5]]
        assert c2["largest_pn"][c, 2] == max(app)
        mine = pk[(pk["level"] == 2) & ok & (np.isin(pk["dgram"], np.nonzero(dgrams["conn"] == c)[0]))]
        assert sorted(int(x) for x in mine["pn"]) == sorted(app)
    # extras: VN / Retry / 0-RTT skipped, truncated header stops the datagram, short < CID -> BTS,
    # a phase flip after the rotation with no next keys -> Crypto
    last = pk[pk["dgram"] >= len(dgrams) - 6]
    assert _lib.MQ_ERR_BUFFER_TOO_SMALL in last["status"]
    # payload offsets point at the plaintext: decrypted frames follow the unmasked header
    for r in pk[ok & (pk["level"] == 2)]:
        c = int(dgrams["conn"][r["dgram"]])
        assert int(r["payload_offset"]) == 1 + int(conns["dcid_len"][c]) + (int(a2[int(r["offset"])]) & 3) + 1
    # failed packets are left as received
    bad = pk[~ok]
    for r in bad:
        o, L = int(r["offset"]), int(r["len"])
        assert a2[o:o + L].tobytes() == arena[o:o + L].tobytes()


@pytest.mark.parametrize("threads", [2, 5, 16])
def test_oracle_recv_threads_identical(orc, threads):
    # orc_batch_recv_mt (connections split over threads; record indices from a parse-only pass)
    # gives the serial loop's records, connection table and arena exactly — what lets the full-size
    # GPU receive parity tests check 2^20 datagrams against the oracle on 16 threads
    keys, conns, scripts = build_traffic(orc, seed=7, n_conns=9, n_app=40, tamper_flip=True)
    arena, dgrams = assemble(orc, keys, conns, scripts, seed=7)
    c1, a1 = conns.copy(), arena.copy()
    p1, n1 = orc.batch_recv(keys, c1, a1, dgrams, 4096)
    c2, a2 = conns.copy(), arena.copy()
    p2, n2 = orc.batch_recv(keys, c2, a2, dgrams, 4096, threads=threads)
    assert n1 == n2 and p1.tobytes() == p2.tobytes()
    assert c1.tobytes() == c2.tobytes() and a1.tobytes() == a2.tobytes()
    c3, a3 = conns.copy(), arena.copy()  # max_pkts below the packet count: the same prefix kept
    p3, n3 = orc.batch_recv(keys, c3, a3, dgrams, 50, threads=threads)
    assert n3 == n1 and p3.tobytes() == p1[:50].tobytes() and a3.tobytes() == a1.tobytes()
