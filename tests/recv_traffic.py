"""Synthetic receive-side traffic for the datagram composite tests (test_recv.py, test_gpu_recv.py).

Packets are built and protected by the oracle's send composite (pinned to RFC 9001 A.5), with
PN lengths chosen from what the receiver has seen (number.rs:9-26), so the receive composite
must recover them (decode_pn against the running largest PN). Per connection: Initial and
Handshake packets coalesced into one datagram (Initial padded to 1200), then 1-RTT packets
with a peer key update (key phase flip to the next generation) part-way; across connections the
datagrams interleave. Extra cases: tampered packets, a Version Negotiation / Retry / 0-RTT
packet (skipped), a truncated long header (iteration stops), a short packet shorter than the
CID, a connection without 1-RTT keys, a phase flip without next-generation keys.
"""
import numpy as np

from milli_quic_amd import _lib, packet, recv, send
from milli_quic_amd.key_schedule import derive_initial_secrets, key_material


def build_traffic(orc, seed=1, n_conns=12, n_app=30, tamper_flip=False):
    """tamper_flip: the first packet of the new key phase is corrupted on every connection, so
    the key update is confirmed by the packet after it (the speculative walk had
    rotated at the flip packet)."""
    rng = np.random.default_rng(seed)
    keys = [_lib.KeyMaterial()]  # row 0: unused
    conns = np.zeros(n_conns, dtype=recv.CONN_DTYPE)
    scripts = []  # per connection: list of (datagram parts), each part = (level, row, phase, pn, frames, tamper)
    for c in range(n_conns):
        dcid = rng.bytes(int(rng.choice([0, 4, 8, 20])))
        client, _ = derive_initial_secrets(rng.bytes(8))
        suite = int(rng.choice([_lib.MQ_SUITE_AES128GCM, _lib.MQ_SUITE_CHACHA20]))
        rows = {}
        rows["init"] = len(keys); keys.append(key_material(_lib.MQ_SUITE_AES128GCM, client))
        rows["hs"] = len(keys); keys.append(key_material(suite, rng.bytes(32)))
        g0 = key_material(suite, rng.bytes(32))
        g1 = key_material(suite, rng.bytes(32))
        g1.hp[:] = g0.hp[:]  # HP keys survive key updates (keys.rs:386-414)
        rows["g0"] = len(keys); keys.append(g0)
        rows["g1"] = len(keys); keys.append(g1)
        conns[c]["initial_row"], conns[c]["handshake_row"] = rows["init"], rows["hs"]
        conns[c]["app_row"] = [0, rows["g0"], rows["g1"]]
        conns[c]["dcid_len"] = len(dcid)
        conns[c]["flags"] = recv.HAS_INITIAL | recv.HAS_HANDSHAKE | recv.HAS_APP | recv.HAS_NEXT
        dg = [[("init", 0, 0, 0, rng.bytes(int(rng.integers(30, 300))), False),
               ("hs", 1, 0, 0, rng.bytes(int(rng.integers(20, 200))), False)],
              [("init", 0, 0, 1, rng.bytes(40), False)],
              [("hs", 1, 0, 1, rng.bytes(int(rng.integers(5, 100))), False),
               ("g0", 2, 0, 0, rng.bytes(int(rng.integers(1, 50))), False)]]
        flip = int(rng.integers(5, n_app - 5))
        pn = 0
        for k in range(n_app):
            pn += int(rng.choice([1, 1, 1, 2, 3, 200, 40000]))
            gen = "g1" if k >= flip else "g0"
            tamper = bool(rng.random() < 0.08) and k not in (flip, flip - 1, flip + 1)
            tamper = tamper or (tamper_flip and k == flip)
            dg.append([(gen, 2, 1 if gen == "g1" else 0, pn, rng.bytes(int(rng.integers(0, 1300))), tamper)])
        scripts.append((dcid, rows, dg))
    return keys, conns, scripts


def protect_one(orc, keys, dcid, level, row, phase, pn, largest, frames, pad):
    cs = send.make_conns([dcid], [b"\x01\x02\x03\x04"], [[row, row, row]], phase)
    req = np.zeros(1, dtype=send.REQ_DTYPE)
    req["pn"], req["largest_acked"], req["frame_len"] = pn, largest, len(frames)
    req["out_cap"], req["level"] = 4096, level
    req["flags"] = send.PAD_TO_MIN if pad else 0
    out = np.zeros(4096, dtype=np.uint8)
    st, ln = orc.batch_protect(keys, cs, np.frombuffer(frames + b"\0", dtype=np.uint8), out, req, _lib.MQ_SUITE_MIXED)
    assert st[0] == 0
    return out[:ln[0]].tobytes()


def assemble(orc, keys, conns, scripts, seed=1, extras=True):
    """Interleave the connections' datagrams (per-connection order kept) into one arena."""
    rng = np.random.default_rng(seed + 100)
    largest = np.zeros((len(scripts), 3), dtype=np.int64)  # what the receiver will have seen
    queues = []
    for c, (dcid, rows, dgs) in enumerate(scripts):
        q = []
        for parts in dgs:
            blob = b""
            for (name, level, phase, pn, frames, tamper) in parts:
                la = int(largest[c, level])
                p = protect_one(orc, keys, dcid, level, rows[name], phase, pn, la, frames,
                                pad=(level == 0 and len(parts) > 1))
                if tamper:
                    b = bytearray(p)
                    b[-20] ^= 0x10
                    p = bytes(b)
                else:
                    largest[c, level] = max(la, pn)
                blob += p
            q.append((c, blob))
        queues.append(q)
    order = []
    idx = [0] * len(queues)
    while any(idx[c] < len(queues[c]) for c in range(len(queues))):
        c = int(rng.choice([k for k in range(len(queues)) if idx[k] < len(queues[k])]))
        order.append(queues[c][idx[c]])
        idx[c] += 1
    if extras:
        c0 = 0
        vn = bytes([0x80]) + bytes(4) + bytes([0]) + bytes([0]) + b"\x00\x00\x00\x01"
        retry = bytes([0xF0]) + (1).to_bytes(4, "big") + bytes([0, 0]) + rng.bytes(20)
        zrtt = bytes([0xD0]) + (1).to_bytes(4, "big") + bytes([0, 0]) + packet.encode_varint(10) + rng.bytes(10)
        trunc = bytes([0xC0]) + (1).to_bytes(4, "big") + bytes([30]) + rng.bytes(5)  # DCID runs past the end
        order += [(c0, vn), (c0, retry), (c0, zrtt + bytes([0x40]) + rng.bytes(30)), (c0, trunc)]
        order.append((c0, bytes([0x40])))                      # shorter than 1 + dcid_len -> BTS
        order.append((1, bytes([0x45]) + rng.bytes(60)))       # phase flip garbage
    dgrams = np.zeros(len(order), dtype=recv.DGRAM_DTYPE)
    pos, blobs = 0, []
    for i, (c, blob) in enumerate(order):
        pos = (pos + 7) // 8 * 8 if i % 3 else pos  # some unaligned datagrams
        dgrams[i]["offset"], dgrams[i]["len"], dgrams[i]["conn"] = pos, len(blob), c
        blobs.append((pos, blob))
        pos += len(blob)
    arena = np.zeros(pos + 64, dtype=np.uint8)
    for o, b in blobs:
        arena[o:o + len(b)] = np.frombuffer(b, dtype=np.uint8)
    return arena, dgrams


def build_pn_jump(orc, suites=(_lib.MQ_SUITE_CHACHA20, _lib.MQ_SUITE_AES128GCM), seed=7):
    """ADVICE r02 (mq_recv.hip walk): per connection, a packet X with a large PN jump arrives
    corrupted, and the sender, believing X acknowledged, encodes the next two packets' PNs in one
    byte against it. The sequential reference never advances its largest PN past X, so it decodes
    those PNs wrongly and fails them (Error::Crypto, datagram untouched); the batch's speculation
    (X opens) decodes them right and opens them. A later packet with a long PN opens for both.
    Returns keys, conns, arena, dgrams (one packet per datagram)."""
    rng = np.random.default_rng(seed)
    keys = [_lib.KeyMaterial()]
    conns = np.zeros(len(suites), dtype=recv.CONN_DTYPE)
    order = []
    for c, suite in enumerate(suites):
        dcid = rng.bytes(8)
        row = len(keys)
        keys.append(key_material(suite, rng.bytes(32)))
        conns[c]["app_row"] = [0, row, 0]
        conns[c]["dcid_len"] = 8
        conns[c]["flags"] = recv.HAS_APP
        # (pn, the sender's largest acknowledged pn, tampered)
        for pn, la, tamper in ((1, 0, False), (1000, 1, False), (41000, 1000, True), (41005, 41000, False),
                               (41006, 41005, False), (41100, 1000, False), (41101, 41100, False)):
            p = protect_one(orc, keys, dcid, 2, row, 0, pn, la, rng.bytes(int(rng.integers(20, 200))), False)
            if tamper:
                b = bytearray(p)
                b[-20] ^= 0x10
                p = bytes(b)
            order.append((c, p))
    dgrams = np.zeros(len(order), dtype=recv.DGRAM_DTYPE)
    pos, blobs = 0, []
    for i, (c, blob) in enumerate(order):
        dgrams[i]["offset"], dgrams[i]["len"], dgrams[i]["conn"] = pos, len(blob), c
        blobs.append((pos, blob))
        pos += len(blob) + 3
    arena = np.zeros(pos + 64, dtype=np.uint8)
    for o, b in blobs:
        arena[o:o + len(b)] = np.frombuffer(b, dtype=np.uint8)
    return keys, conns, arena, dgrams


def long_runs(orc, n_conns, n_per_conn, seed=1, frame_min=20, frame_max=300, gap_p=0.02, big_gap_p=0.001,
              reorder_p=0.01, tamper_p=0.005, flip_at=0.5, lag_max=100, interleave=True):
    """Long 1-RTT runs for the segmented receive walk (r05, mq_recv.hip kSeg): n_conns connections
    of n_per_conn one-packet datagrams each, built by the oracle's send composite in one batch.
    PNs mostly step by 1, with gaps (2..300, rarely ~40000: the sender's largest acknowledged PN
    then lags behind the gap, so its PN length covers it, number.rs:9-26), adjacent packets swapped
    in flight (in-window reordering), a peer key update (phase 1, next-generation keys) from
    packet flip_at * n on, and tampered packets (one flipped bit). Suites alternate ChaCha20 /
    AES-128-GCM by connection. Returns keys, conns, arena, dgrams."""
    rng = np.random.default_rng(seed)
    keys = [_lib.KeyMaterial()]
    rconns = np.zeros(n_conns, dtype=recv.CONN_DTYPE)
    sconns = []
    reqs = []
    frames = []
    fpos = 0
    per_conn_order = []
    for c in range(n_conns):
        suite = _lib.MQ_SUITE_CHACHA20 if c % 2 == 0 else _lib.MQ_SUITE_AES128GCM
        dcid = rng.bytes(8)
        g0 = key_material(suite, rng.bytes(32))
        g1 = key_material(suite, rng.bytes(32))
        g1.hp[:] = g0.hp[:]  # HP keys survive key updates (keys.rs:386-414)
        r0 = len(keys); keys.append(g0)
        r1 = len(keys); keys.append(g1)
        rconns[c]["app_row"] = [0, r0, r1]
        rconns[c]["dcid_len"] = 8
        rconns[c]["flags"] = recv.HAS_APP | recv.HAS_NEXT
        s0 = len(sconns)
        sconns.append((dcid, r0, 0))
        sconns.append((dcid, r1, 1))
        inc = np.ones(n_per_conn, dtype=np.int64)
        u = rng.random(n_per_conn)
        inc[u < gap_p] = rng.integers(2, 300, size=int((u < gap_p).sum()))
        inc[u < big_gap_p] = 40000 + rng.integers(0, 1000, size=int((u < big_gap_p).sum()))
        pns = np.cumsum(inc) + int(rng.integers(0, 1 << 20))
        rconns[c]["largest_pn"][2] = int(pns[0]) - 1  # the run continues what the receiver has seen
        flip = int(flip_at * n_per_conn)
        order = np.arange(n_per_conn)
        for k in range(1, n_per_conn - 1):  # adjacent swaps in flight
            if rng.random() < reorder_p and order[k] == k and order[k + 1] == k + 1:
                order[k], order[k + 1] = k + 1, k
        if 2 <= flip < n_per_conn - 1:  # the first new-phase packet overtakes the last old-phase one
            order[flip - 2:flip + 2] = [flip - 2, flip, flip - 1, flip + 1]
        lag = rng.integers(1, lag_max + 1, size=n_per_conn)
        tamper = set(int(x) for x in np.nonzero(rng.random(n_per_conn) < tamper_p)[0])
        idx0 = len(reqs)
        acked = int(pns[0]) - 1  # the largest PN the receiver accepted so far (what ACKs could report)
        for k in range(n_per_conn):
            pn = int(pns[k])
            prev = int(pns[k - 1]) if k else pn - 1
            # the sender's largest acknowledged PN: behind the last sent, never past what the
            # receiver accepted (a tampered packet is never acknowledged)
            la = max(0, min(prev - int(lag[k]), acked))
            if k not in tamper:
                acked = max(acked, pn)
            fl = int(rng.integers(frame_min, frame_max + 1))
            frames.append(rng.bytes(fl))
            reqs.append((fpos, pn, la, fl, s0 + (1 if k >= flip else 0)))
            fpos += fl
        per_conn_order.append([(c, idx0 + int(k), int(k) in tamper) for k in order])
    sc = send.make_conns([d for d, _, _ in sconns], [b"\x01\x02\x03\x04"] * len(sconns),
                         [[r, r, r] for _, r, _ in sconns], 0)
    sc["key_phase"] = [p for _, _, p in sconns]
    n = len(reqs)
    req = np.zeros(n, dtype=send.REQ_DTYPE)
    cap = frame_max + 64
    req["frames_offset"] = [r[0] for r in reqs]
    req["out_offset"] = np.arange(n, dtype=np.uint64) * np.uint64(cap)
    req["pn"] = [r[1] for r in reqs]
    req["largest_acked"] = [r[2] for r in reqs]
    req["frame_len"] = [r[3] for r in reqs]
    req["out_cap"] = cap
    req["conn"] = [r[4] for r in reqs]
    req["level"] = send.APPLICATION
    fr = np.frombuffer(b"".join(frames) + b"\0", dtype=np.uint8)
    out = np.zeros(n * cap, dtype=np.uint8)
    st, ln = orc.batch_protect(keys, sc, fr, out, req, _lib.MQ_SUITE_MIXED)
    assert (st == 0).all()
    # arrival order: the connections' (reordered) sequences, interleaved at random or one after another
    seqs = [list(s) for s in per_conn_order]
    arrival = []
    if interleave:
        pos = [0] * n_conns
        left = [len(s) for s in seqs]
        while sum(left):
            c = int(rng.choice([k for k in range(n_conns) if left[k]]))
            take = min(left[c], int(rng.integers(1, 64)))
            arrival += seqs[c][pos[c]:pos[c] + take]
            pos[c] += take
            left[c] -= take
    else:
        for s in seqs:
            arrival += s
    dgrams = np.zeros(n, dtype=recv.DGRAM_DTYPE)
    total = int(ln.astype(np.int64).sum()) + 16 * n
    arena = np.zeros(total + 64, dtype=np.uint8)
    p = 0
    for i, (c, r, tam) in enumerate(arrival):
        L = int(ln[r])
        b = out[r * cap:r * cap + L].copy()
        if tam:
            b[L - 20] ^= 0x10
        p = (p + 7) // 8 * 8 if i % 3 else p
        arena[p:p + L] = b
        dgrams[i]["offset"], dgrams[i]["len"], dgrams[i]["conn"] = p, L, c
        p += L
    return keys, rconns, arena, dgrams
