"""Synthetic workloads of BASELINE.json's configs, built on the host with numpy.

  B: N x 1200-B 1-RTT packets, ChaCha20-Poly1305; short header 0x43 (pn_len 4, key phase 0),
     8-B DCID, pn_i = 0x10000000 + i, hdr 13 B, plaintext 1171 B; keys from the RFC 9001 A.5
     secret.
  C: as B with AES-128-GCM; keys derived from the RFC 9001 A.1 server initial secret.
  E: mixed batch: L_i ~ U[64, 1350]; 25 % Initial (long header, AES-128-GCM, per-connection
     keys derived from a random 8-B DCID with the A.1 procedure, SCID 8 B, token 0, 2-B Length),
     75 % 1-RTT split 50/50 ChaCha/AES; pn_len ~ U{1..4}; packets interleaved and packed back to
     back (unaligned) in the arena.
Payload bytes come from SplitMix64 seeded with 0x6D696C6C69717569 ("milliqui"); they do not
affect timing (the cryptographic work is data independent).
"""
from dataclasses import dataclass, field

import numpy as np

from . import _lib
from .batch import make_descs
from .key_schedule import derive_initial_secrets, key_material
from .packet import encode_varint

SEED = 0x6D696C6C69717569
A5_SECRET = bytes.fromhex("9ac312a7f877468ebe69422748ad00a15443f18203a07d6060f688f30f21632b")
A1_SERVER_SECRET = bytes.fromhex("3c199828fd139efd216c155ad844cc81fb82fa8d7446fa7d78be803acdda951b")
DCID8 = bytes.fromhex("8394c8f03e515708")

_G = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def splitmix_words(n, seed=SEED, start=0):
    """n SplitMix64 outputs (state_k = seed + (k+1)*golden) for word indices start..start+n-1."""
    with np.errstate(over="ignore"):
        z = (np.arange(start + 1, start + n + 1, dtype=np.uint64) * _G) + np.uint64(seed)
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def splitmix_bytes(nbytes, seed=SEED, chunk=1 << 24, start=0):
    """Bytes [start, start + nbytes) of the SplitMix64 byte stream (words little-endian), so any
    slice of a global batch can be generated on its own (config D shards, sampled packets)."""
    out = np.empty(nbytes, dtype=np.uint8)
    w_first, skip = divmod(start, 8)
    nwords = (skip + nbytes + 7) // 8
    pos = 0
    for w0 in range(0, nwords, chunk):
        b = splitmix_words(min(chunk, nwords - w0), seed, w_first + w0).view(np.uint8)
        if w0 == 0:
            b = b[skip:]
        k = min(len(b), nbytes - pos)
        out[pos:pos + k] = b[:k]
        pos += k
    return out


@dataclass
class Workload:
    name: str
    arena: np.ndarray          # uint8, plaintext packets (headers unprotected), tag areas zero
    seal_desc: np.ndarray      # DESC_DTYPE, pn = full packet number
    open_desc: np.ndarray      # DESC_DTYPE, pn = largest_pn (pn - 1)
    keys: list                 # KeyMaterial rows
    suite_hint: int
    pns: np.ndarray = field(default=None)

    @property
    def n(self):
        return len(self.seal_desc)

    @property
    def wire_bytes(self):
        return int(self.seal_desc["len"].astype(np.int64).sum())


def uniform_keys(suite, n_keys=1):
    """Key rows of configs B / C: row 0 from the RFC 9001 A.5 secret (ChaCha20) or the A.1 server
    secret (AES-128-GCM); the K-key variant adds rows from secrets A.5 + k (byte-wise)."""
    if suite == _lib.MQ_SUITE_CHACHA20:
        base = key_material(suite, A5_SECRET)
    else:
        base = key_material(suite, A1_SERVER_SECRET)
    keys = [base]
    for k in range(1, n_keys):  # variant: K distinct keys, key_id = i mod K
        keys.append(key_material(suite, bytes(((b + k) & 0xFF) for b in A5_SECRET)))
    return keys


def _uniform_headers(view, pns, pn_len, dcid, L):
    hdr_len = 1 + len(dcid)
    view[:, 0] = 0x40 | (pn_len - 1)
    view[:, 1:hdr_len] = np.frombuffer(dcid, dtype=np.uint8)
    for j in range(pn_len):
        view[:, hdr_len + j] = ((pns >> np.uint64(8 * (pn_len - 1 - j))) & np.uint64(0xFF)).astype(np.uint8)
    view[:, L - 16:] = 0


PN0 = 0x10000000


def uniform(n, suite, L=1200, pn_len=4, dcid=DCID8, seed=SEED, n_keys=1, start=0, keys=None):
    """Configs B (ChaCha20) and C (AES-128-GCM): n x L-byte short-header packets.

    Packets are those of global indices start .. start + n - 1 of one global batch: packet g has
    pn = 0x10000000 + g, key row g mod n_keys and payload bytes [g L, (g + 1) L) of the SplitMix64
    stream, so a shard of config D (start = rank x n) is exactly its slice of the 8M batch.
    `keys` (rows) may be passed in, e.g. received from rank 0 (bench.py broadcasts them)."""
    if keys is None:
        keys = uniform_keys(suite, n_keys)
    n_keys = len(keys)
    arena = splitmix_bytes(n * L, seed, start=start * L)
    view = arena.reshape(n, L)
    g = np.arange(start, start + n, dtype=np.uint64)
    pns = np.uint64(PN0) + g
    _uniform_headers(view, pns, pn_len, dcid, L)
    hdr_len = 1 + len(dcid)
    offs = np.arange(n, dtype=np.uint64) * np.uint64(L)
    kid = (g % np.uint64(n_keys)).astype(np.uint32)
    seal = make_descs(offs, L, kid, pns, hdr_len, pn_len, 0)
    opn = make_descs(offs, L, kid, pns - np.uint64(1), hdr_len, 0, 0)
    return Workload(f"{n}x{L}B-{'chacha' if suite == 2 else 'aes'}", arena, seal, opn, keys, suite, pns)


def uniform_at(indices, suite, L=1200, pn_len=4, dcid=DCID8, seed=SEED, keys=None, n_keys=1):
    """The packets of the given global indices of uniform()'s global batch, packed back to back
    (sampled parity checks of sharded runs: the oracle seals exactly these)."""
    if keys is None:
        keys = uniform_keys(suite, n_keys)
    g = np.asarray(indices, dtype=np.uint64)
    n = len(g)
    arena = np.empty(n * L, dtype=np.uint8)
    view = arena.reshape(n, L)
    for k, gi in enumerate(g):
        view[k] = splitmix_bytes(L, seed, start=int(gi) * L)
    pns = np.uint64(PN0) + g
    _uniform_headers(view, pns, pn_len, dcid, L)
    offs = np.arange(n, dtype=np.uint64) * np.uint64(L)
    kid = (g % np.uint64(len(keys))).astype(np.uint32)
    seal = make_descs(offs, L, kid, pns, 1 + len(dcid), pn_len, 0)
    opn = make_descs(offs, L, kid, pns - np.uint64(1), 1 + len(dcid), 0, 0)
    return Workload(f"sample-{n}x{L}B", arena, seal, opn, keys, suite, pns)


def config_b(n=1 << 20, **kw):
    return uniform(n, _lib.MQ_SUITE_CHACHA20, **kw)


def config_c(n=1 << 20, **kw):
    return uniform(n, _lib.MQ_SUITE_AES128GCM, **kw)


LONG_HDR = 1 + 4 + 1 + 8 + 1 + 8 + 1 + 2  # Initial header without the PN: 26 bytes
SHORT_HDR = 1 + 8


@dataclass
class MixedPlan:
    """Per-packet layout of a global config-E batch (no payload bytes): any range or sample of it
    can be built on its own (sharded runs, sampled parity checks)."""
    kind: np.ndarray    # 0 Initial AES, 1 1-RTT ChaCha, 2 1-RTT AES
    pn_len: np.ndarray
    L: np.ndarray
    conn: np.ndarray
    pns: np.ndarray
    offs: np.ndarray    # byte offset of each packet in the global arena (packed back to back)
    dcids: np.ndarray
    keys: list
    seed: int

    @property
    def n(self):
        return len(self.L)


_PLAN_CACHE = {}


def mixed_plan(n=1 << 20, seed=SEED, n_conns=4096, lmin=64, lmax=1350):
    """The layout of config E's n-packet batch (random draws in a fixed order, so that the plan of
    n packets is the same whatever range of it is built later)."""
    ck = (n, seed, n_conns, lmin, lmax)
    if ck in _PLAN_CACHE:
        return _PLAN_CACHE[ck]
    rng = np.random.default_rng(seed & 0xFFFFFFFF)
    kind = rng.choice(3, size=n, p=[0.25, 0.375, 0.375])
    pn_len = rng.integers(1, 5, size=n).astype(np.uint8)
    L = rng.integers(lmin, lmax + 1, size=n).astype(np.int64)
    # key rows: [0] 1-RTT ChaCha (A.5), [1] 1-RTT AES (A.1 server), [2..] Initial per connection
    keys = [key_material(_lib.MQ_SUITE_CHACHA20, A5_SECRET), key_material(_lib.MQ_SUITE_AES128GCM, A1_SERVER_SECRET)]
    dcids = rng.integers(0, 256, size=(n_conns, 8), dtype=np.uint8)
    for c in range(n_conns):
        client, _server = derive_initial_secrets(dcids[c].tobytes())
        keys.append(key_material(_lib.MQ_SUITE_AES128GCM, client))
    conn = rng.integers(0, n_conns, size=n)
    pn_off = np.where(kind == 0, LONG_HDR, SHORT_HDR).astype(np.int64)
    L = np.maximum(L, pn_off + pn_len + 16 + 4).astype(np.int64)  # sample fits: pn_off + 20 <= L
    L = np.maximum(L, pn_off + 20)
    offs = np.zeros(n, dtype=np.int64)
    offs[1:] = np.cumsum(L[:-1])
    pns = (np.uint64(1 << 20) + rng.integers(0, 1 << 30, size=n).astype(np.uint64))
    plan = MixedPlan(kind, pn_len, L, conn, pns, offs, dcids, keys, seed)
    _PLAN_CACHE.clear()  # one plan at a time (an 8 x 2^20 plan holds ~0.5 GB)
    _PLAN_CACHE[ck] = plan
    return plan


def _mixed_build(plan, sel, arena, pos):
    """Headers and descriptors of the plan's packets `sel` (indices), placed at arena offsets `pos`
    (their payload bytes already in the arena)."""
    kind, pn_len, L, pns = plan.kind[sel], plan.pn_len[sel], plan.L[sel], plan.pns[sel]
    conn = plan.conn[sel]
    pn_off = np.where(kind == 0, LONG_HDR, SHORT_HDR).astype(np.int64)
    key_id = np.where(kind == 0, 2 + conn, np.where(kind == 1, 0, 1)).astype(np.uint32)
    flags = np.where(kind == 0, _lib.MQ_PKT_LONG_HEADER, 0).astype(np.uint8)
    s = np.nonzero(kind != 0)[0]
    o = pos[s]
    arena[o] = (0x40 | (pn_len[s] - 1)).astype(np.uint8)
    for j in range(8):
        arena[o + 1 + j] = DCID8[j]
    li = np.nonzero(kind == 0)[0]
    o = pos[li]
    arena[o] = (0xC0 | (pn_len[li] - 1)).astype(np.uint8)
    arena[o + 1] = 0; arena[o + 2] = 0; arena[o + 3] = 0; arena[o + 4] = 1
    arena[o + 5] = 8
    for j in range(8):
        arena[o + 6 + j] = plan.dcids[conn[li], j]
    arena[o + 14] = 8
    for j in range(8):
        arena[o + 15 + j] = (j * 17 + 3) & 0xFF
    arena[o + 23] = 0  # token length
    length = (L[li] - LONG_HDR).astype(np.int64)  # PN + payload + tag
    arena[o + 24] = (0x40 | (length >> 8)).astype(np.uint8)
    arena[o + 25] = (length & 0xFF).astype(np.uint8)
    for j in range(4):
        idx = np.nonzero(pn_len > j)[0]
        shift = (8 * (pn_len[idx].astype(np.int64) - 1 - j)).astype(np.uint64)
        arena[pos[idx] + pn_off[idx] + j] = ((pns[idx] >> shift) & np.uint64(0xFF)).astype(np.uint8)
    # decode_pn must recover pn from pn_len bytes: largest_pn = pn - 1
    seal = make_descs(pos.astype(np.uint64), L.astype(np.uint32), key_id, pns, pn_off.astype(np.uint16), pn_len, flags)
    opn = make_descs(pos.astype(np.uint64), L.astype(np.uint32), key_id, pns - np.uint64(1), pn_off.astype(np.uint16),
                     0, flags)
    return seal, opn


def config_e(n=1 << 20, seed=SEED, n_conns=4096, lmin=64, lmax=1350, lo=0, hi=None):
    """Mixed batch (config E): packets [lo, hi) of the n-packet global batch (default: all of it).
    The range's arena is the global arena's bytes from the 16-B chunk holding packet lo's first
    byte (so a shard is exactly its slice of the global batch), descriptors rebased."""
    plan = mixed_plan(n, seed, n_conns, lmin, lmax)
    hi = n if hi is None else hi
    sel = np.arange(lo, hi)
    if len(sel) == 0:
        from .batch import DESC_DTYPE
        empty = np.zeros(0, dtype=DESC_DTYPE)
        return Workload(f"mixed-{n}[{lo}:{hi}]", np.zeros(16, np.uint8), empty, empty.copy(), plan.keys,
                        _lib.MQ_SUITE_MIXED, np.zeros(0, np.uint64))
    base = int(plan.offs[lo]) & ~15
    end = int(plan.offs[hi - 1] + plan.L[hi - 1])
    arena = splitmix_bytes(end - base, seed, start=base)
    seal, opn = _mixed_build(plan, sel, arena, plan.offs[sel] - base)
    name = f"mixed-{n}" if (lo, hi) == (0, n) else f"mixed-{n}[{lo}:{hi}]"
    return Workload(name, arena, seal, opn, plan.keys, _lib.MQ_SUITE_MIXED, plan.pns[sel])


def config_e_at(indices, n=1 << 20, seed=SEED, n_conns=4096, lmin=64, lmax=1350):
    """The packets of the given global indices of config E's n-packet batch, each with its own
    bytes of the global arena, packed back to back (the oracle seals exactly these)."""
    plan = mixed_plan(n, seed, n_conns, lmin, lmax)
    g = np.asarray(indices, dtype=np.int64)
    Ls = plan.L[g]
    pos = np.zeros(len(g), dtype=np.int64)
    pos[1:] = np.cumsum(Ls[:-1])
    arena = np.empty(int(Ls.sum()), dtype=np.uint8)
    for k, gi in enumerate(g):
        arena[pos[k]:pos[k] + Ls[k]] = splitmix_bytes(int(Ls[k]), seed, start=int(plan.offs[gi]))
    seal, opn = _mixed_build(plan, g, arena, pos)
    return Workload(f"mixed-sample-{len(g)}", arena, seal, opn, plan.keys, _lib.MQ_SUITE_MIXED, plan.pns[g])
