// mq_recv.hip — the receive composite over raw UDP datagrams on gfx950.
//
// The reference's Connection::recv (src/connection/recv.rs:189-265) walks the coalesced packets
// of each datagram (src/packet/coalesce.rs:26-133), parses long headers (long_header.rs:92-206),
// removes header protection, decodes the packet number against the connection's running
// largest_recv_pn, picks 1-RTT keys by the key-phase bit (current, previous on failure, next +
// rotation on a flip; recv.rs:410-509) and opens the payload. Per connection this is a sequential
// state machine; across connections it is independent. On the device:
//
//   split   one lane per datagram: CoalescedPackets -> packet records (count, scan, emit, so
//           records stay in arrival order)
//   masks   the header-protection pre-pass kernels of the suites (one lane per packet)
//   sort    stable radix sort of record indices by connection (hipCUB) -> per-connection runs
//   plan    one lane per connection walks its run in arrival order: unmasks the first byte,
//           decodes the PN against the running largest PN, chooses the key generation, and
//           SPECULATES that every packet opens (largest PN / rotation advance) -> descriptors
//   open    the ChaCha20-Poly1305 / AES-128-GCM tile kernels, then a retry pass with the
//           previous-generation keys for 1-RTT packets that failed with the current ones
//   commit  one lane per connection replays its run with the real outcomes: statuses, PNs and
//           the connection state; a packet whose inputs the speculation got wrong (only possible
//           after an earlier packet of the connection failed) and that did not open is
//           MQ_ERR_DEFERRED (untouched, to be resubmitted)
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "mq_device.h"
#include "mq_opts.h"

using namespace mq;

namespace {

constexpr uint8_t kPending = 0xFF;
constexpr uint32_t kNoRow = 0xFFFFFFFFu;

// working record of one packet (workspace)
struct RecvWork {
  uint64_t offset;    // packet start in the arena
  uint32_t len;       // long: pn_offset + Length; short: rest of the datagram
  uint32_t dgram;
  uint32_t conn;
  uint16_t pn_off;    // long: from the header; short: 1 + dcid_len (set by plan)
  uint8_t level;
  uint8_t pre;        // kPending, or a status found before any crypto
};

// speculative plan of one packet (workspace)
struct RecvPlan {
  uint64_t pn;        // decoded PN
  uint64_t lbefore;   // largest PN of its level before it
  uint32_t row;       // key row opened with (primary)
  uint32_t retry;     // previous-generation row for the retry pass, or kNoRow
  uint32_t trunc;     // truncated PN (header protection removed; state independent)
  uint8_t status;     // kPending (to open) or a final status
  uint8_t gen;        // key generation of `row`
  uint8_t phase;      // key-phase bit of the unmasked first byte
  uint8_t pn_len;
};

__device__ __forceinline__ bool get_varint(const uint8_t* p, uint64_t avail, uint64_t& v, uint32_t& used) {
  if (avail < 1) return false;
  const uint32_t n = 1u << (p[0] >> 6);
  if (avail < n) return false;
  uint64_t x = p[0] & 0x3f;
  for (uint32_t i = 1; i < n; ++i) x = (x << 8) | p[i];
  v = x;
  used = n;
  return true;
}

// CoalescedPackets::next (coalesce.rs:29-132). kind: 0 Initial, 1 0-RTT, 2 Handshake, 3 Retry,
// 4 short, 5 version negotiation. false = the datagram's iteration stops here.
__device__ __forceinline__ bool next_packet(const uint8_t* r, uint64_t avail, uint64_t& plen, int& kind,
                                            uint32_t& pn_off) {
  if (!(r[0] & 0x80)) { plen = avail; kind = 4; return true; }
  if (avail < 6) return false;
  const uint32_t version = ((uint32_t)r[1] << 24) | ((uint32_t)r[2] << 16) | ((uint32_t)r[3] << 8) | r[4];
  if (version == 0) { plen = avail; kind = 5; return true; }
  uint64_t pos = 6 + (uint64_t)r[5];
  if (pos >= avail) return false;
  const uint64_t scid = r[pos++];
  if (pos + scid > avail) return false;
  pos += scid;
  const int type = (r[0] & 0x30) >> 4;
  uint64_t v;
  uint32_t used;
  if (type == 0) {
    if (!get_varint(r + pos, avail - pos, v, used)) return false;
    pos += used;
    if (v > avail - pos) return false;
    pos += v;
  }
  if (type == 3) { plen = avail; kind = 3; return true; }
  if (!get_varint(r + pos, avail - pos, v, used)) return false;
  pos += used;
  if (v > avail - pos) return false;
  plen = pos + v;
  kind = type;
  pn_off = (uint32_t)pos;
  return true;
}

__device__ __forceinline__ uint64_t decode_pn(uint32_t truncated, uint32_t pn_len, uint64_t largest) {
  const uint64_t win = 1ull << (8 * pn_len), hwin = win >> 1, mask = win - 1;
  const uint64_t expected = largest + 1;
  const uint64_t cand = (expected & ~mask) | truncated;
  if (cand + hwin <= expected && cand + win <= (1ull << 62)) return cand + win;
  if (cand > expected + hwin && cand >= win) return cand - win;
  return cand;
}

}  // namespace

// ---- split ------------------------------------------------------------------------------------
extern "C" __global__ __launch_bounds__(256) void mq_recv_split_kernel(
    const uint8_t* __restrict__ arena, uint64_t arena_len, const mq_dgram* __restrict__ dg, uint32_t n_dgrams,
    uint32_t n_conns, uint32_t* __restrict__ counts, const uint32_t* __restrict__ base, RecvWork* __restrict__ work,
    uint32_t max_pkts) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n_dgrams) return;
  const mq_dgram d = dg[g];
  uint32_t k = 0;
  if (d.conn < n_conns && d.offset + (uint64_t)d.len <= arena_len) {
    const uint8_t* b = arena + d.offset;
    uint64_t off = 0;
    while (off < d.len) {
      uint64_t plen = 0;
      int kind = 0;
      uint32_t pn_off = 0;
      if (!next_packet(b + off, d.len - off, plen, kind, pn_off)) break;
      if (kind != 1 && kind != 3 && kind != 5) {  // 0-RTT, Retry, VN are skipped (recv.rs:221-226)
        if (base) {
          const uint32_t at = base[g] + k;
          if (at < max_pkts) {
            RecvWork w;
            w.offset = d.offset + off;
            w.len = (uint32_t)plen;
            w.dgram = g;
            w.conn = d.conn;
            w.pn_off = (uint16_t)pn_off;
            w.level = kind == 0 ? MQ_LEVEL_INITIAL : kind == 2 ? MQ_LEVEL_HANDSHAKE : MQ_LEVEL_APPLICATION;
            w.pre = kPending;
            work[at] = w;
          }
        }
        ++k;
      }
      off += plen;
    }
  }
  if (!base) counts[g] = k;
}

// sort keys / values and the provisional descriptors the header-protection pre-pass reads
extern "C" __global__ __launch_bounds__(256) void mq_recv_prep_kernel(
    const mq_conn_recv* __restrict__ conns, const uint32_t* __restrict__ total, RecvWork* __restrict__ work,
    uint32_t max_pkts, uint32_t n_rows, uint32_t* __restrict__ keys, uint32_t* __restrict__ vals,
    mq_pkt_desc* __restrict__ desc) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= max_pkts) return;
  const uint32_t n = min(*total, max_pkts);
  vals[i] = i;
  mq_pkt_desc d;
  d.offset = 0; d.len = 0; d.key_id = kNoRow; d.pn = 0; d.pn_offset = 0; d.pn_len = 0; d.flags = 0; d.reserved = 0;
  if (i >= n) {
    keys[i] = 0xFFFFFFFFu;
    desc[i] = d;
    return;
  }
  RecvWork w = work[i];
  const mq_conn_recv c = conns[w.conn];
  keys[i] = w.conn;
  if (w.level == MQ_LEVEL_APPLICATION) w.pn_off = (uint16_t)(1 + c.dcid_len);
  // checks of recv_initial / recv_handshake / recv_short before the sample is read
  uint8_t pre = kPending;
  uint32_t row = kNoRow;
  if (w.level == MQ_LEVEL_APPLICATION) {
    if (w.len < 1u + c.dcid_len) pre = MQ_ERR_BUFFER_TOO_SMALL;  // parse_short_header
    else if (!(c.flags & MQ_RECV_HAS_APP) || c.app_row[1] >= n_rows) pre = MQ_ERR_CRYPTO;
    else if (w.len > 2048) pre = MQ_ERR_BUFFER_TOO_SMALL;          // recv.rs:356-360
    else row = c.app_row[1];                                          // HP keys of every generation
  } else {
    const bool ini = w.level == MQ_LEVEL_INITIAL;
    const uint32_t r = ini ? c.initial_row : c.handshake_row;
    if (!(c.flags & (ini ? MQ_RECV_HAS_INITIAL : MQ_RECV_HAS_HANDSHAKE)) || r >= n_rows) pre = MQ_ERR_CRYPTO;
    else if (w.len > 2048) pre = MQ_ERR_BUFFER_TOO_SMALL;          // decrypt_long_packet :963-965
    else row = r;
  }
  if (pre == kPending && (uint32_t)w.pn_off + 20 > w.len) pre = MQ_ERR_CRYPTO;  // sample (:364-366, :970-973)
  w.pre = pre;
  work[i] = w;
  if (pre == kPending) {
    d.offset = w.offset; d.len = w.len; d.key_id = row; d.pn_offset = w.pn_off;
    d.flags = w.level != MQ_LEVEL_APPLICATION ? MQ_PKT_LONG_HEADER : 0;
  }
  desc[i] = d;
}

// per-connection run boundaries in the sorted order
extern "C" __global__ __launch_bounds__(256) void mq_recv_seg_kernel(const uint32_t* __restrict__ skeys,
                                                                     uint32_t max_pkts, uint32_t n_conns,
                                                                     uint32_t* __restrict__ seg_lo,
                                                                     uint32_t* __restrict__ seg_hi) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= max_pkts) return;
  const uint32_t k = skeys[s];
  if (k >= n_conns) return;
  if (s == 0 || skeys[s - 1] != k) seg_lo[k] = s;
  if (s + 1 == max_pkts || skeys[s + 1] != k) seg_hi[k] = s + 1;
}

// ---- plan: one lane per connection, speculating that every packet opens -----------------------
struct ConnState {
  uint64_t largest[3];
  uint32_t row[3];
  uint8_t phase, flags, updates;
};

// the running largest PN of a level, without indexing the array by a run-time value (an indexed
// private array lives in scratch memory: r03's walk waited on a scratch round trip per packet)
__device__ __forceinline__ uint64_t largest_of(const ConnState& s, uint32_t level) {
  return level == 0 ? s.largest[0] : level == 1 ? s.largest[1] : s.largest[2];
}
__device__ __forceinline__ void raise_largest(ConnState& s, uint32_t level, uint64_t pn) {
#pragma unroll
  for (uint32_t l = 0; l < 3; ++l)
    if (level == l && pn > s.largest[l]) s.largest[l] = pn;
}

__device__ __forceinline__ ConnState load_state(const mq_conn_recv& c) {
  ConnState s;
  for (int l = 0; l < 3; ++l) { s.largest[l] = c.largest_pn[l]; s.row[l] = c.app_row[l]; }
  s.phase = c.key_phase;
  s.flags = c.flags;
  s.updates = c.key_updates;
  return s;
}

// header-protection removal of one packet from the arena as received: truncated PN, PN length and
// key-phase bit (recv.rs:363-391, :968-992); independent of the connection state
__device__ __forceinline__ void unmask(const RecvWork& w, const uint8_t* arena, uint2 m, RecvPlan& p) {
  const bool lng = w.level != MQ_LEVEL_APPLICATION;
  const uint8_t* pk = arena + w.offset;
  // the first byte and the four bytes at pn_offset in one round of loads (a pending packet has
  // pn_offset + 20 <= len, so all four lie inside it)
  const uint8_t raw0 = pk[0];
  const uint32_t pnw = *(const u32_u*)(pk + w.pn_off) ^ ((m.x >> 8) | (m.y << 24));
  const uint8_t b0 = raw0 ^ ((uint8_t)m.x & (lng ? 0x0f : 0x1f));
  const uint32_t pn_len = (b0 & 3u) + 1;
  uint32_t trunc = 0;
  for (uint32_t b = 0; b < pn_len; ++b) trunc = (trunc << 8) | ((pnw >> (8 * b)) & 0xffu);
  p.trunc = trunc;
  p.pn_len = (uint8_t)pn_len;
  p.phase = (b0 >> 2) & 1;
  p.row = b0;  // header entries carry the unmasked first byte here (the open pre-pass value)
}

// what the sequential reference decides for one packet in state s: decoded PN and key choice
// (status kPending = goes to the AEAD); p.trunc / pn_len / phase from unmask()
__device__ __forceinline__ void decide(const ConnState& s, const RecvWork& w, const mq_conn_recv& c, uint32_t n_rows,
                                       RecvPlan& p) {
  p.retry = kNoRow;
  p.gen = 1;
  p.row = kNoRow;
  p.pn = 0;
  p.lbefore = 0;
  p.status = w.pre;
  if (w.pre != kPending) return;
  p.lbefore = largest_of(s, w.level);
  p.pn = decode_pn(p.trunc, p.pn_len, p.lbefore);
  if (p.pn > (1ull << 62) - 1) { p.status = MQ_ERR_PROTOCOL; return; }  // recv.rs:393-395, 994-997
  if (w.level != MQ_LEVEL_APPLICATION) {
    p.row = w.level == MQ_LEVEL_INITIAL ? c.initial_row : c.handshake_row;
  } else if (p.phase == s.phase) {
    p.row = s.row[1];
    if ((s.flags & MQ_RECV_HAS_PREV) && s.row[0] < n_rows) p.retry = s.row[0];
  } else if (!(s.flags & MQ_RECV_HAS_NEXT) || s.row[2] >= n_rows) {
    // no next-generation keys: derive_next_recv_keys fails (Crypto) when none were installed;
    // after a rotation in this batch the next-next keys need the host (DEFERRED)
    p.status = s.updates != c.key_updates ? (uint8_t)MQ_ERR_DEFERRED : (uint8_t)MQ_ERR_CRYPTO;
  } else {
    p.row = s.row[2];
    p.gen = 2;
  }
}

__device__ __forceinline__ void advance(ConnState& s, const RecvWork& w, const RecvPlan& p, uint8_t gen) {
  raise_largest(s, w.level, p.pn);  // recv.rs:239-247
  if (w.level == MQ_LEVEL_APPLICATION && gen == 2) {          // confirm_peer_key_update (keys.rs:532-583)
    s.row[0] = s.row[1];
    s.row[1] = s.row[2];
    s.flags = (uint8_t)((s.flags | MQ_RECV_HAS_PREV) & ~MQ_RECV_HAS_NEXT);
    s.phase ^= 1;
    s.updates++;
  }
}

// Records in connection order (r04): everything after the sort — the walks, the AEAD passes'
// descriptors and statuses, the outcomes — is indexed by the sorted position k, so a walk reads each
// connection's run contiguously; only the output records keep arrival order. The header-protection
// removal (state independent) happens here too, straight into connection order (r04: it was a
// pass of its own in arrival order, 64 us per 2^20 packets, profiles/r04k2_kernel_trace_recv.csv).
extern "C" __global__ __launch_bounds__(256) void mq_recv_gather_kernel(const uint32_t* __restrict__ total,
                                                                        uint32_t max_pkts,
                                                                        const uint32_t* __restrict__ svals,
                                                                        const RecvWork* __restrict__ work,
                                                                        const uint8_t* __restrict__ arena,
                                                                        const uint2* __restrict__ hpm,
                                                                        RecvWork* __restrict__ work_s,
                                                                        RecvPlan* __restrict__ hdr_s,
                                                                        uint8_t* __restrict__ outcome) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= max_pkts) return;
  outcome[k] = 0;
  if (k >= min(*total, max_pkts)) return;
  const uint32_t i = svals[k];
  const RecvWork w = work[i];
  RecvPlan p{};
  if (w.pre == kPending) unmask(w, arena, hpm[i], p);
  work_s[k] = w;
  hdr_s[k] = p;
}

// ---- walk: connections replay their packets in arrival order ---------------------------------------
// With every outcome known so far it decides each packet exactly as the sequential reference does;
// a packet whose AEAD attempt is missing or was made with other inputs gets a new attempt (d1 / d2)
// and is SPECULATED to open, so the walk can go on. Repeated after each pair of AEAD passes until
// nothing new is attempted; the last walk (`final`) marks what is still unresolved DEFERRED.
enum : uint8_t { kNone = 0, kOk1 = 1, kOk0 = 2, kFail = 3 };

// A connection per wave (r04). The wave loads the inputs of its next 64 packets together (lane q:
// packet k0 + q of the run, contiguous in sorted order) and decides them IN PARALLEL against the
// state at the chunk's start: every lane decodes its PN with that largest PN, takes its decision and
// outcome, then a per-level exclusive prefix max over the lanes gives the largest PN each packet
// really follows (only opened packets raise it, recv.rs:239-247) and the lanes decide again with
// it. The chunk is exact when every PN comes out the same (induction over the lanes: same PNs, same
// statuses, so the same prefix max) and no packet confirms a key update (the only other state
// change, keys.rs:532-583). Otherwise — a PN window crossing or a rotation in the chunk — the
// wave's first lane replays the chunk in arrival order from LDS, as the sequential reference does.
// Then every lane writes its packet's descriptors, attempt and output record. r03 walked one
// packet per lane-step straight from memory (372 us per walk of 2^20 packets over 4096
// connections, three walks per batch); r04's first version, a 16-lane group per connection whose
// first lane replayed every packet, still took 285-310 us (profiles/r04j_kernel_trace_recv.csv):
// ~600 single-lane instructions per packet.
struct WalkIn {      // 32 B: the state-dependent decision's inputs
  uint64_t tpn;      // last attempt: pn, rows, generation (tried[k]); o = its outcome
  uint32_t trow, tretry;
  uint32_t trunc;
  uint8_t pn_len, phase, level, pre;
  uint8_t o, tgen, pad0, pad1;
  uint32_t pad2;
};
struct WalkOut {     // 32 B: the decision
  uint64_t pn, lbefore;
  uint32_t row, retry;
  uint8_t st, gen, pgen, mode;  // mode: 0 no AEAD, 1 (re)attempt, 2 hand to the re-seal pass
  uint32_t pad;
};
constexpr uint32_t kWalkThreads = 256, kWalkConns = kWalkThreads / kWave;

// the sequential reference's decision for one packet in state s, and its outcome from what is known
// (the state is advanced by the caller: raise_largest / advance when st == MQ_OK)
__device__ __forceinline__ WalkOut walk_eval(const ConnState& s, const mq_conn_recv& c, uint32_t n_rows,
                                             const WalkIn& in, int final_walk) {
  RecvWork w;
  w.level = in.level;
  w.pre = in.pre;
  RecvPlan p;
  p.trunc = in.trunc;
  p.pn_len = in.pn_len;
  p.phase = in.phase;
  decide(s, w, c, n_rows, p);
  WalkOut r;
  r.pn = p.pn; r.lbefore = p.lbefore; r.row = p.row; r.retry = p.retry; r.pgen = p.gen; r.pad = 0;
  uint8_t st = p.status, gen = p.gen, mode = 0;
  if (p.status == kPending) {
    const bool same = in.o != kNone && in.tpn == p.pn && in.trow == p.row && in.tretry == p.retry && in.tgen == p.gen;
    if (in.o == kOk1 || in.o == kOk0) {
      // Opened (its bytes are already plaintext, so it is never attempted again). A packet
      // authenticates under exactly one (key row, pn), the one that opened it, so the reference's
      // outcome for its own decision p follows: p.row first, then p.retry (recv.rs:412-474); for
      // a next-generation open the rotation is p's (gen 2).
      const uint32_t opened = in.o == kOk1 ? in.trow : in.tretry;
      if (in.tpn == p.pn && opened == p.row) {
        st = MQ_OK;
      } else if (in.tpn == p.pn && opened == p.retry) {
        st = MQ_OK;
        gen = 0;
      } else {
        // the reference's keys fail on it: Error::Crypto. It opened under the speculation's
        // inputs, so its bytes hold plaintext; the final walk hands it to the re-seal pass
        // (mq_host.cpp) with the key row and PN that opened it, which brings back ciphertext, tag
        // and masked header exactly as received — the reference never touches the datagram of a
        // failed packet (it opens a 2048-B copy, recv.rs:356-361)
        st = MQ_ERR_CRYPTO;
        if (final_walk) mode = 2;
      }
    } else if (same) {  // failed with exactly the reference's inputs
      st = MQ_ERR_CRYPTO;
    } else if (final_walk) {
      st = MQ_ERR_DEFERRED;
    } else {  // (re)attempt with the inputs the reference would use; speculate it opens
      mode = 1;
      st = MQ_OK;
    }
  }
  r.st = st;
  r.gen = gen;
  r.mode = mode;
  return r;
}

__device__ __forceinline__ uint64_t shfl_up_u64(uint64_t x, int d) {
  const uint32_t lo = (uint32_t)__shfl_up((int)(uint32_t)x, d, kWave), hi = (uint32_t)__shfl_up((int)(uint32_t)(x >> 32), d, kWave);
  return (uint64_t)hi << 32 | lo;
}
// exclusive prefix max over the wave's lanes (lane 0: 0) and the wave's total max
__device__ __forceinline__ uint64_t excl_max_u64(uint64_t v, uint32_t lane, uint64_t& total) {
  uint64_t x = v;
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    const uint64_t y = shfl_up_u64(x, d);
    if (lane >= (uint32_t)d) x = x > y ? x : y;
  }
  total = (uint64_t)__builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), kWave - 1) << 32 |
          (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, kWave - 1);
  const uint64_t e = shfl_up_u64(x, 1);
  return lane == 0 ? 0ull : e;
}

// Long runs across waves (r05): a connection's run is cut into SEGMENTS of at most
// kSeg packets, one wave each, so 2^20 packets over one connection are walked by 512 waves instead
// of one (12.5 GiB/s in r04: 16 k sequential chunk steps per walk). Segment 0 starts from the
// connection's state; a later segment starts from a guess — the state at the batch start with the
// largest PN of its first packet's level set just below that packet's PN, decoded against the
// batch-start largest PN plus the packets before it in the run (exact for in-order runs whose PNs
// stay inside the PN window of the guess). Its walk is then the usual exact chunk walk from that
// state. After a walk a verify pass re-walks every later segment from the end state its
// predecessor recorded and compares each packet's decision with the records: if every segment of a
// connection agrees, the chained walk equals the sequential one (induction over the segments);
// otherwise (a key update, a PN gap or reordering across a segment boundary outside the window)
// the connection is flagged and walked again sequentially from its batch-start state by one wave
// (fallback). The earlier walks only speculate (their attempts are checked by the AEAD passes
// and the final walk), so they take the guessed starts unverified.
constexpr uint32_t kSeg = 1024;
constexpr uint32_t kNoSeg = 0xFFFFFFFFu;  // one segment per run
// the segment length in packets: kSeg, or MQ_RECV_SEG (diagnostic, mq_opts.h; 0 = one segment per
// run, the r04 walk). Read ONCE per batch (mq_batch_recv) and handed to every walk: segprev[] slots
// are indexed by the segment layout, which must not change between the walks of a batch.
uint32_t mq_recv_seg_len() {
  const long v = mq::opt(mq::Opt::RecvSeg);
  if (v < 0) return kSeg;
  return v == 0 ? kNoSeg : (uint32_t)(v < 64 ? 64 : (unsigned long)v & ~63ul);  // whole walk chunks
}
struct SegState { uint64_t largest[3]; uint32_t row[3]; uint32_t misc; };  // misc: phase | flags << 8 | updates << 16

__device__ __forceinline__ SegState pack_state(const ConnState& s) {
  SegState x;
  for (int l = 0; l < 3; ++l) { x.largest[l] = s.largest[l]; x.row[l] = s.row[l]; }
  x.misc = s.phase | (uint32_t)s.flags << 8 | (uint32_t)s.updates << 16;
  return x;
}
__device__ __forceinline__ ConnState unpack_state(const SegState& x) {
  ConnState s;
  for (int l = 0; l < 3; ++l) { s.largest[l] = x.largest[l]; s.row[l] = x.row[l]; }
  s.phase = (uint8_t)x.misc;
  s.flags = (uint8_t)(x.misc >> 8);
  s.updates = (uint8_t)(x.misc >> 16);
  return s;
}
__device__ __forceinline__ bool same_state(const ConnState& a, const ConnState& b) {
  bool eq = a.phase == b.phase && a.flags == b.flags && a.updates == b.updates;
  for (int l = 0; l < 3; ++l) eq = eq && a.largest[l] == b.largest[l] && a.row[l] == b.row[l];
  return eq;
}

enum : int { kWalkMode = 0, kVerifyMode = 1, kFallbackMode = 2 };

// A segment: its connection ci, its packets [lo, hi) in sorted order, the connection's run
// [run_lo, run_hi), its index g (its end-state slot) and its predecessor's (pred). Segment j of a
// run covers [run_lo + j*seg, run_lo + (j+1)*seg), so a run of at most seg packets is one segment.
// The table is arithmetic (no per-batch segment table): index g < n_conns is connection g's segment
// 0; index n_conns + e stands for sorted position P = (e + 1) * seg, and takes segment m of the run
// holding P, m = the number of multiples of seg in (run_lo, P] — every window of seg positions holds
// exactly one multiple, so each later segment gets exactly one index (a run's last multiple may be
// spare: then there is no segment g).
struct SegGeo { uint32_t ci, lo, hi, run_lo, run_hi, g, pred; bool first, last; };

// the number of segments after the first in a run
__device__ __forceinline__ uint32_t later_segs(uint32_t run_lo, uint32_t run_hi, uint32_t seg) {
  return run_hi > run_lo ? (run_hi - run_lo - 1) / seg : 0u;
}

__device__ __forceinline__ bool seg_geo(uint32_t g, uint32_t n_conns, uint32_t seg, uint32_t max_pkts,
                                        const uint32_t* __restrict__ skeys, const uint32_t* __restrict__ seg_lo,
                                        const uint32_t* __restrict__ seg_hi, SegGeo& x) {
  if (g < n_conns) {
    x.ci = g;
    x.run_lo = seg_lo[g];
    x.run_hi = seg_hi[g];
    x.lo = x.run_lo;
    x.hi = seg == kNoSeg ? x.run_hi : (uint32_t)min((uint64_t)x.run_hi, (uint64_t)x.run_lo + seg);
    x.first = true;
    x.pred = 0;
  } else {
    if (seg == kNoSeg) return false;
    const uint64_t P = (uint64_t)(g - n_conns + 1) * seg;
    if (P >= max_pkts) return false;
    const uint32_t ci = skeys[P];  // the sorted connection keys (padding past the count: all ones)
    if (ci >= n_conns) return false;
    x.ci = ci;
    x.run_lo = seg_lo[ci];
    x.run_hi = seg_hi[ci];
    const uint32_t m = (uint32_t)(P / seg) - x.run_lo / seg;
    if (m == 0 || m > later_segs(x.run_lo, x.run_hi, seg)) return false;
    x.lo = x.run_lo + m * seg;
    x.hi = min(x.run_hi, x.lo + seg);
    x.first = false;
    x.pred = m == 1 ? ci : g - 1;
  }
  x.g = g;
  x.last = x.hi == x.run_hi;
  return true;
}
// the slot of segment j of connection ci's run
__device__ __forceinline__ uint32_t seg_slot(uint32_t j, uint32_t ci, uint32_t run_lo, uint32_t n_conns,
                                             uint32_t seg) {
  return j == 0 ? ci : n_conns + run_lo / seg + j - 1;
}

// One wave walks segment x. Walk: from the connection's state (first segment), the previous walk's
// end state of the predecessor (later segments, walks after the first) or the guessed start (later
// segments, first walk). Verify: from this walk's recorded end state of the predecessor; returns
// whether any decision or the end state differs. Fallback: the whole run from the connection's
// state, recording the exact end state of every segment for the next walk.
template <int MODE>
__device__ __forceinline__ bool recv_walk(const mq_conn_recv* __restrict__ conn0, mq_conn_recv* __restrict__ conns,
                                          uint32_t n_conns, const RecvWork* __restrict__ work,
                                          const uint32_t* __restrict__ svals, const RecvPlan* __restrict__ hdr,
                                          uint32_t n_rows, const RecvPlan* __restrict__ tried,
                                          RecvPlan* __restrict__ tried2,
                                          const uint8_t* __restrict__ outcome, mq_pkt_desc* __restrict__ d1,
                                          mq_pkt_desc* __restrict__ d2, mq_recv_pkt* __restrict__ out,
                                          uint32_t* __restrict__ attempts, int final_walk, uint2* __restrict__ hpm,
                                          SegState* __restrict__ segend, const SegState* __restrict__ segprev,
                                          uint32_t seg, uint32_t walk_idx, const SegGeo& x, WalkIn* sin,
                                          WalkOut* sout) {
  const uint32_t q = threadIdx.x % kWave;
  const uint32_t ci = x.ci, lo = x.lo, hi = x.hi;
  const mq_conn_recv c = conn0[ci];  // every lane: the state is kept wave-uniform
  ConnState s = load_state(c);
  if (MODE == kVerifyMode) {
    s = unpack_state(segend[x.pred]);  // the predecessor's recorded end state
  } else if (MODE == kWalkMode && !x.first && walk_idx > 0) {
    s = unpack_state(segprev[x.pred]);  // the previous walk's end state of the segment before
  } else if (MODE == kWalkMode && !x.first) {
    // the guessed start: the first packet's PN decoded against the batch-start largest PN plus
    // the packets before it in the run, minus one, as its level's largest PN
    const RecvWork w0 = work[lo];
    if (w0.pre == kPending) {
      const RecvPlan p0 = hdr[lo];
      const uint32_t l0 = w0.level;
      const uint64_t base = largest_of(s, l0) + (uint64_t)(lo - x.run_lo);
      const uint64_t est = decode_pn(p0.trunc, p0.pn_len, base);
      if (est > 0) raise_largest(s, l0, est - 1);
    }
  }
  // attempts = keyed d1 entries of the pass. A fallback re-walks a run whose segment walks already
  // counted their keyed entries in this walk: it takes those back and counts its own.
  uint32_t new_attempts = 0, prior = 0;
  if (MODE == kFallbackMode)
    for (uint32_t k0 = lo; k0 < hi; k0 += kWave)  // wave-uniform
      prior += (uint32_t)__popcll(__ballot(k0 + q < hi && d1[k0 + q].key_id != kNoRow));
  bool mismatch = false;
  // Settled prefix (walks after the first): while every packet so far OPENED with the keys the
  // speculation chose (outcome kOk1, no key update), the reference's decisions are exactly the
  // speculation's — same state, same inputs — so the previous walk's records stand; the walk only
  // clears the chunk's descriptors (nothing to attempt) and raises the largest PNs. The first chunk
  // that is not settled switches the connection to the full path for the rest of its run. The
  // verify and fallback passes decide every packet.
  bool settled = MODE == kWalkMode;
  for (uint32_t k0 = lo; k0 < hi; k0 += kWave) {  // wave-uniform
    const uint32_t m = min((uint32_t)kWave, hi - k0), k = k0 + q;
    const bool mine = q < m;
    // a segment boundary (seg is a multiple of kWave): the exact state, the next walk's start there
    if (MODE == kFallbackMode && seg != kNoSeg && k0 > lo && (k0 - lo) % seg == 0 && q == 0)
      segend[seg_slot((k0 - lo) / seg - 1, ci, x.run_lo, n_conns, seg)] = pack_state(s);
    if (settled) {
      uint8_t so = kOk1;
      RecvPlan st{};
      if (mine) {
        so = outcome[k];
        st = tried[k];
      }
      if (!wave_any(mine && (so != kOk1 || st.gen == 2))) {
        if (mine) {
          d1[k].key_id = kNoRow;
          d2[k].key_id = kNoRow;
        }
#pragma unroll
        for (uint32_t l = 0; l < 3; ++l) {
          uint64_t tot;
          (void)excl_max_u64(mine && st.status == l ? st.pn : 0ull, q, tot);
          if (tot > s.largest[l]) s.largest[l] = tot;
        }
        continue;
      }
      settled = false;
    }
    RecvWork w{};
    RecvPlan p{}, t{};
    uint8_t o = kNone;
    uint32_t i = 0;
    WalkIn in{};
    if (mine) {  // work, hdr, tried, outcome: sorted order
      i = svals[k];
      w = work[k];
      p = hdr[k];
      t = tried[k];
      o = outcome[k];
      in.tpn = t.pn; in.trow = t.row; in.tretry = t.retry; in.trunc = p.trunc;
      in.pn_len = p.pn_len; in.phase = p.phase; in.level = w.level; in.pre = w.pre;
      in.o = o; in.tgen = t.gen;
    }
    // parallel decision against the chunk-start state, then against each packet's true largest PN
    WalkOut r = walk_eval(s, c, n_rows, in, final_walk);
    bool ok = mine && r.st == MQ_OK;
    const bool rot = ok && w.level == MQ_LEVEL_APPLICATION && r.gen == 2;
    bool exact = false;
    if (!wave_any(rot)) {
      uint64_t tot[3], mx = 0;
#pragma unroll
      for (uint32_t l = 0; l < 3; ++l) {
        const uint64_t e = excl_max_u64(ok && w.level == l ? r.pn : 0ull, q, tot[l]);
        if (w.level == l) mx = e;
      }
      ConnState sx = s;
#pragma unroll
      for (uint32_t l = 0; l < 3; ++l)
        if (w.level == l && mx > sx.largest[l]) sx.largest[l] = mx;
      const WalkOut r2 = walk_eval(sx, c, n_rows, in, final_walk);
      exact = !wave_any(mine && (r2.pn != r.pn || r2.st != r.st));
      if (exact) {
        r = r2;
#pragma unroll
        for (uint32_t l = 0; l < 3; ++l)
          if (tot[l] > s.largest[l]) s.largest[l] = tot[l];
      }
    }
    if (!exact) {  // the sequential replay of the chunk by lane 0, from LDS
      if (mine) sin[q] = in;
      wave_sync();
      if (q == 0) {
        for (uint32_t x = 0; x < m; ++x) {
          const WalkIn e = sin[x];
          const WalkOut rx = walk_eval(s, c, n_rows, e, final_walk);
          sout[x] = rx;
          if (rx.st == MQ_OK) {
            RecvWork wx;
            wx.level = e.level;
            RecvPlan px;
            px.pn = rx.pn;
            advance(s, wx, px, rx.gen);
          }
        }
      }
      wave_sync();
      if (mine) r = sout[q];
      // lane 0's state to every lane
#pragma unroll
      for (uint32_t l = 0; l < 3; ++l) {
        s.largest[l] = (uint64_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(s.largest[l] >> 32)) << 32 |
                       (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)s.largest[l]);
        s.row[l] = (uint32_t)__builtin_amdgcn_readfirstlane((int)s.row[l]);
      }
      s.phase = (uint8_t)__builtin_amdgcn_readfirstlane((int)s.phase);
      s.flags = (uint8_t)__builtin_amdgcn_readfirstlane((int)s.flags);
      s.updates = (uint8_t)__builtin_amdgcn_readfirstlane((int)s.updates);
      wave_sync();  // the entries are read before the next round overwrites them
    }
    if (MODE == kVerifyMode) {
      // the walk's records of this packet: the output record, whether d1 holds an attempt or a
      // re-seal, and an attempt's inputs
      bool diff = false;
      if (mine) {
        const mq_recv_pkt rec = out[i];
        diff = rec.status != r.st || (r.st == MQ_OK && (rec.pn != r.pn ||
               rec.key_gen != ((w.level == MQ_LEVEL_APPLICATION) ? r.gen : 0))) ||
               ((d1[k].key_id != kNoRow) != (r.mode != 0));
        if (!diff && r.mode == 1) {
          const RecvPlan ta = tried2[k];  // the attempt this walk made
          diff = ta.pn != r.pn || ta.row != r.row || ta.retry != r.retry || ta.gen != r.pgen;
        }
      }
      mismatch = mismatch || wave_any(diff);
      continue;
    }
    bool att = false;
    if (mine) {
      mq_pkt_desc a;
      a.offset = w.offset; a.len = w.len; a.key_id = kNoRow; a.pn = r.lbefore; a.pn_offset = w.pn_off;
      a.pn_len = 0; a.flags = w.level != MQ_LEVEL_APPLICATION ? MQ_PKT_LONG_HEADER : 0; a.reserved = 0;
      mq_pkt_desc b = a;
      if (r.mode == 1) {
        RecvPlan tp;
        tp.pn = r.pn; tp.lbefore = r.lbefore; tp.row = r.row; tp.retry = r.retry; tp.trunc = p.trunc;
        // tried entries: status = the packet's level (the settled prefix's largest PNs). Written
        // as PENDING (tried2): the outcome kernel commits them to tried[] with their outcome, so a
        // fallback walk that drops this attempt (d1 unkeyed) leaves tried[] matching outcome[]
        tp.status = w.level; tp.gen = r.pgen; tp.phase = p.phase; tp.pn_len = p.pn_len;
        tried2[k] = tp;
        a.key_id = r.row;
        b.key_id = r.retry;
        // the open pre-pass value of both passes (prepass_decode: truncated PN, unmasked first
        // byte), from the front's unmask — so the passes run no header-protection pre-pass
        hpm[k] = make_uint2(p.trunc, 0x100u | (p.row & 0xffu));
      } else if (r.mode == 2) {
        a.key_id = o == kOk1 ? t.row : t.retry;
        a.pn = t.pn;
        a.pn_len = t.pn_len;
      }
      d1[k] = a;
      d2[k] = b;
      mq_recv_pkt rec;
      rec.offset = w.offset; rec.len = w.len; rec.dgram = w.dgram; rec.level = w.level; rec.status = r.st;
      rec.pn = r.st == MQ_OK ? r.pn : 0;
      rec.payload_offset = r.st == MQ_OK ? (uint16_t)(w.pn_off + p.pn_len) : 0;
      rec.key_gen = (w.level == MQ_LEVEL_APPLICATION && r.st == MQ_OK) ? r.gen : 0;
      rec.reserved[0] = rec.reserved[1] = rec.reserved[2] = 0;
      out[i] = rec;
      att = a.key_id != kNoRow;  // keyed d1 entry: an attempt, or a re-seal (final walk)
    }
    new_attempts += (uint32_t)__popcll(__ballot(att));
  }
  if (MODE == kVerifyMode) return mismatch || !same_state(s, unpack_state(segend[x.g]));
  if (q != 0) return false;
  if (new_attempts != prior) atomicAdd(attempts, new_attempts - prior);  // mod 2^32: the total stays >= 0
  if (MODE == kWalkMode) segend[x.g] = pack_state(s);
  if (MODE == kFallbackMode && seg != kNoSeg && hi > lo) segend[seg_slot((hi - lo - 1) / seg, ci, x.run_lo, n_conns, seg)] = pack_state(s);
  if (!x.last) return false;  // the connection's state: its last segment's (or the fallback's)
  mq_conn_recv u = c;
  for (int l = 0; l < 3; ++l) { u.largest_pn[l] = s.largest[l]; u.app_row[l] = s.row[l]; }
  u.key_phase = s.phase;
  u.flags = s.flags;
  u.key_updates = s.updates;
  conns[ci] = u;
  return false;
}

#define MQ_RECV_WALK_PARAMS                                                                                  \
  const mq_conn_recv *__restrict__ conn0, mq_conn_recv *__restrict__ conns, uint32_t n_conns,               \
      const RecvWork *__restrict__ work, const uint32_t *__restrict__ svals, const uint32_t *__restrict__ skeys, \
      const uint32_t *__restrict__ seg_lo, const uint32_t *__restrict__ seg_hi, const RecvPlan *__restrict__ hdr, \
      uint32_t n_rows, const RecvPlan *__restrict__ tried, RecvPlan *__restrict__ tried2,                   \
      const uint8_t *__restrict__ outcome, mq_pkt_desc *__restrict__ d1, mq_pkt_desc *__restrict__ d2,      \
      mq_recv_pkt *__restrict__ out, uint32_t *__restrict__ attempts, int final_walk, uint2 *__restrict__ hpm, \
      SegState *__restrict__ segend_all, uint32_t *__restrict__ vstate, uint32_t max_segs, uint32_t seg,    \
      uint32_t max_pkts, uint32_t walk_idx
#define MQ_RECV_WALK_ARGS(MODE, X)                                                                           \
  recv_walk<MODE>(conn0, conns, n_conns, work, svals, hdr, n_rows, tried, tried2, outcome, d1, d2, out, attempts, \
                  final_walk, hpm, segend, segprev, seg, walk_idx, X, s_in + wv * kWave, s_out + wv * kWave)
#define MQ_RECV_WALK_PROLOGUE                                                                                \
  __shared__ WalkIn s_in[kWalkThreads];                                                                      \
  __shared__ WalkOut s_out[kWalkThreads];                                                                    \
  const uint32_t wv = threadIdx.x / kWave, q = threadIdx.x % kWave;                                          \
  (void)q;                                                                                                   \
  /* this walk's end states, and the previous walk's (the starts of this walk's later segments) */         \
  SegState* segend = segend_all + (size_t)(walk_idx & 1) * max_segs;                                         \
  const SegState* segprev = segend_all + (size_t)((walk_idx & 1) ^ 1) * max_segs;

// the walk: one wave per segment (every connection's first segment, then the later ones)
extern "C" __global__ __launch_bounds__(kWalkThreads) void mq_recv_walk_kernel(MQ_RECV_WALK_PARAMS) {
  MQ_RECV_WALK_PROLOGUE
  SegGeo x;
  if (!seg_geo(blockIdx.x * kWalkConns + wv, n_conns, seg, max_pkts, skeys, seg_lo, seg_hi, x)) return;
  (void)vstate;
  (void)MQ_RECV_WALK_ARGS(kWalkMode, x);
}

// verify + fallback: one wave per later segment re-walks it from its predecessor's recorded end
// state. Connection c's checks meet in ONE 64-bit word, vstate[2c..2c+1] read as a uint64: each
// check adds 1 (low half: checks done) plus 2^32 when its segment disagreed (high half), so the
// check whose add completes the count reads every other check's verdict in the value its own add
// returns — one location, one modification order, no fence or ordering between two words needed
// (r05 kept verdict and count in two words and relied on s_waitcnt between them). That
// check resets the word and, when a segment disagreed, walks the whole run again from the
// connection's state (no further launch: a batch whose runs fit one segment each costs one
// early-exit launch per walk).
extern "C" __global__ __launch_bounds__(kWalkThreads) void mq_recv_verify_kernel(MQ_RECV_WALK_PARAMS) {
  MQ_RECV_WALK_PROLOGUE
  SegGeo x;
  if (!seg_geo(n_conns + blockIdx.x * kWalkConns + wv, n_conns, seg, max_pkts, skeys, seg_lo, seg_hi, x)) return;
  const bool differs = MQ_RECV_WALK_ARGS(kVerifyMode, x);
  uint32_t redo = 0;
  if (q == 0) {
    unsigned long long* word = (unsigned long long*)(vstate + 2 * (size_t)x.ci);
    const unsigned long long old = atomicAdd(word, 1ull + (differs ? (1ull << 32) : 0ull));
    if ((uint32_t)old + 1 == later_segs(x.run_lo, x.run_hi, seg)) {
      redo = (uint32_t)(old >> 32) + (differs ? 1u : 0u);
      *word = 0ull;  // the next walk's verify launch (stream-ordered) starts from zero
      if (redo) atomicAdd(&vstate[2 * n_conns], 1u);  // fallbacks run (MQ_RECV_TRACE)
    }
  }
  if (!__builtin_amdgcn_readfirstlane((int)redo)) return;
  SegGeo f;
  f.ci = x.ci; f.lo = f.run_lo = x.run_lo; f.hi = f.run_hi = x.run_hi; f.g = f.pred = x.ci;
  f.first = f.last = true;
  (void)MQ_RECV_WALK_ARGS(kFallbackMode, f);
}

// retry pass descriptors: only 1-RTT packets whose current keys failed (recv.rs:441-474); live[1]
// counts them (live[0]: the walk's keyed primary descriptors — none, none to retry either)
extern "C" __global__ __launch_bounds__(256) void mq_recv_retry_kernel(const uint8_t* __restrict__ st1,
                                                                       mq_pkt_desc* __restrict__ d2, uint32_t max_pkts,
                                                                       uint32_t* __restrict__ live) {
  if (live[0] == 0) return;
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  bool keep = false;
  if (i < max_pkts) {
    keep = d2[i].key_id != kNoRow && st1[i] == MQ_ERR_CRYPTO;
    if (!keep && d2[i].key_id != kNoRow) d2[i].key_id = kNoRow;
  }
  const uint32_t c = (uint32_t)__popcll(__ballot(keep));
  if (c && (threadIdx.x & (kWave - 1)) == 0) atomicAdd(live + 1, c);
}

// outcomes of this round's attempts
extern "C" __global__ __launch_bounds__(256) void mq_recv_outcome_kernel(const mq_pkt_desc* __restrict__ d1,
                                                                         const mq_pkt_desc* __restrict__ d2,
                                                                         const uint8_t* __restrict__ st1,
                                                                         const uint8_t* __restrict__ st2,
                                                                         uint8_t* __restrict__ outcome,
                                                                         RecvPlan* __restrict__ tried,
                                                                         const RecvPlan* __restrict__ tried2,
                                                                         uint32_t max_pkts,
                                                                         const uint32_t* __restrict__ live) {
  if (live[0] == 0) return;  // nothing attempted this round
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= max_pkts || d1[i].key_id == kNoRow) return;
  outcome[i] = st1[i] == MQ_OK ? kOk1 : (d2[i].key_id != kNoRow && st2[i] == MQ_OK) ? kOk0 : kFail;
  tried[i] = tried2[i];  // the attempt's inputs, with its outcome
}

// ---- stable sort of the records by connection (r04) ----------------------------------------------
// LSD radix sort, 8-bit digits, as many passes as the connection indices need (4096 connections and
// the padding key: 13 bits, two passes). Per pass: block digit histograms (count), their exclusive
// scan in digit-major order (hipcub), and a stable scatter — a block's 4096 items in four rounds of
// 1024 in index order; inside a round, a wave ranks its lanes among equal digits with eight ballots
// and the waves take their places by a per-digit prefix over the workgroup. r03/r04 used hipcub's
// SortPairs, which rocprim runs as a block sort plus 18 merge passes for 2^20 pairs at this key
// width: 158 us (profiles/r04w kernel trace); this is two passes of three kernels.
constexpr uint32_t kSortThreads = 1024, kSortItems = 4, kSortBlock = kSortThreads * kSortItems, kSortDigits = 256;
constexpr uint32_t kSortWaves = kSortThreads / kWave;

extern "C" __global__ __launch_bounds__(kSortThreads) void mq_sort_count_kernel(const uint32_t* __restrict__ keys,
                                                                                uint32_t n, uint32_t shift,
                                                                                uint32_t nblocks,
                                                                                uint32_t* __restrict__ hist) {
  __shared__ uint32_t s_h[kSortDigits];
  if (threadIdx.x < kSortDigits) s_h[threadIdx.x] = 0;
  __syncthreads();
#pragma unroll
  for (uint32_t k = 0; k < kSortItems; ++k) {
    const uint32_t i = blockIdx.x * kSortBlock + k * kSortThreads + threadIdx.x;
    if (i < n) atomicAdd(&s_h[(keys[i] >> shift) & (kSortDigits - 1)], 1u);
  }
  __syncthreads();
  if (threadIdx.x < kSortDigits) hist[(size_t)threadIdx.x * nblocks + blockIdx.x] = s_h[threadIdx.x];
}

// vals_in == nullptr: the values are the indices (the first pass)
extern "C" __global__ __launch_bounds__(kSortThreads) void mq_sort_scatter_kernel(
    const uint32_t* __restrict__ keys_in, const uint32_t* __restrict__ vals_in, uint32_t n, uint32_t shift,
    uint32_t nblocks, const uint32_t* __restrict__ hist, uint32_t* __restrict__ keys_out,
    uint32_t* __restrict__ vals_out) {
  __shared__ uint32_t s_run[kSortDigits];                // this block's next position per digit
  __shared__ uint32_t s_wc[kSortWaves][kSortDigits];     // a round's count per (wave, digit)
  const uint32_t lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
  const uint64_t below = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  if (threadIdx.x < kSortDigits) s_run[threadIdx.x] = hist[(size_t)threadIdx.x * nblocks + blockIdx.x];
  for (uint32_t k = 0; k < kSortItems; ++k) {
    for (uint32_t q = threadIdx.x; q < kSortWaves * kSortDigits; q += kSortThreads) (&s_wc[0][0])[q] = 0;
    __syncthreads();
    const uint32_t i = blockIdx.x * kSortBlock + k * kSortThreads + threadIdx.x;
    const bool in = i < n;
    const uint32_t key = in ? keys_in[i] : 0u, val = in ? (vals_in ? vals_in[i] : i) : 0u;
    const uint32_t d = (key >> shift) & (kSortDigits - 1);
    uint64_t peers = __ballot(in);
#pragma unroll
    for (int bit = 0; bit < 8; ++bit) {
      const uint64_t b = __ballot((d >> bit) & 1u);
      peers &= ((d >> bit) & 1u) ? b : ~b;
    }
    const uint32_t rank = (uint32_t)__popcll(peers & below);
    if (in && rank == 0) s_wc[w][d] = (uint32_t)__popcll(peers);  // the group's first lane
    __syncthreads();
    if (threadIdx.x < kSortDigits) {  // per digit: the waves' exclusive prefix, then the round total
      uint32_t run = s_run[threadIdx.x];
#pragma unroll
      for (uint32_t v = 0; v < kSortWaves; ++v) {
        const uint32_t c = s_wc[v][threadIdx.x];
        s_wc[v][threadIdx.x] = run;
        run += c;
      }
      s_run[threadIdx.x] = run;
    }
    __syncthreads();
    if (in) {
      const uint32_t pos = s_wc[w][d] + rank;
      keys_out[pos] = key;
      vals_out[pos] = val;
    }
    __syncthreads();  // s_wc is rewritten by the next round
  }
}

// ---- launch helpers ------------------------------------------------------------------------------
namespace {
size_t al(size_t b) { return (b + 255) & ~(size_t)255; }

struct RecvWs {
  uint32_t *counts, *base, *total, *keys, *vals, *skeys, *svals, *seg_lo, *seg_hi, *attempts;
  uint32_t *shist, *tkeys, *tvals;  // the sort's digit histograms and ping-pong buffers
  uint32_t* vstate;  // per connection: one 64-bit word (checks done | disagreeing checks << 32)
  SegState* segend;
  uint32_t max_segs;
  RecvWork *work, *work_s;
  RecvPlan *hdr_s, *tried, *tried2;
  mq_conn_recv* conn0;
  uint2* hpm;
  mq_pkt_desc *d1, *d2;
  uint8_t *st1, *st2, *outcome;
  void* cub;
  size_t cub_bytes;
  uint8_t* open_ws;
  size_t bytes;
};

uint32_t sort_blocks(uint32_t n) { return (n + kSortBlock - 1) / kSortBlock; }

size_t cub_bytes(uint32_t n_dgrams, uint32_t max_pkts) {
  size_t a = 0, b = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, a, (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)n_dgrams + 1);
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, b, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                         (int)(kSortDigits * sort_blocks(max_pkts)));
  return a > b ? a : b;
}

RecvWs layout(uint8_t* p, uint32_t n_dgrams, uint32_t max_pkts, uint32_t n_conns, size_t open_ws_bytes) {
  RecvWs w;
  size_t o = 0;
  auto take = [&](size_t bytes) { uint8_t* q = p ? p + o : nullptr; o += al(bytes); return q; };
  w.counts = (uint32_t*)take(4ull * n_dgrams + 4);
  w.base = (uint32_t*)take(4ull * n_dgrams + 4);
  w.total = (uint32_t*)take(8);
  w.attempts = (uint32_t*)take(8);
  w.keys = (uint32_t*)take(4ull * max_pkts);
  w.vals = (uint32_t*)take(4ull * max_pkts);
  w.skeys = (uint32_t*)take(4ull * max_pkts);
  w.svals = (uint32_t*)take(4ull * max_pkts);
  w.shist = (uint32_t*)take(4ull * kSortDigits * sort_blocks(max_pkts));
  w.tkeys = (uint32_t*)take(4ull * max_pkts);
  w.tvals = (uint32_t*)take(4ull * max_pkts);
  w.seg_lo = (uint32_t*)take(4ull * n_conns);
  w.seg_hi = (uint32_t*)take(4ull * n_conns);
  const size_t max_segs = (size_t)n_conns + ((size_t)max_pkts + 63) / 64;  // segments of >= 64 packets
  w.vstate = (uint32_t*)take(8ull * n_conns + 8);
  w.segend = (SegState*)take(2 * sizeof(SegState) * max_segs);  // this walk's and the previous walk's
  w.max_segs = (uint32_t)max_segs;
  w.conn0 = (mq_conn_recv*)take(sizeof(mq_conn_recv) * (size_t)n_conns);
  w.work = (RecvWork*)take(sizeof(RecvWork) * (size_t)max_pkts);
  w.work_s = (RecvWork*)take(sizeof(RecvWork) * (size_t)max_pkts);
  w.hdr_s = (RecvPlan*)take(sizeof(RecvPlan) * (size_t)max_pkts);
  w.tried = (RecvPlan*)take(sizeof(RecvPlan) * (size_t)max_pkts);
  w.tried2 = (RecvPlan*)take(sizeof(RecvPlan) * (size_t)max_pkts);
  w.hpm = (uint2*)take(8ull * max_pkts);
  w.d1 = (mq_pkt_desc*)take(sizeof(mq_pkt_desc) * (size_t)max_pkts);
  w.d2 = (mq_pkt_desc*)take(sizeof(mq_pkt_desc) * (size_t)max_pkts);
  w.st1 = take(max_pkts);
  w.st2 = take(max_pkts);
  w.outcome = take(max_pkts);
  w.cub_bytes = cub_bytes(n_dgrams, max_pkts);
  w.cub = take(w.cub_bytes);
  w.open_ws = take(open_ws_bytes);
  w.bytes = o;
  return w;
}
}  // namespace

size_t mq_recv_workspace(uint32_t n_dgrams, uint32_t max_pkts, uint32_t n_conns, size_t open_ws_bytes) {
  return layout(nullptr, n_dgrams, max_pkts, n_conns, open_ws_bytes).bytes;
}

hipError_t mq_launch_chacha_prepass(const KeyRow* kt, uint32_t n_rows, const uint8_t* arena, uint64_t arena_len,
                                    const mq_pkt_desc* desc, uint32_t n, uint2* hpm, hipStream_t s);
hipError_t mq_launch_aes_prepass(const KeyRow* kt, uint32_t n_rows, const uint8_t* arena, uint64_t arena_len,
                                 const mq_pkt_desc* desc, uint32_t n, uint2* hpm, hipStream_t s);

hipError_t mq_recv_walk(const KeyRow* kt, uint32_t n_rows, mq_conn_recv* conns, uint32_t n_conns,
                        uint32_t n_dgrams, uint32_t max_pkts, mq_recv_pkt* out, void* ws_ptr, size_t open_ws_bytes,
                        bool final_walk, bool verify, uint32_t walk_idx, uint32_t seg, hipStream_t s);

// split, header-protection masks, sort, first walk (mq_host.cpp then runs the AEAD passes)
hipError_t mq_recv_front(const KeyRow* kt, uint32_t n_rows, mq_conn_recv* conns, uint32_t n_conns, uint8_t* arena,
                         uint64_t arena_len, const mq_dgram* dg, uint32_t n_dgrams, uint32_t max_pkts,
                         uint32_t* n_pkts, mq_recv_pkt* out, void* ws_ptr, size_t open_ws_bytes, MQRecvPass* pass,
                         uint32_t seg, hipStream_t s) {
  RecvWs w = layout((uint8_t*)ws_ptr, n_dgrams, max_pkts, n_conns, open_ws_bytes);
  pass->d1 = w.d1; pass->d2 = w.d2; pass->st1 = w.st1; pass->st2 = w.st2; pass->open_ws = w.open_ws;
  pass->live1 = w.attempts; pass->live2 = w.attempts + 1;
  const dim3 b256(256);
  hipError_t e = hipSuccess;
  if (n_dgrams) {
    hipLaunchKernelGGL(mq_recv_split_kernel, dim3((n_dgrams + 255) / 256), b256, 0, s, arena, arena_len, dg, n_dgrams,
                       n_conns, w.counts, (const uint32_t*)nullptr, w.work, max_pkts);
    if ((e = hipMemsetAsync(w.counts + n_dgrams, 0, 4, s)) != hipSuccess) return e;  // total lands in base[n]
    size_t cb = w.cub_bytes;
    if ((e = hipcub::DeviceScan::ExclusiveSum(w.cub, cb, w.counts, w.base, (int)n_dgrams + 1, s)) != hipSuccess)
      return e;
    if ((e = hipMemcpyAsync(w.total, w.base + n_dgrams, 4, hipMemcpyDeviceToDevice, s)) != hipSuccess) return e;
    hipLaunchKernelGGL(mq_recv_split_kernel, dim3((n_dgrams + 255) / 256), b256, 0, s, arena, arena_len, dg, n_dgrams,
                       n_conns, w.counts, (const uint32_t*)w.base, w.work, max_pkts);
  } else if ((e = hipMemsetAsync(w.total, 0, 4, s)) != hipSuccess) {
    return e;
  }
  if ((e = hipMemcpyAsync(n_pkts, w.total, 4, hipMemcpyDeviceToDevice, s)) != hipSuccess) return e;
  if (n_conns && (e = hipMemcpyAsync(w.conn0, conns, sizeof(mq_conn_recv) * (size_t)n_conns,
                                     hipMemcpyDeviceToDevice, s)) != hipSuccess)
    return e;
  if (max_pkts == 0) return hipGetLastError();
  hipLaunchKernelGGL(mq_recv_prep_kernel, dim3((max_pkts + 255) / 256), b256, 0, s, w.conn0, w.total, w.work, max_pkts,
                     n_rows, w.keys, w.vals, w.d1);
  if ((e = mq_launch_chacha_prepass(kt, n_rows, arena, arena_len, w.d1, max_pkts, w.hpm, s)) != hipSuccess) return e;
  if ((e = mq_launch_aes_prepass(kt, n_rows, arena, arena_len, w.d1, max_pkts, w.hpm, s)) != hipSuccess) return e;
  // keys are connection indices (< n_conns) and 0xFFFFFFFF past the packet count: the low
  // ceil(log2(n_conns + 1)) bits order them (the padding's all-ones bits sort last), so the radix
  // sort makes that many passes' worth of digits instead of 32 bits' 
  int end_bit = 1;
  while (end_bit < 32 && (1ull << end_bit) <= (uint64_t)n_conns) ++end_bit;
  {  // stable LSD passes of 8-bit digits; the last one writes skeys / svals
    const uint32_t passes = ((uint32_t)end_bit + 7) / 8, nb = sort_blocks(max_pkts);
    const uint32_t* kin = w.keys;
    const uint32_t* vin = nullptr;  // first pass: the values are the indices
    for (uint32_t p = 0; p < passes; ++p) {
      uint32_t* kout = ((passes - 1 - p) % 2 == 0) ? w.skeys : w.tkeys;
      uint32_t* vout = ((passes - 1 - p) % 2 == 0) ? w.svals : w.tvals;
      hipLaunchKernelGGL(mq_sort_count_kernel, dim3(nb), dim3(kSortThreads), 0, s, kin, max_pkts, 8 * p, nb, w.shist);
      size_t sb = w.cub_bytes;
      if ((e = hipcub::DeviceScan::ExclusiveSum(w.cub, sb, w.shist, w.shist, (int)(kSortDigits * nb), s)) != hipSuccess)
        return e;
      hipLaunchKernelGGL(mq_sort_scatter_kernel, dim3(nb), dim3(kSortThreads), 0, s, kin, vin, max_pkts, 8 * p, nb,
                         (const uint32_t*)w.shist, kout, vout);
      kin = kout;
      vin = vout;
    }
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  if (n_conns) {
    if ((e = hipMemsetAsync(w.seg_lo, 0, 4ull * n_conns, s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(w.seg_hi, 0, 4ull * n_conns, s)) != hipSuccess) return e;
  }
  if ((e = hipMemsetAsync(w.vstate, 0, 8ull * n_conns + 8, s)) != hipSuccess) return e;
  hipLaunchKernelGGL(mq_recv_seg_kernel, dim3((max_pkts + 255) / 256), b256, 0, s, w.skeys, max_pkts, n_conns, w.seg_lo,
                     w.seg_hi);
  hipLaunchKernelGGL(mq_recv_gather_kernel, dim3((max_pkts + 255) / 256), b256, 0, s, w.total, max_pkts, w.svals, w.work,
                     arena, w.hpm, w.work_s, w.hdr_s, w.outcome);
  return mq_recv_walk(kt, n_rows, conns, n_conns, n_dgrams, max_pkts, out, ws_ptr, open_ws_bytes, false, false, 0, seg, s);
}

// one walk (after the first, the previous round's AEAD outcomes are folded in first)
hipError_t mq_recv_walk(const KeyRow* /*kt*/, uint32_t n_rows, mq_conn_recv* conns, uint32_t n_conns,
                        uint32_t n_dgrams, uint32_t max_pkts, mq_recv_pkt* out, void* ws_ptr, size_t open_ws_bytes,
                        bool final_walk, bool verify, uint32_t walk_idx, uint32_t seg, hipStream_t s) {
  RecvWs w = layout((uint8_t*)ws_ptr, n_dgrams, max_pkts, n_conns, open_ws_bytes);
  hipError_t e;
  if ((e = hipMemsetAsync(w.attempts, 0, 4, s)) != hipSuccess) return e;
  if (!n_conns) return hipGetLastError();
  const uint32_t later = seg == kNoSeg ? 0u : (max_pkts + seg - 1) / seg;  // bound on later segments
#define MQ_RECV_WALK_LAUNCH(KERNEL, GRID)                                                                     \
  hipLaunchKernelGGL(KERNEL, dim3(GRID), dim3(kWalkThreads), 0, s, (const mq_conn_recv*)w.conn0, conns, n_conns,  \
                     (const RecvWork*)w.work_s, (const uint32_t*)w.svals, (const uint32_t*)w.skeys,             \
                     (const uint32_t*)w.seg_lo, (const uint32_t*)w.seg_hi, (const RecvPlan*)w.hdr_s, n_rows,   \
                     (const RecvPlan*)w.tried, w.tried2, (const uint8_t*)w.outcome, w.d1, w.d2, out, w.attempts, \
                     (int)final_walk, (uint2*)w.open_ws, w.segend, w.vstate, w.max_segs, seg, max_pkts, walk_idx)
  MQ_RECV_WALK_LAUNCH(mq_recv_walk_kernel, (n_conns + later + kWalkConns - 1) / kWalkConns);
  // later segments (none when no run can exceed one segment): the walk's chained starts are
  // verified, and connections whose segments disagree are walked again sequentially
  if (verify && later > 1) MQ_RECV_WALK_LAUNCH(mq_recv_verify_kernel, (later + kWalkConns - 1) / kWalkConns);
#undef MQ_RECV_WALK_LAUNCH
  return hipGetLastError();
}

// between the primary and the retry AEAD pass / after both
hipError_t mq_recv_retry(uint32_t n_dgrams, uint32_t max_pkts, uint32_t n_conns, void* ws_ptr, size_t open_ws_bytes,
                         hipStream_t s) {
  RecvWs w = layout((uint8_t*)ws_ptr, n_dgrams, max_pkts, n_conns, open_ws_bytes);
  hipError_t e;
  if ((e = hipMemsetAsync(w.attempts + 1, 0, 4, s)) != hipSuccess) return e;
  if (max_pkts)
    hipLaunchKernelGGL(mq_recv_retry_kernel, dim3((max_pkts + 255) / 256), dim3(256), 0, s, w.st1, w.d2, max_pkts,
                       w.attempts);
  return hipGetLastError();
}

hipError_t mq_recv_outcomes(uint32_t n_dgrams, uint32_t max_pkts, uint32_t n_conns, void* ws_ptr,
                            size_t open_ws_bytes, hipStream_t s) {
  RecvWs w = layout((uint8_t*)ws_ptr, n_dgrams, max_pkts, n_conns, open_ws_bytes);
  if (max_pkts)
    hipLaunchKernelGGL(mq_recv_outcome_kernel, dim3((max_pkts + 255) / 256), dim3(256), 0, s, w.d1, w.d2, w.st1, w.st2,
                       w.outcome, w.tried, (const RecvPlan*)w.tried2, max_pkts, (const uint32_t*)w.attempts);
  return hipGetLastError();
}

// MQ_RECV_TRACE=1 (diagnostic): after each walk, the segment count, flagged connections and
// attempts, printed to stderr (synchronizes the stream)
void mq_recv_trace(const char* what, uint32_t n_dgrams, uint32_t max_pkts, uint32_t n_conns, void* ws_ptr,
                   size_t open_ws_bytes, uint32_t seg, hipStream_t s) {
  static const bool on = [] {
    const char* e = std::getenv("MQ_RECV_TRACE");
    return e && e[0] == '1';
  }();
  if (!on) return;
  RecvWs w = layout((uint8_t*)ws_ptr, n_dgrams, max_pkts, n_conns, open_ws_bytes);
  (void)hipStreamSynchronize(s);
  uint32_t nfb = 0, att[2] = {0, 0};
  (void)hipMemcpy(&nfb, w.vstate + 2ull * n_conns, 4, hipMemcpyDeviceToHost);
  (void)hipMemcpy(att, w.attempts, 8, hipMemcpyDeviceToHost);
  std::fprintf(stderr, "[recv %s] segment %u fallbacks so far %u attempts %u retries %u\n", what, seg, nfb,
               att[0], att[1]);
}
