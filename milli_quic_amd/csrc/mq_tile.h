// mq_tile.h — tile framework shared by the ChaCha20-Poly1305 and AES-128-GCM kernels:
// descriptor validation, HBM<->LDS gather/scatter of whole packets, packet-number decoding.
//
// One wave = one tile = kPktsPerTile (8) packets, lane = 8*p + j. The tile's packets are copied
// whole into a private kLdsBytes LDS region ("image"), processed there, and written back.
// Packet p's image is the run of 16-B arena chunks covering it, placed at LDS chunk slot_p
// (an octet prefix sum of the chunk counts). Staging moves one packet per LDS-DMA instruction
// group (SGPR base address, lane = chunk), write-back likewise with plain 16-B stores; only the
// partial first/last chunks of unaligned packets go byte-wise, in one 16-lane pass per tile.
// Tiles whose images exceed the LDS budget run the same policy code on HBM directly ("direct").
#pragma once
#include "mq_device.h"

namespace mq {

// per-wave scratch after the image: per packet a 32-B ChaCha pool record (mq_chacha.hip) and the
// 32-B one-time MAC key. No slack: reads past the last packet's image land in the scratch.
constexpr uint32_t kScratchBytes = 64 * kPktsPerTile;
constexpr uint32_t kDataBudget = kLdsBytes - kScratchBytes;  // bytes of packet images (9728: 8 x 1216)
constexpr uint64_t kMaxPn = (1ull << 62) - 1;         // varint::MAX_VARINT
constexpr uint32_t kListHole = 0xFFFFFFFFu;            // index-list entry without a packet (mq_partition.hip)

// Per-lane view of its octet's packet.
struct PktCtx {
  uint32_t i;        // descriptor index
  bool valid;        // lane maps to a descriptor
  bool act;          // still being processed (no error so far)
  int st;            // MQ_* status
  mq_pkt_desc d;
  uint64_t pn;       // full packet number (seal: from d; open: decoded)
  uint32_t tile;     // tile index (diagnostic stamps)
  bool pre_hp;       // open: header-protection mask precomputed by the pre-pass (wave-uniform)
  uint32_t hm0, hm1; // that mask: bytes 0..3, byte 4
  uint32_t* otk;     // this packet's 32-B LDS scratch (one-time MAC key / E_K(J0)), in both paths
};

// decode_pn, reference src/packet/number.rs:52-70 (RFC 9000 A.3)
__device__ __forceinline__ uint64_t decode_pn(uint32_t truncated, uint32_t pn_len, uint64_t largest) {
  uint64_t win = 1ull << (8 * pn_len), hwin = win >> 1, mask = win - 1;
  uint64_t expected = largest + 1;
  uint64_t cand = (expected & ~mask) | truncated;
  if (cand + hwin <= expected && cand + win <= (1ull << 62)) return cand + win;
  if (cand > expected + hwin && cand >= win) return cand - win;
  return cand;
}

__device__ __forceinline__ bool is_record(const mq_pkt_desc& d) { return (d.flags & 0x04) != 0; }

// TLS record seal (encrypt_into, tcp_tls/connection.rs:561-600; seal_record, record.rs:88-113):
// record header = ApplicationData, legacy version 0x0303, length = len - 5 (the AAD), and the
// inner content type after the plaintext. Written by one lane before any keystream or MAC touches
// the record.
template <class S>
__device__ __forceinline__ void write_record_header(const S& sp, typename S::off_t rec, const mq_pkt_desc& d) {
  const uint32_t outer = d.len - 5u;
  sp.st8(rec, 23);
  sp.st8(rec + 1, 3);
  sp.st8(rec + 2, 3);
  sp.st8(rec + 3, (uint8_t)(outer >> 8));
  sp.st8(rec + 4, (uint8_t)outer);
  sp.st8(rec + (d.len - 17u), (uint8_t)d.reserved);
}

// Descriptor checks in the order of the oracle (oracle/mq_oracle.c orc_run / orc_protect_packet /
// orc_unprotect_packet), which follows transmit.rs:593-597,721-725 and recv.rs:364-366,970-973.
// SINGLE: one-row key table, so the suite check reads row 0 (a scalar load that does not wait
// for the descriptor).
template <uint32_t SUITE, bool OPEN, bool SINGLE = false>
__device__ __forceinline__ int validate(const mq_pkt_desc& d, const KeyRow* kt, uint32_t n_rows,
                                        uint64_t arena_len) {
  if (d.key_id >= n_rows || d.offset + (uint64_t)d.len > arena_len) return MQ_ERR_INVALID_ARG;
  if ((SINGLE ? kt[0].suite : kt[d.key_id].suite) != SUITE) return MQ_ERR_SUITE;
  const bool no_hp = (d.flags & MQ_PKT_NO_HP) != 0;
  if (is_record(d)) {  // TLS record (record.rs): 5-byte header AAD, no PN, u16 length field
    if (!no_hp || d.pn_offset != 5 || d.pn_len != 0 || d.len > 5u + 0xFFFFu) return MQ_ERR_INVALID_ARG;
    if (!OPEN && d.len < 5u + 1u + 16u) return MQ_ERR_BUFFER_TOO_SMALL;  // seal_record :97-99
  }
  if (!OPEN) {
    if (!no_hp && (d.pn_len < 1 || d.pn_len > 4)) return MQ_ERR_INVALID_ARG;
    if ((uint64_t)d.len < (uint64_t)d.pn_offset + d.pn_len + 16) return MQ_ERR_BUFFER_TOO_SMALL;
    if (!no_hp && (uint64_t)d.pn_offset + 20 > d.len) return MQ_ERR_CRYPTO;
  } else {
    // recv.rs:356-360 / :962-965: the packet is copied into a 2048-B buffer first
    if (!no_hp && !(d.flags & MQ_PKT_NO_RECV_LIMIT) && d.len > MQ_RECV_MAX_PACKET) return MQ_ERR_BUFFER_TOO_SMALL;
    if (!no_hp && (uint64_t)d.pn_offset + 20 > d.len) return MQ_ERR_CRYPTO;
    if (no_hp && (uint64_t)d.len < (uint64_t)d.pn_offset + d.pn_len + 16) return MQ_ERR_CRYPTO;
  }
  return MQ_OK;
}

__device__ __forceinline__ uint4 load_chunk_guarded(const uint8_t* arena, uint64_t addr, uint64_t len) {
  if (addr + 16 <= len) return *(const uint4*)(arena + addr);
  uint32_t w[4] = {0, 0, 0, 0};
  for (int b = 0; b < 16; ++b)
    if (addr + b < len) w[b >> 2] |= (uint32_t)arena[addr + b] << (8 * (b & 3));
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// Per-lane copy of its octet's packet placement (octet-uniform values; the rest is derived so
// that only these stay live across the policy code).
struct Placement {
  uint32_t slot;     // first LDS chunk of the packet's image
  uint64_t off;      // arena byte offset of the packet
  uint32_t len;      // packet bytes (0: packet inactive)
  __device__ __forceinline__ uint64_t base() const { return off & ~15ull; }  // image start
  __device__ __forceinline__ uint32_t head() const { return (uint32_t)off & 15u; }
  __device__ __forceinline__ uint32_t nch() const { return len ? (head() + len + 15) >> 4 : 0u; }
};

__device__ __forceinline__ uint32_t lane_u32(uint32_t x, int l) {
  return (uint32_t)__builtin_amdgcn_readlane((int)x, l);
}
__device__ __forceinline__ uint64_t lane_u64(uint64_t x, int l) {
  return (uint64_t)lane_u32((uint32_t)(x >> 32), l) << 32 | lane_u32((uint32_t)x, l);
}

// HBM -> LDS staging with LDS-DMA (global_load_lds_dwordx4): per packet, one instruction per 64
// chunks (1 KiB) whose LDS destination is lane-linear from the packet's slot; the HBM source is
// the packet's (SGPR) base + 16 * lane, so every instruction is one contiguous 1-KiB read
// (tools/ubench/ubench3.hip: 5.5 TB/s). A chunk that would read past the arena end is loaded
// byte-wise instead. issue() returns immediately; complete() waits.
struct DmaStager {
  uint8_t* smem;
  const uint8_t* arena;
  uint64_t arena_len;
  int lane, j;
  Placement pl;

  __device__ __forceinline__ bool tail_fix() const {  // last chunk reaches past the arena end
    return pl.len && pl.base() + 16ull * pl.nch() > arena_len;
  }
  __device__ __forceinline__ void issue() {
#if MQ_PROF_SKIP & 8
    return;
#endif
    const uint32_t ndma = pl.nch() - (tail_fix() ? 1u : 0u);
#pragma unroll
    for (int q = 0; q < kPktsPerTile; ++q) {
      const uint32_t n = lane_u32(ndma, kLanesPerPkt * q);
      if (n == 0) continue;
      const uint8_t* src = arena + lane_u64(pl.base(), kLanesPerPkt * q);
      uint8_t* dst = smem + 16u * lane_u32(pl.slot, kLanesPerPkt * q);
      for (uint32_t k = 0; k < n; k += kWave)
        if (k + lane < n)
          __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + 16u * (k + lane)),
                                           (__attribute__((address_space(3))) void*)(dst + 16u * k), 16, 0, 0);
    }
  }
  __device__ __forceinline__ void complete() {
    wave_sync();  // workgroup-scope fence: s_waitcnt vmcnt(0) covers the LDS-DMA writes
    if (j == 0 && tail_fix())
      *(uint4*)(smem + 16u * (pl.slot + pl.nch() - 1)) =
          load_chunk_guarded(arena, pl.base() + 16ull * (pl.nch() - 1), arena_len);
    wave_sync();
  }
};

// Direct path: packets are accessed in HBM in place; nothing to stage.
struct NoStager {
  __device__ __forceinline__ void issue() {}
  __device__ __forceinline__ void complete() { wave_sync(); }
};

// LDS -> HBM for packets with write=1: whole chunks with 16-B stores, then the partial edge
// chunks of unaligned packets byte-wise (lane 2q: packet q's first chunk, lane 2q+1: its last),
// so bytes of neighbouring packets (other tiles) are never touched.
__device__ __forceinline__ void stage_out(const uint8_t* smem, uint8_t* arena, int lane, bool write,
                                          const Placement& pl) {
#if MQ_PROF_SKIP & 4
  return;
#endif
  const uint32_t nw = write ? pl.nch() : 0u, head = pl.head();
  const uint32_t tail = (head + pl.len) & 15;
#pragma unroll
  for (int q = 0; q < kPktsPerTile; ++q) {
    const int l = kLanesPerPkt * q;
    const uint32_t n = lane_u32(nw, l);
    if (n == 0) continue;
    uint8_t* dst = arena + lane_u64(pl.base(), l);
    const uint8_t* src = smem + 16u * lane_u32(pl.slot, l);
    const uint32_t c0 = lane_u32(head, l) ? 1u : 0u, c1 = n - (lane_u32(tail, l) ? 1u : 0u);
    for (uint32_t k = 0; k < n; k += kWave) {
      const uint32_t c = k + lane;
      if (c >= c0 && c < c1) *(uint4*)(dst + 16u * c) = *(const uint4*)(src + 16u * c);
    }
  }
  // edge pass
  const int q = (lane >> 1) & (kPktsPerTile - 1), e = lane & 1, l = kLanesPerPkt * q;
  const uint32_t n = (uint32_t)__shfl((int)nw, l, kWave);
  const uint32_t h = (uint32_t)__shfl((int)head, l, kWave), t = (uint32_t)__shfl((int)tail, l, kWave);
  uint32_t c = 0, lo = 0, hi = 0;
  if (e == 0 && h) { c = 0; lo = h; hi = (n == 1 && t) ? t : 16u; }
  if (e == 1 && t && (n > 1 || !h)) { c = n - 1; lo = 0; hi = t; }
  const bool edge = lane < 2 * kPktsPerTile && n && hi > lo;
  if (wave_any(edge)) {
    const uint32_t slot = (uint32_t)__shfl((int)pl.slot, l, kWave);
    const uint64_t base = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(pl.off >> 32), l, kWave) << 32 |
                           (uint32_t)__shfl((int)(uint32_t)pl.off, l, kWave)) & ~15ull;
    if (edge) {
      const uint4 v = *(const uint4*)(smem + 16u * (slot + c));
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
      uint8_t* dst = arena + base + 16ull * c;
#pragma unroll
      for (uint32_t b = 0; b < 16; ++b)
        if (b >= lo && b < hi) dst[b] = (uint8_t)(w[b >> 2] >> (8 * (b & 3)));
    }
  }
}

// Tile driver shared by every suite policy. `smem` is the wave's private kLdsBytes region.
// Policy provides kSuite and
//   template <class S, class G> static __device__ void seal(const S&, S::off_t pkt, PktCtx&, const KeyRow*, int j, G& stg);
//   template <class S, class G> static __device__ void open(const S&, S::off_t pkt, PktCtx&, const KeyRow*, int j, bool direct, G& stg);
// calling stg.issue() once (after their own global loads have been consumed) and stg.complete()
// before touching packet bytes. Both must execute every wave_sync() in wave-uniform control flow.
// Open pre-pass (RFC 9001 §5.4.2 sampling, recv.rs:363-370): one packet per lane; picks the packets
// whose mask the tile kernel will need. Packets failing these checks are skipped here and
// reported by the tile kernel's own validation.
__device__ __forceinline__ bool prepass_pick(uint32_t t, uint32_t suite, const KeyRow* __restrict__ kt,
                                             uint32_t n_rows, uint64_t arena_len,
                                             const mq_pkt_desc* __restrict__ desc, uint32_t n,
                                             const uint32_t* __restrict__ index,
                                             const uint32_t* __restrict__ n_dev, uint32_t& i,
                                             const KeyRow*& row, uint64_t& sample_at, mq_pkt_desc& d) {
  const uint32_t count = n_dev ? *n_dev : n;
  if (t >= count) return false;
  i = index ? index[t] : t;
  if (i == kListHole) return false;
  d = desc[i];
  if (d.key_id >= n_rows || d.offset + (uint64_t)d.len > arena_len || (d.flags & MQ_PKT_NO_HP) ||
      (uint64_t)d.pn_offset + 20 > d.len)
    return false;
  row = kt + d.key_id;
  if (row->suite != suite) return false;
  sample_at = d.offset + d.pn_offset + 4;
  return true;
}

// Pre-pass header read: the received first byte and the 20 bytes at pn_offset (PN bytes, then the
// sample) as 5 little-endian words, with one 16-B and one 4-B unaligned load — prepass_pick has
// checked that the packet, and so these bytes, lie inside the arena
__device__ __forceinline__ void prepass_header(const uint8_t* __restrict__ arena, const mq_pkt_desc& d, uint8_t& b0,
                                               uint32_t (&w)[5]) {
  const uint8_t* p = arena + d.offset + d.pn_offset;
  const uint4 a = ld16(p);
  w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w;
  w[4] = *(const u32_u*)(p + 16);
  b0 = arena[d.offset];
}

// Seal post-pass: XOR the 5-byte HP mask (m0 = bytes 0..3, m1 = byte 4) into the sealed packet's
// first byte (low 4 / 5 bits) and PN bytes. w0 = the 4 bytes at pn_offset as loaded by
// prepass_header: the PN bytes change with one unaligned dword store (bytes past pn_len keep
// their values; the tile kernel is done and no other lane owns them).
__device__ __forceinline__ void seal_apply_hp(uint8_t* __restrict__ arena, const mq_pkt_desc& d, uint8_t b0,
                                              uint32_t w0, uint32_t m0, uint32_t m1) {
  uint8_t* h = arena + d.offset;
  h[0] = b0 ^ ((uint8_t)m0 & ((d.flags & MQ_PKT_LONG_HEADER) ? 0x0f : 0x1f));
  const uint32_t mk = (m0 >> 8) | (m1 << 24);
  const uint32_t keep = d.pn_len >= 4 ? 0xffffffffu : (1u << (8 * d.pn_len)) - 1u;
  *(u32_u*)(h + d.pn_offset) = w0 ^ (mk & keep);
}

// Batch-open pre-pass output: instead of the raw mask, what the tile kernel derives from it —
// the unmasked first byte (| 0x100) and the unmasked truncated packet number (recv.rs:371-391) —
// so the tile kernel knows pn_len and the nonce before its packet has landed in LDS.
__device__ __forceinline__ uint2 prepass_decode(const uint8_t* __restrict__ arena, const mq_pkt_desc& d,
                                                uint32_t m0, uint32_t m1) {
  const uint8_t fb = (d.flags & MQ_PKT_LONG_HEADER) ? 0x0f : 0x1f;
  const uint8_t b0 = arena[d.offset] ^ ((uint8_t)m0 & fb);
  const uint32_t pn_len = (b0 & 3u) + 1, mk = (m0 >> 8) | (m1 << 24);
  uint32_t trunc = 0;
  for (uint32_t b = 0; b < pn_len; ++b)
    trunc = (trunc << 8) | (uint8_t)(arena[d.offset + d.pn_offset + b] ^ (uint8_t)(mk >> (8 * b)));
  return make_uint2(trunc, 0x100u | b0);
}

// prepass_decode from registers: b0 = the received first byte, pnw = the 4 received bytes at
// pn_offset (little-endian word), loaded together with the sample so that the pre-pass waits on
// memory once per packet
__device__ __forceinline__ uint2 prepass_decode_words(uint8_t b0raw, uint32_t pnw, const mq_pkt_desc& d,
                                                      uint32_t m0, uint32_t m1) {
  const uint8_t fb = (d.flags & MQ_PKT_LONG_HEADER) ? 0x0f : 0x1f;
  const uint8_t b0 = b0raw ^ ((uint8_t)m0 & fb);
  const uint32_t pn_len = (b0 & 3u) + 1, x = pnw ^ ((m0 >> 8) | (m1 << 24));
  uint32_t trunc = 0;
  for (uint32_t b = 0; b < pn_len; ++b) trunc = (trunc << 8) | ((x >> (8 * b)) & 0xffu);
  return make_uint2(trunc, 0x100u | b0);
}

// Open, header part (recv.rs:363-395 / :968-997) with the pre-pass values: pn_len, truncated PN,
// decode_pn and the PN range check. Returns the unmasked first byte.
__device__ __forceinline__ uint8_t header_from_prepass(PktCtx& c, uint32_t& pn_len, uint32_t& trunc) {
  const uint8_t b0 = (uint8_t)c.hm1;
  pn_len = (b0 & 3u) + 1;
  trunc = c.hm0;
  c.pn = decode_pn(trunc, pn_len, c.d.pn);
  if (c.pn > kMaxPn) {
    c.st = MQ_ERR_PROTOCOL;
    c.act = false;
  }
  return b0;
}

// Open, header part without the pre-pass: mask (from the policy), unmask byte 0 and the PN in
// the packet bytes, decode_pn, range check. Returns the unmasked first byte.
template <class S>
__device__ __forceinline__ uint8_t header_from_mask(const S& sp, typename S::off_t pkt, PktCtx& c, uint32_t m0,
                                                    uint32_t m1, uint32_t& pn_len, uint32_t& trunc) {
  const mq_pkt_desc& d = c.d;
  const uint8_t fb = (d.flags & MQ_PKT_LONG_HEADER) ? 0x0f : 0x1f;
  const uint8_t b0 = sp.ld8(pkt) ^ ((uint8_t)m0 & fb);
  pn_len = (b0 & 3u) + 1;
  const uint32_t mk = (m0 >> 8) | (m1 << 24);
  trunc = 0;
  for (uint32_t b = 0; b < pn_len; ++b)
    trunc = (trunc << 8) | (uint8_t)(sp.ld8(pkt + d.pn_offset + b) ^ (uint8_t)(mk >> (8 * b)));
  c.pn = decode_pn(trunc, pn_len, d.pn);
  if (c.pn > kMaxPn) {
    c.st = MQ_ERR_PROTOCOL;
    c.act = false;
  }
  return b0;
}

// Writes the unmasked header of an opened packet (octet lane 0), keeping the received bytes for
// the direct path's undo on failure.
template <class S>
__device__ __forceinline__ bool write_unmasked_header(const S& sp, typename S::off_t pkt, const PktCtx& c, int j,
                                                      uint8_t b0, uint32_t pn_len, uint32_t trunc,
                                                      uint8_t& orig_b0, uint32_t& orig_pn) {
  if (!c.act || j != 0) return false;
  orig_b0 = sp.ld8(pkt);
  orig_pn = 0;
  for (uint32_t b = 0; b < pn_len; ++b) orig_pn |= (uint32_t)sp.ld8(pkt + c.d.pn_offset + b) << (8 * b);
  sp.st8(pkt, b0);
  for (uint32_t b = 0; b < pn_len; ++b) sp.st8(pkt + c.d.pn_offset + b, (uint8_t)(trunc >> (8 * (pn_len - 1 - b))));
  return true;
}

// SINGLE_KEY: the key table has one row, so every valid packet uses row 0; the policies then get
// a wave-uniform row pointer and read key material with scalar loads into SGPRs.
// Descriptor words of a tile fetched ahead of time (for_tiles): lane 8p + j holds dword j of
// packet p's descriptor (dw) and, for open, dword j < 2 of its HP mask (hm), and idx = packet p's
// descriptor index (kListHole for a hole of an index list); octet swizzles rebuild the
// descriptor, so a prefetch costs three VGPRs. Tiles of 16 packets on 4 lanes each (the narrow AES
// kernels): lane 4p + j holds dwords 2j (dw) and 2j + 1 (dw1).
struct TilePrefetch {
  bool on;  // wave-uniform
  uint32_t dw, hm, idx, dw1, dw2, dw3;  // dw2, dw3: tiles of 32 packets on 2 lanes (dwords 4j .. 4j + 3)
};

template <int K>
__device__ __forceinline__ uint32_t oct_lane(uint32_t x) {  // lane K of the octet
  return (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, 0x18 | (K << 5));
}

// Per-lane packet context of tile `tile_id` (descriptor from the prefetch or from memory, HP
// pre-pass values, validation). Returns false when the tile lies past the batch (wave-uniform).
template <uint32_t SUITE, bool OPEN, bool SINGLE_KEY, int G = kLanesPerPkt>
__device__ __forceinline__ bool tile_ctx(uint32_t tile_id, const KeyRow* __restrict__ kt, uint32_t n_rows,
                                         uint64_t arena_len, const mq_pkt_desc* __restrict__ desc, uint32_t n,
                                         const uint32_t* __restrict__ index, const uint32_t* __restrict__ n_dev,
                                         const uint2* __restrict__ hpm, const TilePrefetch& pf, PktCtx& c,
                                         const KeyRow*& row, uint32_t tid = threadIdx.x, uint32_t e0 = 0) {
  static_assert(G == 8 || G == 4 || G == 2, "tiles of 8, 16 or 32 packets");
  const int lane = tid & (kWave - 1), p = lane / G;
  const uint32_t count = n_dev ? *n_dev : n;
  const uint32_t tile0 = e0 + tile_id * (uint32_t)(kWave / G);  // its first entry
  if (tile0 >= count) return false;  // wave-uniform
  c.tile = tile_id;
  const uint32_t t = tile0 + p;
  c.valid = t < count;
  c.pre_hp = OPEN && hpm != nullptr;
  c.hm0 = c.hm1 = 0;
  if (pf.on) {  // words already in registers
    c.i = c.valid ? pf.idx : 0u;
    if (c.i == kListHole) { c.valid = false; c.i = 0; }
    uint32_t w0, w1, w2, w3, w4, w5, w6, w7;
    if (G == 8) {
      w0 = oct_lane<0>(pf.dw); w1 = oct_lane<1>(pf.dw); w2 = oct_lane<2>(pf.dw); w3 = oct_lane<3>(pf.dw);
      w4 = oct_lane<4>(pf.dw); w5 = oct_lane<5>(pf.dw); w6 = oct_lane<6>(pf.dw); w7 = oct_lane<7>(pf.dw);
    } else if (G == 4) {
      w0 = Grp<4>::lane<0>(pf.dw); w1 = Grp<4>::lane<0>(pf.dw1); w2 = Grp<4>::lane<1>(pf.dw);
      w3 = Grp<4>::lane<1>(pf.dw1); w4 = Grp<4>::lane<2>(pf.dw); w5 = Grp<4>::lane<2>(pf.dw1);
      w6 = Grp<4>::lane<3>(pf.dw); w7 = Grp<4>::lane<3>(pf.dw1);
    } else {
      w0 = Grp<2>::lane<0>(pf.dw); w1 = Grp<2>::lane<0>(pf.dw1); w2 = Grp<2>::lane<0>(pf.dw2);
      w3 = Grp<2>::lane<0>(pf.dw3); w4 = Grp<2>::lane<1>(pf.dw); w5 = Grp<2>::lane<1>(pf.dw1);
      w6 = Grp<2>::lane<1>(pf.dw2); w7 = Grp<2>::lane<1>(pf.dw3);
    }
    c.d.offset = (uint64_t)w1 << 32 | w0;
    c.d.len = w2; c.d.key_id = w3;
    c.d.pn = (uint64_t)w5 << 32 | w4;
    c.d.pn_offset = (uint16_t)w6; c.d.pn_len = (uint8_t)(w6 >> 16); c.d.flags = (uint8_t)(w6 >> 24);
    c.d.reserved = w7;
    if (OPEN && hpm) {
      c.hm0 = G == 8 ? oct_lane<0>(pf.hm) : Grp<G>::template lane<0>(pf.hm);
      c.hm1 = G == 8 ? oct_lane<1>(pf.hm) : Grp<G>::template lane<1 % G>(pf.hm);
    }
    if (!c.valid) {
      c.d.offset = 0; c.d.len = 0; c.d.key_id = 0; c.d.pn = 0; c.d.pn_offset = 0; c.d.pn_len = 0;
      c.d.flags = 0; c.d.reserved = 0;
      c.hm0 = c.hm1 = 0;
    }
  } else {
    c.i = c.valid ? (index ? index[t] : t) : 0u;
    if (c.i == kListHole) { c.valid = false; c.i = 0; }
    if (c.valid) {
      c.d = desc[c.i];
    } else {
      c.d.offset = 0; c.d.len = 0; c.d.key_id = 0; c.d.pn = 0; c.d.pn_offset = 0; c.d.pn_len = 0;
      c.d.flags = 0; c.d.reserved = 0;
    }
    if (OPEN && hpm && c.valid) {
      const uint2 m = hpm[c.i];
      c.hm0 = m.x;
      c.hm1 = m.y;
    }
  }
  c.st = c.valid ? validate<SUITE, OPEN, SINGLE_KEY>(c.d, kt, n_rows, arena_len) : (int)MQ_ERR_INVALID_ARG;
  c.act = c.valid && c.st == MQ_OK;
  c.pn = c.d.pn;
  row = SINGLE_KEY ? kt : kt + (c.act ? c.d.key_id : 0u);
  return true;
}

// Status (and, for open, the decoded PN) of the tile's packets: octet lane 0.
template <bool OPEN>
__device__ __forceinline__ void tile_status(const PktCtx& c, int j, uint8_t* __restrict__ status,
                                            uint64_t* __restrict__ pn_out) {
  if (c.valid && j == 0) {
    status[c.i] = (uint8_t)c.st;
    if (OPEN && pn_out && c.st == MQ_OK) pn_out[c.i] = c.pn;
  }
}

template <class Policy, bool OPEN, bool SINGLE_KEY = false>
__device__ __forceinline__ void run_tile(uint8_t* smem, uint32_t tile_id, const KeyRow* __restrict__ kt,
                                         uint32_t n_rows, uint8_t* __restrict__ arena, uint64_t arena_len,
                                         const mq_pkt_desc* __restrict__ desc, uint32_t n,
                                         const uint32_t* __restrict__ index,
                                         const uint32_t* __restrict__ n_dev,
                                         uint8_t* __restrict__ status, uint64_t* __restrict__ pn_out,
                                         const uint2* __restrict__ hpm,
                                         TilePrefetch pf = TilePrefetch{false, 0u, 0u}) {
  const int lane = threadIdx.x & (kWave - 1), p = lane / kLanesPerPkt, j = lane % kLanesPerPkt;
  PktCtx c;
  const KeyRow* row;
  if (!tile_ctx<Policy::kSuite, OPEN, SINGLE_KEY>(tile_id, kt, n_rows, arena_len, desc, n, index, n_dev, hpm, pf,
                                                  c, row))
    return;
  MQ_STAMP(tile_id, 0);
  c.otk = (uint32_t*)(smem + kLdsBytes - kScratchBytes + 32u * (uint32_t)p);
  const uint64_t off = c.act ? c.d.offset : 0;
  // chunks of the packet image, clamped so sums cannot overflow; a clamped (huge) packet always
  // exceeds the budget and sends the tile down the direct path
  Placement pl;
  pl.off = off;
  pl.len = c.act ? c.d.len : 0u;
  const uint64_t nch64 = c.act ? ((off & 15) + (uint64_t)c.d.len + 15) >> 4 : 0u;
  const uint32_t nch = (uint32_t)(nch64 < 0xFFFFu ? nch64 : 0xFFFFu);
  const uint32_t incl = oct_incl_scan(nch);
  const uint32_t total = lane_u32(incl, kWave - 1);
#if MQ_PROF_SKIP & 32
  if ((void)total, false) {  // diagnostic: every tile on the direct path
#else
  if (total * 16u <= kDataBudget) {
#endif
    pl.slot = incl - nch;
    DmaStager stg{smem, arena, arena_len, lane, j, pl};
    LdsSpace sp{smem};
    MQ_STAMP(tile_id, 1);
    const uint32_t pkt = pl.slot * 16u + pl.head();
    if (OPEN) Policy::template open<LdsSpace>(sp, pkt, c, row, j, false, stg);
    else Policy::template seal<LdsSpace>(sp, pkt, c, row, j, stg);
    MQ_STAMP(tile_id, 6);
    wave_sync();
    stage_out(smem, arena, lane, c.act, pl);
    MQ_STAMP(tile_id, 7);
  } else {
    GlobalSpace sp{arena, arena_len};
    NoStager stg;
    if (OPEN) Policy::template open<GlobalSpace>(sp, off, c, row, j, true, stg);
    else Policy::template seal<GlobalSpace>(sp, off, c, row, j, stg);
  }
  tile_status<OPEN>(c, j, status, pn_out);
}

// Work distribution of the persistent tile kernels (r04). Wave g of a grid of
// `waves` waves runs tile base + g first. After that:
//   static  (ctr null): tiles base + g + waves, base + g + 2 waves, ...;
//   dynamic (ctr = the launch's schedule slot, mq_runtime.h SchedSlots): the remaining tiles are
//     cut into blocks of kSchedBlock; block k belongs to head k mod kSchedHeads (one head per XCD:
//     ≈88 claims/µs saturate one word, MI355X_MICROARCH.md 'dequeue'), so every head's tiles sample
//     the whole range — a length-sorted list (config E: longest class first) gives every XCD the
//     same mix, and all heads advance through the arena together. A wave claims entries of its
//     XCD's head with a returning device-scope atomicAdd — chunks of remaining / (2 x the waves per
//     head), 1..kMaxChunk entries (guided self-scheduling) — then, once that head is empty, single
//     entries of the other heads. The next chunk is claimed when the current one starts, so a
//     claim's latency hides behind at least one tile.
// Why: the static stride gives every workgroup a fixed share, so a workgroup that is placed late —
// its CU held by another kernel, e.g. the resident per-packet server (mq_resident.hip) or the
// hot-key kernel forked beside this one — ends the launch a whole share late. Dynamically, the
// others take what it has not started (tests/test_gpu_resident.py: config C 1.01x beside the
// server). Measured first with each head owning a contiguous eighth and chunks up to 16: config C
// +8 %, E +5 % over the static stride; chunks up to 4: C -5 %, E +6 % (profiles/r04g_ab_sched.txt).
// Slot layout (uint32 words): head h at word kSchedHeadWords * h, the finished-workgroup count at
// word kSchedDoneWord. The last workgroup to finish zeroes the slot (sched_done) for the next
// kernel on the same stream.
// (kSchedHeads, kSchedHeadWords, kSchedDoneWord, kSchedSlotBytes: mq_device.h, shared with the host)
#ifndef MQ_SCHED_MAX_CHUNK
#define MQ_SCHED_MAX_CHUNK 4
#endif
#ifndef MQ_SCHED_BLOCK
#define MQ_SCHED_BLOCK 16
#endif
constexpr uint32_t kMaxChunk = MQ_SCHED_MAX_CHUNK;
constexpr uint32_t kSchedBlock = MQ_SCHED_BLOCK;

struct TileSched {
  uint32_t* ctr;   // null: static
  uint32_t g;      // this wave's index in the grid (blockIdx.x * W + wave)
  uint32_t waves;  // waves in the grid
  uint32_t xcd;    // this workgroup's head (blockIdx.x % kSchedHeads: workgroups go to the XCDs round robin)
};

__device__ __forceinline__ uint32_t sched_claim(uint32_t* head, uint32_t c) {
  uint32_t h = 0;
  if ((threadIdx.x & (kWave - 1)) == 0) h = __hip_atomic_fetch_add(head, c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return (uint32_t)__builtin_amdgcn_readlane((int)h, 0);
}

// End of a workgroup's part in a dynamically scheduled launch (every workgroup of the grid exactly
// once, workgroup-uniform, after all its waves are done with the schedule — the callers put it
// after a barrier or, for a workgroup without work, at its only exit). The last one zeroes the
// slot: every claim of every wave has returned by then (its value was used), so no claim is lost.
__device__ __forceinline__ void sched_done(uint32_t* ctr) {
  if (!ctr || threadIdx.x != 0) return;
  const uint32_t old = __hip_atomic_fetch_add(ctr + kSchedDoneWord, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (old + 1 == gridDim.x) {
#pragma unroll
    for (uint32_t h = 0; h < kSchedHeads; ++h)
      __hip_atomic_store(ctr + kSchedHeadWords * h, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(ctr + kSchedDoneWord, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Persistent tile loop: this wave runs its tiles (TileSched) calling body(tile, prefetch), each
// tile's descriptor words (and HP masks) loaded while the previous tile is processed, so a tile
// starts without waiting on a descriptor fetch; with an index list the list entries are read one
// tile further ahead still (list entry, then descriptor: two dependent loads off the critical
// path). Tiles below `base` are not this launch's. With a device-side count (n_dev) the tiles end
// at that count. Tile t holds entries e0 + PPT t .. e0 + PPT t + PPT - 1 (e0: the key-segmented
// kernels' segment start, which need not be a multiple of PPT).
template <bool OPEN, int G = kLanesPerPkt, class F>
__device__ __forceinline__ void for_tiles(const TileSched& ts, const mq_pkt_desc* __restrict__ desc, uint32_t n,
                                          const uint32_t* __restrict__ index, const uint32_t* __restrict__ n_dev,
                                          const uint2* __restrict__ hpm, F&& body, uint32_t base = 0, uint32_t e0 = 0) {
  constexpr uint32_t PPT = kWave / G;  // packets per tile
  const uint32_t count = n_dev ? *n_dev : n;
  const uint32_t tiles = count > e0 ? (count - e0 + PPT - 1) / PPT : 0u;
  const uint32_t lane = threadIdx.x & (kWave - 1), p = lane / G, j = lane % G;
  constexpr uint32_t kNone = 0xFFFFFFFFu;
  // dynamic schedule (wave-uniform state): the tiles from dyn0 on, in blocks dealt to the heads
  const uint32_t dyn0 = base + ts.waves;
  const uint32_t D = tiles > dyn0 ? tiles - dyn0 : 0u;
  const uint32_t nb = (D + kSchedBlock - 1) / kSchedBlock;  // blocks; the last may be partial
  auto head_size = [&](uint32_t h) -> uint32_t {  // entries (tiles) of head h
    const uint32_t cnt = nb > h ? (nb - 1 - h) / kSchedHeads + 1 : 0u;
    const uint32_t part = ((nb - 1) % kSchedHeads == h && D % kSchedBlock) ? kSchedBlock - D % kSchedBlock : 0u;
    return cnt * kSchedBlock - (cnt ? part : 0u);
  };
  auto tile_of = [&](uint32_t h, uint32_t e) -> uint32_t {  // entry e of head h
    return dyn0 + ((e / kSchedBlock) * kSchedHeads + h) * kSchedBlock + e % kSchedBlock;
  };
  const uint32_t per_head = ts.waves / kSchedHeads > 1u ? ts.waves / kSchedHeads : 1u;
  uint32_t state = 0;       // 0: own head, 1: the other heads, 2: none left
  uint32_t seen = 0;        // own head: entries claimed as of this wave's last claim
  uint32_t ch = 0, ce = 0, cend = 0;  // the chunk being walked: head, entry, end entry
  // the claim of the next chunk, issued when the current one starts and resolved when it ends: the
  // atomic's result stays in a VGPR meanwhile (lane 0), so no wave waits on it (or on the stores
  // before it: vmcnt counts both) in steady state
  uint32_t qh = 0, qc = 0;
  bool pending = false;
  const uint32_t own_size = head_size(ts.xcd);
  auto issue = [&]() {
    if (state != 0) return;  // the other heads are claimed at resolve time
    const uint32_t rem = own_size > seen ? own_size - seen : 0u;
    uint32_t c = rem / (2 * per_head);
    qc = c < 1u ? 1u : (c > kMaxChunk ? kMaxChunk : c);
    qh = 0;
    if (lane == 0 && own_size)
      qh = __hip_atomic_fetch_add(ts.ctr + kSchedHeadWords * ts.xcd, qc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    pending = true;
  };
  // the next chunk: the pending own-head claim, else a single entry of another head
  auto resolve = [&]() -> bool {
    if (state == 0) {
      const uint32_t got = own_size ? (uint32_t)__builtin_amdgcn_readlane((int)qh, 0) : 0u;
      const bool ok = pending && got < own_size;
      pending = false;
      if (ok) {
        ch = ts.xcd;
        ce = got;
        cend = got + qc < own_size ? got + qc : own_size;
        seen = got + qc;
        return true;
      }
      state = 1;
    }
    // the other heads, single entries: one round trip reads all heads (a returning add of 0 on
    // lanes 0..7: atomics are coherent across the XCDs' L2s, plain loads are not), then a claim from
    // the first one after this XCD's with entries left; a lost race rescans (someone progressed)
#pragma nounroll
    for (uint32_t tries = 0; state == 1 && tries < 64; ++tries) {
      uint32_t v = 0xFFFFFFFFu, sz = 0;
      if (lane < kSchedHeads) {
        v = __hip_atomic_fetch_add(ts.ctr + kSchedHeadWords * lane, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        sz = head_size(lane);
      }
      const uint32_t open = (uint32_t)__ballot(lane < kSchedHeads && v < sz) & 0xFFu;
      if (!open) break;
      const uint32_t x = (ts.xcd + 1) % kSchedHeads;
      const uint32_t rot = ((open >> x) | (open << (kSchedHeads - x))) & 0xFFu;
      const uint32_t h = (x + (uint32_t)__builtin_ctz(rot)) % kSchedHeads;
      const uint32_t got = sched_claim(ts.ctr + kSchedHeadWords * h, 1u);
      if (got < head_size(h)) {
        ch = h;
        ce = got;
        cend = got + 1;
        return true;
      }
    }
    state = 2;
    return false;
  };
  auto next = [&](uint32_t t) -> uint32_t {
    if (t >= tiles) return kNone;
    if (!ts.ctr) return t + ts.waves;
    if (ce + 1 < cend) return tile_of(ch, ++ce);
    if (!resolve()) return kNone;
    issue();  // the chunk after this one
    return tile_of(ch, ce);
  };
  auto idx_of = [&](uint32_t t) -> uint32_t {  // packet p's descriptor index (list: a load)
    const uint32_t e = e0 + t * PPT + p;
    if (t >= tiles || e >= count) return kListHole;
    return index ? index[e] : e;
  };
  auto fetch = [&](uint32_t ix, uint32_t& dw, uint32_t& dw1, uint32_t& dw2, uint32_t& dw3, uint32_t& hm) {
    const bool ok = ix != kListHole;
    dw1 = dw2 = dw3 = 0;
    if (G == 8) {
      dw = ok ? reinterpret_cast<const uint32_t*>(desc)[(size_t)ix * 8 + j] : 0u;
    } else if (G == 4) {
      const uint2 v = ok ? reinterpret_cast<const uint2*>(desc)[(size_t)ix * 4 + j] : make_uint2(0, 0);
      dw = v.x;
      dw1 = v.y;
    } else {
      const uint4 v = ok ? reinterpret_cast<const uint4*>(desc)[(size_t)ix * 2 + j] : make_uint4(0, 0, 0, 0);
      dw = v.x;
      dw1 = v.y;
      dw2 = v.z;
      dw3 = v.w;
    }
    hm = (OPEN && hpm && ok && j < 2) ? reinterpret_cast<const uint32_t*>(hpm)[(size_t)ix * 2 + j] : 0u;
  };
  uint32_t t = base + ts.g;
  if (ts.ctr && t < tiles) issue();  // resolved right away by next(t): one wait per wave, at its start
  uint32_t t1 = next(t);
  uint32_t ix0 = idx_of(t), ix1 = idx_of(t1), dw, dw1, dw2, dw3, hm;
  fetch(ix0, dw, dw1, dw2, dw3, hm);
  while (t < tiles) {
    const TilePrefetch pf{true, dw, hm, ix0, dw1, dw2, dw3};
    const uint32_t t2 = next(t1);
    const uint32_t ix2 = idx_of(t2);
    fetch(ix1, dw, dw1, dw2, dw3, hm);
    body(t, pf);
    t = t1; t1 = t2; ix0 = ix1; ix1 = ix2;
  }
}

}  // namespace mq
