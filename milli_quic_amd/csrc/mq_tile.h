// mq_tile.h — tile framework shared by the ChaCha20-Poly1305 and AES-128-GCM kernels:
// descriptor validation, HBM<->LDS gather/scatter of whole packets, packet-number decoding.
//
// One wave = one tile = kPktsPerTile (8) packets, lane = 8*p + j. The tile's packets are copied
// whole into a private kLdsBytes LDS region ("image"), processed there, and written back. Two
// image layouts (wave-uniform choice):
//   fixed    every packet gets S = max(chunks) 16-B chunks: chunk g belongs to packet g / S
//            (a multiply-shift, no lookups) — the common case (1-RTT packets up to ~1.2 KB);
//   variable packets packed back to back; chunk g -> packet by a 3-step search of the slot
//            table (mixed batches whose largest packet does not fit the fixed layout).
// Tiles that fit neither run the same policy code on HBM directly ("direct" path).
#pragma once
#include "mq_device.h"

namespace mq {

constexpr uint32_t kSlotBytes = 32;
constexpr uint32_t kTableOff = kLdsBytes - kPktsPerTile * kSlotBytes;  // 9984
constexpr uint32_t kDataBudget = kTableOff - kSlack;                   // 9920 bytes of packets
constexpr uint64_t kMaxPn = (1ull << 62) - 1;                           // varint::MAX_VARINT

struct SlotEnt {  // one per packet of the tile, in LDS
  uint32_t slot;      // first 16-B chunk of the packet's image
  uint32_t nch;       // chunks the packet occupies
  uint32_t delta_lo;  // (arena chunk index of the packet's first chunk) - slot
  uint32_t delta_hi;
  uint32_t off_lo;    // arena byte offset of the packet
  uint32_t off_hi;
  uint32_t len;       // packet bytes
  uint32_t write;     // 1: store the packet back (status OK)
};

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

// Descriptor checks in the order of the oracle (oracle/mq_oracle.c orc_run / orc_protect_packet /
// orc_unprotect_packet), which follows transmit.rs:593-597,721-725 and recv.rs:364-366,970-973.
template <uint32_t SUITE, bool OPEN>
__device__ __forceinline__ int validate(const mq_pkt_desc& d, const KeyRow* kt, uint32_t n_rows,
                                        uint64_t arena_len) {
  if (d.key_id >= n_rows || d.offset + (uint64_t)d.len > arena_len) return MQ_ERR_INVALID_ARG;
  if (kt[d.key_id].suite != SUITE) return MQ_ERR_SUITE;
  const bool no_hp = (d.flags & MQ_PKT_NO_HP) != 0;
  if (!OPEN) {
    if (!no_hp && (d.pn_len < 1 || d.pn_len > 4)) return MQ_ERR_INVALID_ARG;
    if ((uint64_t)d.len < (uint64_t)d.pn_offset + d.pn_len + 16) return MQ_ERR_BUFFER_TOO_SMALL;
    if (!no_hp && (uint64_t)d.pn_offset + 20 > d.len) return MQ_ERR_CRYPTO;
  } else {
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

// chunk g of the image -> packet index p (wave-uniform layout choice)
struct Layout {
  const SlotEnt* tab;
  uint32_t S;      // fixed layout: chunks per packet slot (0 = variable layout)
  uint32_t magic;  // ceil(2^20 / S): g / S == (g * magic) >> 20 for g < 1024
  __device__ __forceinline__ int pkt_of(uint32_t g) const {
    if (S) return (int)((g * magic) >> 20);
    int j = 0;  // largest j with slot[j] <= g (slots are non-decreasing)
#pragma unroll
    for (int step = kPktsPerTile / 2; step >= 1; step >>= 1)
      if (tab[j + step].slot <= g) j += step;
    return j;
  }
};

// HBM -> LDS staging with LDS-DMA (global_load_lds_dwordx4): the image's `total` 16-B chunks
// land at LDS byte 16*g; one wave instruction moves 64 consecutive chunks (1 KiB) whose LDS
// destination is lane-linear, while each lane supplies its own HBM source address, so whole
// packets are gathered with contiguous HBM reads (tools/ubench/ubench3.hip: 5.5 TB/s vs 2.7 TB/s
// for one-packet-per-lane strides). issue() returns immediately; complete() waits.
struct DmaStager {
  uint8_t* smem;
  Layout lay;
  uint32_t total;
  const uint8_t* arena;
  uint64_t arena_len;
  int lane;
  uint64_t fix_addr = ~0ull;  // owned chunk that straddles the arena end (loaded byte-wise)
  uint32_t fix_g = 0;

  __device__ __forceinline__ void issue() {
#if MQ_PROF_SKIP & 8
    return;
#endif
    const uint32_t nk = (total + kWave - 1) / kWave;
    for (uint32_t k = 0; k < nk; ++k) {
      const uint32_t g = k * kWave + lane;
      if (g < total) {
        const SlotEnt& e = lay.tab[lay.pkt_of(g)];
        const uint64_t addr = (((uint64_t)e.delta_hi << 32 | e.delta_lo) + g) << 4;
        uint64_t src = addr;
        if (addr + 16 > arena_len) {  // tail of the arena (or an unowned pad chunk beyond it)
          if (g - e.slot < e.nch) { fix_addr = addr; fix_g = g; }
          src = 0;
        }
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(arena + src),
                                         (__attribute__((address_space(3))) void*)(smem + k * 1024u), 16, 0, 0);
      }
    }
  }
  __device__ __forceinline__ void complete() {
    wave_sync();  // workgroup-scope fence: s_waitcnt vmcnt(0) covers the LDS-DMA writes
    if (fix_addr != ~0ull) *(uint4*)(smem + 16 * fix_g) = load_chunk_guarded(arena, fix_addr, arena_len);
    wave_sync();
  }
};

// Direct path: packets are accessed in HBM in place; nothing to stage.
struct NoStager {
  __device__ __forceinline__ void issue() {}
  __device__ __forceinline__ void complete() { wave_sync(); }
};

// LDS -> HBM for packets with write=1; chunks at packet edges are written byte-wise so bytes
// of neighbouring packets (other tiles) are never touched.
__device__ __forceinline__ void stage_out(const uint8_t* smem, const Layout& lay, uint32_t total,
                                          uint8_t* arena, int lane) {
#if MQ_PROF_SKIP & 4
  return;
#endif
  for (uint32_t g0 = 0; g0 < total; g0 += 4 * kWave) {
    uint4 v[4];
    int jj[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint32_t g = g0 + u * kWave + lane;
      jj[u] = g < total ? lay.pkt_of(g) : 0;
      if (g < total) v[u] = *(const uint4*)(smem + 16 * g);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint32_t g = g0 + u * kWave + lane;
      if (g >= total) continue;
      const SlotEnt& e = lay.tab[jj[u]];
      if (!e.write) continue;
      const uint64_t addr = (((uint64_t)e.delta_hi << 32 | e.delta_lo) + g) << 4;
      const uint64_t off = (uint64_t)e.off_hi << 32 | e.off_lo, end = off + e.len;
      const uint64_t lo = off > addr ? off : addr, hi = end < addr + 16 ? end : addr + 16;
      if (lo == addr && hi == addr + 16) {
        *(uint4*)(arena + addr) = v[u];
      } else {
        const uint32_t w[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
        for (uint64_t a = lo; a < hi; ++a) arena[a] = (uint8_t)(w[(a - addr) >> 2] >> (8 * ((a - addr) & 3)));
      }
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
                                             const KeyRow*& row, uint64_t& sample_at) {
  const uint32_t count = n_dev ? *n_dev : n;
  if (t >= count) return false;
  i = index ? index[t] : t;
  const mq_pkt_desc d = desc[i];
  if (d.key_id >= n_rows || d.offset + (uint64_t)d.len > arena_len || (d.flags & MQ_PKT_NO_HP) ||
      (uint64_t)d.pn_offset + 20 > d.len)
    return false;
  row = kt + d.key_id;
  if (row->suite != suite) return false;
  sample_at = d.offset + d.pn_offset + 4;
  return true;
}

template <class Policy, bool OPEN>
__device__ __forceinline__ void run_tile(uint8_t* smem, uint32_t tile_id, const KeyRow* __restrict__ kt,
                                         uint32_t n_rows, uint8_t* __restrict__ arena, uint64_t arena_len,
                                         const mq_pkt_desc* __restrict__ desc, uint32_t n,
                                         const uint32_t* __restrict__ index,
                                         const uint32_t* __restrict__ n_dev,
                                         uint8_t* __restrict__ status, uint64_t* __restrict__ pn_out,
                                         const uint2* __restrict__ hpm) {
  const int lane = threadIdx.x & (kWave - 1), p = lane / kLanesPerPkt, j = lane % kLanesPerPkt;
  const uint32_t count = n_dev ? *n_dev : n;
  const uint32_t tile0 = tile_id * kPktsPerTile;
  if (tile0 >= count) return;  // wave-uniform
  MQ_STAMP(tile_id, 0);
  PktCtx c;
  c.tile = tile_id;
  const uint32_t t = tile0 + p;
  c.valid = t < count;
  c.i = c.valid ? (index ? index[t] : t) : 0u;
  if (c.valid) {
    c.d = desc[c.i];
  } else {
    c.d.offset = 0; c.d.len = 0; c.d.key_id = 0; c.d.pn = 0; c.d.pn_offset = 0; c.d.pn_len = 0;
    c.d.flags = 0; c.d.reserved = 0;
  }
  c.pre_hp = OPEN && hpm != nullptr;
  c.hm0 = c.hm1 = 0;
  if (OPEN && hpm && c.valid) {
    const uint2 m = hpm[c.i];
    c.hm0 = m.x;
    c.hm1 = m.y;
  }
  c.st = c.valid ? validate<Policy::kSuite, OPEN>(c.d, kt, n_rows, arena_len) : (int)MQ_ERR_INVALID_ARG;
  c.act = c.valid && c.st == MQ_OK;
  c.pn = c.d.pn;
  const KeyRow* row = kt + (c.act ? c.d.key_id : 0u);
  const uint64_t off = c.act ? c.d.offset : 0;
  // chunks of the packet's image, clamped so sums cannot overflow; a clamped (huge) packet always
  // exceeds the budget and sends the tile down the direct path
  const uint64_t nch64 = c.act ? ((off + c.d.len + 15) >> 4) - (off >> 4) : 0u;
  const uint32_t nch = (uint32_t)(nch64 < 0xFFFFu ? nch64 : 0xFFFFu);
  const uint32_t S = wave_max_u32(nch);
  const uint32_t mine = (j == 0) ? nch : 0u;
  const uint32_t incl = wave_incl_scan(mine, lane);
  const uint32_t sum = (uint32_t)__shfl((int)incl, kWave - 1, kWave);
  const bool fixed = S * 16u * kPktsPerTile <= kDataBudget;
  const uint32_t total = fixed ? S * kPktsPerTile : sum;
  if (fixed || total * 16u <= kDataBudget) {
    SlotEnt* tab = (SlotEnt*)(smem + kTableOff);
    const uint32_t slot = fixed ? S * (uint32_t)p : oct_bcast0(incl - mine);
    if (j == 0) {
      const uint64_t delta = (off >> 4) - slot;
      tab[p].slot = slot; tab[p].nch = nch; tab[p].delta_lo = (uint32_t)delta;
      tab[p].delta_hi = (uint32_t)(delta >> 32); tab[p].off_lo = (uint32_t)off;
      tab[p].off_hi = (uint32_t)(off >> 32); tab[p].len = c.act ? c.d.len : 0u; tab[p].write = 0;
    }
    wave_sync();
    const Layout lay{tab, fixed ? S : 0u, fixed && S ? ((1u << 20) + S - 1) / S : 0u};
    DmaStager stg{smem, lay, total, arena, arena_len, lane};
    LdsSpace sp{smem};
    MQ_STAMP(tile_id, 1);
    const uint32_t pkt = slot * 16u + (uint32_t)(off & 15);
    if (OPEN) Policy::template open<LdsSpace>(sp, pkt, c, row, j, false, stg);
    else Policy::template seal<LdsSpace>(sp, pkt, c, row, j, stg);
    MQ_STAMP(tile_id, 6);
    wave_sync();
    if (j == 0) tab[p].write = c.act ? 1u : 0u;
    wave_sync();
    stage_out(smem, lay, total, arena, lane);
    MQ_STAMP(tile_id, 7);
  } else {
    GlobalSpace sp{arena, arena_len};
    NoStager stg;
    if (OPEN) Policy::template open<GlobalSpace>(sp, off, c, row, j, true, stg);
    else Policy::template seal<GlobalSpace>(sp, off, c, row, j, stg);
  }
  if (c.valid && j == 0) {
    status[c.i] = (uint8_t)c.st;
    if (OPEN && pn_out && c.st == MQ_OK) pn_out[c.i] = c.pn;
  }
}

}  // namespace mq
