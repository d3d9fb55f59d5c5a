// mq_tile.h — tile framework shared by the ChaCha20-Poly1305 and AES-128-GCM kernels:
// descriptor validation, HBM<->LDS gather/scatter of whole packets, packet-number decoding.
#pragma once
#include "mq_device.h"

namespace mq {

constexpr uint32_t kSlotBytes = 32;
constexpr uint32_t kTableOff = kLdsBytes - kPktsPerTile * kSlotBytes;  // 19968
constexpr uint32_t kDataBudget = kTableOff - kSlack;                   // 19904 bytes of packets
constexpr uint64_t kMaxPn = (1ull << 62) - 1;                           // varint::MAX_VARINT

struct SlotEnt {  // one per packet of the tile, in LDS
  uint32_t slot;    // first 16-B chunk of the packet's LDS image
  uint32_t nch;     // chunks in the image
  uint32_t off_lo;  // arena byte offset of the packet (low / high words)
  uint32_t off_hi;
  uint32_t len;     // packet bytes
  uint32_t write;   // 1: store the packet back (status OK)
  uint32_t pad[2];
};

// Per-lane view of its quad's packet.
struct PktCtx {
  uint32_t i;        // descriptor index
  bool valid;        // lane maps to a descriptor
  bool act;          // still being processed (no error so far)
  int st;            // MQ_* status
  mq_pkt_desc d;
  uint64_t pn;       // full packet number (seal: from d; open: decoded)
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

// Largest j with slot[j] <= g (slots are non-decreasing; empty images share the next slot).
__device__ __forceinline__ int find_slot(const SlotEnt* tab, uint32_t g) {
  int j = 0;
#pragma unroll
  for (int step = 8; step >= 1; step >>= 1)
    if (tab[j + step].slot <= g) j += step;
  return j;
}

__device__ __forceinline__ uint4 load_chunk_guarded(const uint8_t* arena, uint64_t addr, uint64_t len) {
  if (addr + 16 <= len) return *(const uint4*)(arena + addr);
  uint32_t w[4] = {0, 0, 0, 0};
  for (int b = 0; b < 16; ++b)
    if (addr + b < len) w[b >> 2] |= (uint32_t)arena[addr + b] << (8 * (b & 3));
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// HBM -> LDS: `total` 16-B chunks, whole packets, 1 KiB contiguous per wave instruction for
// adjacent packets; 4 chunks in flight per lane.
__device__ __forceinline__ void stage_in(uint8_t* smem, const SlotEnt* tab, uint32_t total,
                                         const uint8_t* arena, uint64_t arena_len, int lane) {
  for (uint32_t g0 = 0; g0 < total; g0 += 4 * kWave) {
    uint4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      uint32_t g = g0 + u * kWave + lane;
      if (g < total) {
        int j = find_slot(tab, g);
        uint64_t off = ((uint64_t)tab[j].off_hi << 32) | tab[j].off_lo;
        uint64_t addr = ((off >> 4) + (g - tab[j].slot)) << 4;
        v[u] = load_chunk_guarded(arena, addr, arena_len);
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      uint32_t g = g0 + u * kWave + lane;
      if (g < total) *(uint4*)(smem + 16 * g) = v[u];
    }
  }
}

// LDS -> HBM for packets with write=1; chunks at packet edges are written byte-wise so bytes
// of neighbouring packets (other tiles) are never touched.
__device__ __forceinline__ void stage_out(const uint8_t* smem, const SlotEnt* tab, uint32_t total,
                                          uint8_t* arena, int lane) {
  for (uint32_t g0 = 0; g0 < total; g0 += 4 * kWave) {
    uint4 v[4];
    int jj[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      uint32_t g = g0 + u * kWave + lane;
      jj[u] = g < total ? find_slot(tab, g) : 0;
      if (g < total) v[u] = *(const uint4*)(smem + 16 * g);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      uint32_t g = g0 + u * kWave + lane;
      if (g >= total) continue;
      const SlotEnt& e = tab[jj[u]];
      if (!e.write) continue;
      uint64_t off = ((uint64_t)e.off_hi << 32) | e.off_lo;
      uint64_t addr = ((off >> 4) + (g - e.slot)) << 4;
      uint64_t lo = off > addr ? off : addr, end = off + e.len;
      uint64_t hi = end < addr + 16 ? end : addr + 16;
      if (lo == addr && hi == addr + 16) {
        *(uint4*)(arena + addr) = v[u];
      } else {
        uint32_t w[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
        for (uint64_t a = lo; a < hi; ++a) arena[a] = (uint8_t)(w[(a - addr) >> 2] >> (8 * ((a - addr) & 3)));
      }
    }
  }
}

}  // namespace mq

namespace mq {

// Tile driver shared by every suite policy. One 64-lane wave = one tile of 16 packets; `smem`
// is the wave's private kLdsBytes LDS region.
// Policy provides kSuite and
//   template <class S> static __device__ void seal(const S&, S::off_t pkt, PktCtx&, const KeyRow*, int q);
//   template <class S> static __device__ void open(const S&, S::off_t pkt, PktCtx&, const KeyRow*, int q, bool direct);
// Both must execute every wave_sync() in wave-uniform control flow.
template <class Policy, bool OPEN>
__device__ __forceinline__ void run_tile(uint8_t* smem, uint32_t tile_id, const KeyRow* __restrict__ kt,
                                         uint32_t n_rows,
                                         uint8_t* __restrict__ arena, uint64_t arena_len,
                                         const mq_pkt_desc* __restrict__ desc, uint32_t n,
                                         const uint32_t* __restrict__ index,
                                         const uint32_t* __restrict__ n_dev,
                                         uint8_t* __restrict__ status, uint64_t* __restrict__ pn_out) {
  const int lane = threadIdx.x & (kWave - 1), p = lane >> 2, q = lane & 3;
  const uint32_t count = n_dev ? *n_dev : n;
  const uint32_t tile0 = tile_id * kPktsPerTile;
  if (tile0 >= count) return;  // wave-uniform
  PktCtx c;
  const uint32_t t = tile0 + p;
  c.valid = t < count;
  c.i = c.valid ? (index ? index[t] : t) : 0u;
  if (c.valid) {
    c.d = desc[c.i];
  } else {
    c.d.offset = 0; c.d.len = 0; c.d.key_id = 0; c.d.pn = 0; c.d.pn_offset = 0; c.d.pn_len = 0;
    c.d.flags = 0; c.d.reserved = 0;
  }
  c.st = c.valid ? validate<Policy::kSuite, OPEN>(c.d, kt, n_rows, arena_len) : (int)MQ_ERR_INVALID_ARG;
  c.act = c.valid && c.st == MQ_OK;
  c.pn = c.d.pn;
  const KeyRow* row = kt + (c.act ? c.d.key_id : 0u);
  const uint64_t off = c.act ? c.d.offset : 0;
  // chunks of the packet's LDS image, clamped so the 16-packet scan cannot overflow; a clamped
  // (huge) packet always exceeds the budget and sends the tile down the direct path
  const uint64_t nch64 = c.act ? ((off + c.d.len + 15) >> 4) - (off >> 4) : 0u;
  const uint32_t nch = (uint32_t)(nch64 < 0xFFFFu ? nch64 : 0xFFFFu);
  const uint32_t mine = (q == 0) ? nch : 0u;
  const uint32_t incl = wave_incl_scan(mine, lane);
  const uint32_t total = (uint32_t)__shfl((int)incl, 63, 64);
  const uint32_t slot = quad_bcast0(incl - mine);
  if (total * 16u <= kDataBudget) {
    SlotEnt* tab = (SlotEnt*)(smem + kTableOff);
    if (q == 0) {
      tab[p].slot = slot; tab[p].nch = nch; tab[p].off_lo = (uint32_t)off;
      tab[p].off_hi = (uint32_t)(off >> 32); tab[p].len = c.act ? c.d.len : 0u; tab[p].write = 0;
    }
    wave_sync();
    stage_in(smem, tab, total, arena, arena_len, lane);
    wave_sync();
    LdsSpace sp{smem};
    const uint32_t pkt = slot * 16u + (uint32_t)(off & 15);
    if (OPEN) Policy::template open<LdsSpace>(sp, pkt, c, row, q, false);
    else Policy::template seal<LdsSpace>(sp, pkt, c, row, q);
    wave_sync();
    if (q == 0) tab[p].write = c.act ? 1u : 0u;
    wave_sync();
    stage_out(smem, tab, total, arena, lane);
  } else {
    GlobalSpace sp{arena, arena_len};
    if (OPEN) Policy::template open<GlobalSpace>(sp, off, c, row, q, true);
    else Policy::template seal<GlobalSpace>(sp, off, c, row, q);
  }
  if (c.valid && q == 0) {
    status[c.i] = (uint8_t)c.st;
    if (OPEN && pn_out && c.st == MQ_OK) pn_out[c.i] = c.pn;
  }
}

}  // namespace mq
