// mq_device.h — device-side building blocks of the MI355X (gfx950) packet-protection kernels.
//
// Execution model: one 64-lane wave processes a TILE of kPktsPerTile = 8
// packets; each packet is owned by an OCTET of kLanesPerPkt = 8 lanes (lane = 8*p + j).
//   * staging: the tile's packets are gathered HBM -> LDS with whole-packet contiguous
//     16-B-per-lane loads (1 KiB per wave instruction), because one-packet-per-lane strided
//     access measured 2.7 TB/s vs 5.5 TB/s contiguous on MI355X (tools/ubench/ubench3.hip);
//   * keystream blocks of a packet are spread over its octet (ChaCha20 64-B blocks / AES-CTR
//     16-B blocks, block b on lane b % 8), XORed in LDS;
//   * the MAC (Poly1305 / GHASH) is an 8-way interleaved Horner evaluation (lane j takes MAC
//     blocks i = 8k + j with multiplier r^8 / H^8, then one final multiply by r^(8-j) / H^(8-j))
//     followed by an octet reduction through DPP;
//   * header protection and the store back to HBM close the tile.
// Tiles whose packets do not fit the LDS budget run the same code on HBM directly ("direct").
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mq_aead.h"

namespace mq {

constexpr int kWave = 64;
constexpr int kPktsPerTile = 8;
// dynamic tile schedule slot of a persistent launch (mq_tile.h TileSched), uint32 words: head h at
// word kSchedHeadWords * h (128 B apart), the finished-workgroup count at kSchedDoneWord
constexpr uint32_t kSchedHeads = 8;
constexpr uint32_t kSchedHeadWords = 32;
constexpr uint32_t kSchedDoneWord = kSchedHeads * kSchedHeadWords;
constexpr uint32_t kSchedSlotBytes = 4 * (kSchedDoneWord + kSchedHeadWords);  // 1152 B
constexpr int kLanesPerPkt = kWave / kPktsPerTile;  // 8: one octet of lanes per packet
constexpr uint32_t kLdsBytes = 10240;                // LDS per tile (wave) -> 16 waves/CU
constexpr uint32_t kCuLdsBytes = 160 * 1024;         // LDS per CU (gfx950)

// Device key-table row (576 B). Filled on the host by mq_keytable_create (mq_host.cpp).
struct alignas(16) KeyRow {
  uint32_t suite;
  uint32_t pad0[3];
  uint32_t iv[3];      // IV bytes as 3 little-endian words
  uint32_t pad1;
  uint32_t key[8];     // ChaCha20 key (LE words)
  uint32_t hp[8];      // ChaCha20 HP key (LE words)
  uint32_t aes_rk[44]; // AES-128 round keys of the AEAD key (FIPS-197 big-endian words)
  uint32_t hp_rk[44];  // AES-128 round keys of the HP key
  uint32_t H[8][4];    // GHASH H^1..H^8 (GCM byte order, big-endian words)
};
static_assert(sizeof(KeyRow) == 576, "KeyRow layout");

constexpr uint32_t kMaxCidLen = 20;  // RFC 9000 §17.2 (reference ConnectionId capacity)

// Constants of the batched Initial key derivation (mq_derive.hip), computed once on the host:
// the compressed HMAC pads of the QUIC v1 salt (key_schedule.rs:10-13) and the padded HMAC
// message blocks of HKDF-Expand-Label(secret, label, "", L) || 0x01 for "client in" (32),
// "server in" (32), "quic key" (16), "quic iv" (12), "quic hp" (16) (key_schedule.rs:23-55).
struct MQDeriveConsts {
  uint32_t salt_ist[8], salt_ost[8];
  uint32_t lbl[5][16];
};

// The AEAD passes of the datagram receive composite (mq_recv.hip), run by mq_host.cpp's batch
// driver: primary descriptors / statuses, retry (previous-generation keys) descriptors / statuses.
struct MQRecvPass {
  mq_pkt_desc *d1, *d2;
  uint8_t *st1, *st2;
  void* open_ws;
  const uint32_t *live1, *live2;  // keyed descriptors of d1 (the last walk) / d2 (the retry kernel)
};

// ------------------------------------------------------------------------------------------
// byte-address spaces: LDS (staged tile) or the HBM arena (direct path)
struct LdsSpace {
  uint8_t* base;
  typedef uint32_t off_t;
  __device__ __forceinline__ uint32_t ld32(uint32_t a) const { return *(const uint32_t*)(base + a); }
  __device__ __forceinline__ void st32(uint32_t a, uint32_t v) const { *(uint32_t*)(base + a) = v; }
  __device__ __forceinline__ uint8_t ld8(uint32_t a) const { return base[a]; }
  __device__ __forceinline__ void st8(uint32_t a, uint8_t v) const { base[a] = v; }
  __device__ __forceinline__ void xor32(uint32_t a, uint32_t v) const { atomicXor((uint32_t*)(base + a), v); }
  // dword at a: bytes under `mask` become those of v (the wave's private image: no other writer)
  __device__ __forceinline__ void merge32(uint32_t a, uint32_t old, uint32_t v, uint32_t mask) const {
    st32(a, (old & ~mask) | (v & mask));
  }
};

struct GlobalSpace {
  uint8_t* base;
  uint64_t len;  // reads at or beyond len return 0 (never fault)
  typedef uint64_t off_t;
  __device__ __forceinline__ uint32_t ld32(uint64_t a) const {
    if (a + 4 <= len) return *(const uint32_t*)(base + a);
    uint32_t w = 0;  // tail of an arena whose length is not a multiple of 4
    for (int b = 0; b < 4; ++b)
      if (a + b < len) w |= (uint32_t)base[a + b] << (8 * b);
    return w;
  }
  __device__ __forceinline__ void st32(uint64_t a, uint32_t v) const { *(uint32_t*)(base + a) = v; }
  __device__ __forceinline__ uint8_t ld8(uint64_t a) const { return a < len ? base[a] : (uint8_t)0; }
  __device__ __forceinline__ void st8(uint64_t a, uint8_t v) const { base[a] = v; }
  __device__ __forceinline__ void xor32(uint64_t a, uint32_t v) const { atomicXor((uint32_t*)(base + a), v); }
  // dword at a: bytes under `mask` become those of v. Another wave may be updating the other
  // bytes (a neighbouring packet on the direct path), so only the change of ours is XORed in.
  __device__ __forceinline__ void merge32(uint64_t a, uint32_t old, uint32_t v, uint32_t mask) const {
    xor32(a, (old ^ v) & mask);
  }
};

// v_perm_b32 selectors: loads realign memory dwords to a payload that starts `v` bytes into a
// dword; stores realign payload words back to memory dwords. perm(hi, lo, sel) picks bytes of
// the 8-byte {hi, lo} pair (lo = bytes 0..3).
__device__ __forceinline__ uint32_t sel_load(uint32_t v) { return 0x03020100u + v * 0x01010101u; }
__device__ __forceinline__ uint32_t sel_store(uint32_t v) { return 0x07060504u - v * 0x01010101u; }
__device__ __forceinline__ uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel) {
  return __builtin_amdgcn_perm(hi, lo, sel);
}

// Read N payload-aligned words starting at dword-aligned address b + (alignment encoded in the
// v_perm selector `sel` = sel_load(a & 3)), for loops that step a fixed stride.
template <int N, class S>
__device__ __forceinline__ void load_words_sel(const S& sp, typename S::off_t b, uint32_t sel, uint32_t (&w)[N]) {
  uint32_t m[N + 1];
#pragma unroll
  for (int k = 0; k <= N; ++k) m[k] = sp.ld32(b + 4 * k);
#pragma unroll
  for (int k = 0; k < N; ++k) w[k] = perm(m[k + 1], m[k], sel);
}

// Read N payload-aligned words starting at byte address `a` (any alignment).
template <int N, class S>
__device__ __forceinline__ void load_words(const S& sp, typename S::off_t a, uint32_t (&w)[N]) {
  load_words_sel<N>(sp, a & ~(typename S::off_t)3, sel_load((uint32_t)(a & 3)), w);
}

// bytes [lo, hi) of a dword
__device__ __forceinline__ uint32_t range_mask(int lo, int hi) {
  const uint32_t h = hi >= 4 ? 0xffffffffu : ((1u << (8 * hi)) - 1u);
  const uint32_t l = lo <= 0 ? 0u : ((1u << (8 * lo)) - 1u);
  return h & ~l;
}

// Raw memory dwords covering N payload words at byte address `a` (for xor_words).
template <int N, class S>
__device__ __forceinline__ void load_raw(const S& sp, typename S::off_t a, uint32_t (&raw)[N + 1]) {
  const typename S::off_t b = a & ~(typename S::off_t)3;
#pragma unroll
  for (int m = 0; m <= N; ++m) raw[m] = sp.ld32(b + 4 * m);
}

// bytes [a, a + len) ^= payload-aligned keystream words ks (len <= 4N); `raw` = load_raw(a).
// Dwords wholly inside the range are rewritten from raw; the (at most two) edge dwords, which
// other lanes of the octet may be updating in the same instruction, take an atomic XOR of only
// this lane's bytes (ds_xor_b32), so neighbouring ranges never race.
template <int N, class S>
__device__ __forceinline__ void xor_words(const S& sp, typename S::off_t a, const uint32_t (&ks)[N], int len,
                                          const uint32_t (&raw)[N + 1]) {
  const typename S::off_t b = a & ~(typename S::off_t)3;
  const int v = (int)(a & 3);
  const uint32_t sel = sel_store((uint32_t)v);
  if (len == 4 * N) {
#pragma unroll
    for (int m = 1; m < N; ++m) sp.st32(b + 4 * m, raw[m] ^ perm(ks[m], ks[m - 1], sel));
    sp.xor32(b, perm(ks[0], 0u, sel) & range_mask(v, 4));
    if (v) sp.xor32(b + 4 * N, perm(0u, ks[N - 1], sel) & range_mask(0, v));
    return;
  }
#pragma unroll
  for (int m = 0; m <= N; ++m) {
    const uint32_t out = perm(m < N ? ks[m] : 0u, m > 0 ? ks[m - 1] : 0u, sel);
    const int lo_idx = 4 * m - v;  // payload index of byte 0 of this memory dword
    if (lo_idx >= 0 && lo_idx + 4 <= len) {
      sp.st32(b + 4 * m, raw[m] ^ out);
    } else if (lo_idx + 4 > 0 && lo_idx < len) {
      sp.xor32(b + 4 * m, out & range_mask(-lo_idx, len - lo_idx));
    }
  }
}

// Write N payload-aligned words at byte address `a` (any alignment), preserving the bytes of
// the two edge dwords outside the range. Only for a single writer per packet (e.g. the tag,
// written by lane j == 0 after every keystream update of its packet).
template <int N, class S>
__device__ __forceinline__ void store_words(const S& sp, typename S::off_t a, const uint32_t (&w)[N]) {
  const typename S::off_t b = a & ~(typename S::off_t)3;
  const int v = (int)(a & 3);
  const uint32_t sel = sel_store((uint32_t)v);
  if (v == 0) {
#pragma unroll
    for (int m = 0; m < N; ++m) sp.st32(b + 4 * m, w[m]);
    return;
  }
  const uint32_t keep = range_mask(0, v);
  const uint32_t e0 = sp.ld32(b), eN = sp.ld32(b + 4 * N);
#pragma unroll
  for (int m = 1; m < N; ++m) sp.st32(b + 4 * m, perm(w[m], w[m - 1], sel));
  // edge dwords: only this packet's bytes change (merge32: race-free on the direct path)
  sp.merge32(b, e0, perm(w[0], 0u, sel), ~keep);
  sp.merge32(b + 4 * N, eN, perm(0u, w[N - 1], sel), keep);
}

// Keep the compiler from sinking the wait for `x`'s load past this point (used to retire the
// key loads before LDS-DMA is issued: hipcc would otherwise wait vmcnt(0) on the DMA too).
__device__ __forceinline__ void pin(uint32_t& x) { asm volatile("" : "+v"(x)); }

__device__ __forceinline__ uint32_t byte_mask(int rem, int k) {  // keep bytes < rem of word k
  int r = rem - 4 * k;
  return r >= 4 ? 0xffffffffu : (r <= 0 ? 0u : ((1u << (8 * r)) - 1u));
}

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

// 16-B packet accesses at any byte alignment (global_load/store_dwordx4; gfx950 runs with
// unaligned access enabled). A store writes exactly its 16 bytes, so lanes storing adjacent
// ranges of a packet (or of neighbouring packets) never need a read-modify-write.
typedef uint4 __attribute__((aligned(1))) uint4_u;
typedef uint32_t __attribute__((aligned(1))) u32_u;  // unaligned dword access
__device__ __forceinline__ uint4 ld16(const uint8_t* p) { return *(const uint4_u*)p; }
__device__ __forceinline__ void st16(uint8_t* p, const uint32_t (&w)[4]) {
  *(uint4_u*)p = make_uint4(w[0], w[1], w[2], w[3]);
}
__device__ __forceinline__ void st_bytes(uint8_t* p, const uint32_t (&w)[4], uint32_t n) {
  for (uint32_t k = 0; k < n; ++k) p[k] = (uint8_t)(w[k >> 2] >> (8 * (k & 3)));
}
__device__ __forceinline__ void st_block(uint8_t* p, const uint32_t (&w)[4], uint32_t rem) {
  if (rem >= 16) st16(p, w);
  else st_bytes(p, w, rem);
}
__device__ __forceinline__ void u4w(uint4 v, uint32_t (&w)[4]) { w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w; }

// ------------------------------------------------------------------------------------------
// MQ_PROF_SKIP (diagnostic builds from `make prof-variants`, never the product library): bit 1
// skips the ChaCha rounds, 2 the MAC, 4 the LDS->HBM store, 8 the HBM->LDS staging, 16 the AES
// rounds, 64 the AES tag's final multiply by H^e; the timing differences give each phase's cost
// under full load (tools/phase_cost.py).
#ifndef MQ_PROF_SKIP
#define MQ_PROF_SKIP 0
#endif

// Diagnostic phase stamps (only in the -DMQ_STAMPS build, libmq_aead_stamps.so): lane 0 of each
// tile records s_memtime at phase boundaries into mq_stamp_buf[tile][slot]. Never compiled into
// the product library; read by tools/stamps.py.
#ifdef MQ_STAMPS
constexpr int kStampSlots = 8;
static __device__ uint64_t* mq_stamp_buf;  // one copy per translation unit, set by mq_debug_set_stamps
#define MQ_STAMP(tile, slot)                                                        \
  do {                                                                              \
    __builtin_amdgcn_sched_barrier(0);                                              \
    uint64_t _t = __builtin_amdgcn_s_memtime();                                     \
    if ((threadIdx.x & 63) == 0 && mq_stamp_buf)                                    \
      mq_stamp_buf[(size_t)(tile) * kStampSlots + (slot)] = _t;                     \
    __builtin_amdgcn_sched_barrier(0);                                              \
  } while (0)
#else
#define MQ_STAMP(tile, slot) do { } while (0)
#endif

// ------------------------------------------------------------------------------------------
// DPP within a quad (lanes 4p..4p+3): quad_perm selectors
__device__ __forceinline__ uint32_t quad_bcast0(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x00, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t quad_swap1(uint32_t x) {  // [1,0,3,2]
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t quad_swap2(uint32_t x) {  // [2,3,0,1]
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x4E, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t half_mirror(uint32_t x) {  // lane i <- lane 7-i within 8
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x141, 0xf, 0xf, false);
}
// octet (8-lane group) broadcast of lane 0 / sums: ds_swizzle bit mode, and_mask 0x18
__device__ __forceinline__ uint32_t oct_bcast0(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, 0x18);
}
__device__ __forceinline__ uint32_t oct_lane3(uint32_t x) {  // lane 3 of the octet
  return (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, 0x78);
}
__device__ __forceinline__ uint32_t oct_lane7(uint32_t x) {  // lane 7 of the octet
  return (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, 0xF8);
}
__device__ __forceinline__ uint32_t oct_sum(uint32_t x) {
  x += quad_swap1(x);
  x += quad_swap2(x);
  return x + half_mirror(x);
}
__device__ __forceinline__ uint32_t oct_xor(uint32_t x) {
  x ^= quad_swap1(x);
  x ^= quad_swap2(x);
  return x ^ half_mirror(x);
}

// Wave-local barrier: tiles are private to one wave, so ordering the wave's own LDS / HBM
// accesses (and keeping the compiler from moving them) is all a phase boundary needs. Unlike
// __syncthreads() it is safe in multi-wave workgroups whose waves take different paths.
// this wave's index in its workgroup (scalar)
__device__ __forceinline__ uint32_t wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// Reductions over the wave for OCTET-UNIFORM values (every lane of an octet holds the same
// value, as for per-packet quantities): DPP row_mirror folds the two octets of a row, then
// row_bcast15 / row_bcast31 fold the rows; the result is read from lane 63 (wave-uniform).
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t x) {
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x140, 0xf, 0xf, false));  // row_mirror
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x142, 0xa, 0xf, false));  // row_bcast15
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x143, 0xc, 0xf, false));  // row_bcast31
  return (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}
// inclusive prefix sum over the octets (octet-uniform x): octet q gets x_0 + ... + x_q
__device__ __forceinline__ uint32_t oct_incl_scan(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, true);   // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast15
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast31
  return x;
}
// minimum over the wave of an octet-uniform value
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t x) { return ~wave_max_u32(~x); }
// inclusive prefix sum over the 64 lanes of a wave (DPP row shifts + row broadcasts)
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);  // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);  // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return x;
}
__device__ __forceinline__ bool wave_any(bool b) { return __builtin_amdgcn_ballot_w64(b) != 0; }
// maximum / minimum over the wave of ANY per-lane value (quads, then octets, then the octet fold)
__device__ __forceinline__ uint32_t wave_max_any(uint32_t x) {
  x = max(x, quad_swap1(x));
  x = max(x, quad_swap2(x));
  x = max(x, half_mirror(x));
  return wave_max_u32(x);
}
__device__ __forceinline__ uint32_t wave_min_any(uint32_t x) { return ~wave_max_any(~x); }

// Lane groups of G = 1, 2, 4 or 8 lanes (one packet per group, lane = G p + j; the narrow ChaCha20
// tiles, mq_chacha.hip): broadcast of group lane 0, of the last lane, the mirror j -> G-1-j, the sum
// over the group. DPP quad_perm inside a quad (G <= 4), the octet ops above for G = 8.
template <int G>
struct Grp {
  static_assert(G == 1 || G == 2 || G == 4 || G == 8, "lane group of 1, 2, 4 or 8");
  template <int SEL>
  static __device__ __forceinline__ uint32_t qp(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, SEL, 0xf, 0xf, false);
  }
  static __device__ __forceinline__ uint32_t bcast0(uint32_t x) {
    if (G == 1) return x;
    if (G == 2) return qp<0xA0>(x);  // [0,0,2,2]
    if (G == 4) return qp<0x00>(x);  // [0,0,0,0]
    return oct_bcast0(x);
  }
  static __device__ __forceinline__ uint32_t last(uint32_t x) {
    if (G == 1) return x;
    if (G == 2) return qp<0xF5>(x);  // [1,1,3,3]
    if (G == 4) return qp<0xFF>(x);  // [3,3,3,3]
    return oct_lane7(x);
  }
  static __device__ __forceinline__ uint32_t mirror(uint32_t x) {
    if (G == 1) return x;
    if (G == 2) return quad_swap1(x);
    if (G == 4) return qp<0x1B>(x);  // [3,2,1,0]
    return half_mirror(x);
  }
  static __device__ __forceinline__ uint32_t sum(uint32_t x) {
    if (G == 1) return x;
    x += quad_swap1(x);
    if (G == 2) return x;
    x += quad_swap2(x);
    if (G == 4) return x;
    return x + half_mirror(x);
  }
  static __device__ __forceinline__ uint32_t xr(uint32_t x) {  // XOR over the group
    if (G == 1) return x;
    x ^= quad_swap1(x);
    if (G == 2) return x;
    x ^= quad_swap2(x);
    if (G == 4) return x;
    return x ^ half_mirror(x);
  }
  template <int K>  // group lane K, to every lane of the group
  static __device__ __forceinline__ uint32_t lane(uint32_t x) {
    static_assert(K >= 0 && K < G, "lane of the group");
    if (G == 1) return x;
    if (G == 2) return qp<K | (K << 2) | ((K + 2) << 4) | ((K + 2) << 6)>(x);
    if (G == 4) return qp<K | (K << 2) | (K << 4) | (K << 6)>(x);
    return (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, 0x18 | (K << 5));
  }
  // maximum over the wave of a GROUP-UNIFORM value (fold the groups of an octet, then the octets)
  static __device__ __forceinline__ uint32_t wave_max(uint32_t x);
  static __device__ __forceinline__ uint32_t wave_min(uint32_t x) { return ~wave_max(~x); }
};
template <int G>
__device__ __forceinline__ uint32_t Grp<G>::wave_max(uint32_t x) {
  if (G <= 2) x = max(x, quad_swap2(x));
  if (G <= 4) x = max(x, half_mirror(x));
  if (G == 1) x = max(x, quad_swap1(x));
  return wave_max_u32(x);
}
__device__ __forceinline__ uint64_t wave_min_u64(uint64_t x) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    uint64_t y = __shfl_xor(x, d, 64);
    x = x < y ? x : y;
  }
  return x;
}
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t x) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    uint64_t y = __shfl_xor(x, d, 64);
    x = x > y ? x : y;
  }
  return x;
}

// ------------------------------------------------------------------------------------------
// ChaCha20 block function (RFC 8439 §2.3): out = keystream words of block `ctr`.
__device__ __forceinline__ uint32_t rotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

#define MQ_QR(a, b, c, d)                 \
  a += b; d ^= a; d = rotl(d, 16);        \
  c += d; b ^= c; b = rotl(b, 12);        \
  a += b; d ^= a; d = rotl(d, 8);         \
  c += d; b ^= c; b = rotl(b, 7);

__device__ __forceinline__ void chacha20_block(const uint32_t (&key)[8], uint32_t ctr,
                                               uint32_t n0, uint32_t n1, uint32_t n2,
                                               uint32_t (&out)[16]) {
#if MQ_PROF_SKIP & 1  // phase-cost diagnostic build only (tools/phase_cost.py): no rounds
#pragma unroll
  for (int k = 0; k < 16; ++k) out[k] = key[k & 7] ^ ctr ^ n0 ^ (k == 13 ? n1 : n2);
  return;
#endif
  uint32_t x0 = 0x61707865u, x1 = 0x3320646eu, x2 = 0x79622d32u, x3 = 0x6b206574u;
  uint32_t x4 = key[0], x5 = key[1], x6 = key[2], x7 = key[3];
  uint32_t x8 = key[4], x9 = key[5], x10 = key[6], x11 = key[7];
  uint32_t x12 = ctr, x13 = n0, x14 = n1, x15 = n2;
#pragma unroll 2
  for (int i = 0; i < 10; ++i) {
    MQ_QR(x0, x4, x8, x12) MQ_QR(x1, x5, x9, x13) MQ_QR(x2, x6, x10, x14) MQ_QR(x3, x7, x11, x15)
    MQ_QR(x0, x5, x10, x15) MQ_QR(x1, x6, x11, x12) MQ_QR(x2, x7, x8, x13) MQ_QR(x3, x4, x9, x14)
  }
  out[0] = x0 + 0x61707865u; out[1] = x1 + 0x3320646eu; out[2] = x2 + 0x79622d32u;
  out[3] = x3 + 0x6b206574u;
  out[4] = x4 + key[0]; out[5] = x5 + key[1]; out[6] = x6 + key[2]; out[7] = x7 + key[3];
  out[8] = x8 + key[4]; out[9] = x9 + key[5]; out[10] = x10 + key[6]; out[11] = x11 + key[7];
  out[12] = x12 + ctr; out[13] = x13 + n0; out[14] = x14 + n1; out[15] = x15 + n2;
}

// ------------------------------------------------------------------------------------------
// Poly1305 arithmetic mod 2^130-5 in radix 2^26 (5 limbs), general multiplier (r, r^2..r^4).
struct P26 { uint32_t l[5]; };
struct P26m { uint32_t r[5], s[4]; };  // multiplier with s[i] = 5 * r[i+1]

__device__ __forceinline__ P26m p26_mult(const P26& r) {
  P26m m;
#pragma unroll
  for (int i = 0; i < 5; ++i) m.r[i] = r.l[i];
#pragma unroll
  for (int i = 0; i < 4; ++i) m.s[i] = r.l[i + 1] * 5u;
  return m;
}

__device__ __forceinline__ P26 p26_from_words(uint32_t t0, uint32_t t1, uint32_t t2, uint32_t t3,
                                              uint32_t hibit) {
  P26 h;
  h.l[0] = t0 & 0x3ffffff;
  h.l[1] = ((t0 >> 26) | (t1 << 6)) & 0x3ffffff;
  h.l[2] = ((t1 >> 20) | (t2 << 12)) & 0x3ffffff;
  h.l[3] = ((t2 >> 14) | (t3 << 18)) & 0x3ffffff;
  h.l[4] = (t3 >> 8) | (hibit << 24);
  return h;
}

// h = h * m (mod 2^130 - 5), partially reduced (limbs < 2^26, l[1] < 2^26 + 2^9). Inputs: limbs
// < 2^27 (a product plus one absorbed block), multiplier limbs < 2^26 (s < 2^28.4), so every
// column sum stays below 2^58 and each carry (d >> 26) below 2^32, so the top carry is a 32-bit
// operand of the x5 fold.
__device__ __forceinline__ void p26_mul(P26& h, const P26m& m) {
  const uint32_t h0 = h.l[0], h1 = h.l[1], h2 = h.l[2], h3 = h.l[3], h4 = h.l[4];
  const uint64_t d0 = (uint64_t)h0 * m.r[0] + (uint64_t)h1 * m.s[3] + (uint64_t)h2 * m.s[2] + (uint64_t)h3 * m.s[1] + (uint64_t)h4 * m.s[0];
  const uint64_t d1 = (d0 >> 26) + (uint64_t)h0 * m.r[1] + (uint64_t)h1 * m.r[0] + (uint64_t)h2 * m.s[3] + (uint64_t)h3 * m.s[2] + (uint64_t)h4 * m.s[1];
  const uint64_t d2 = (d1 >> 26) + (uint64_t)h0 * m.r[2] + (uint64_t)h1 * m.r[1] + (uint64_t)h2 * m.r[0] + (uint64_t)h3 * m.s[3] + (uint64_t)h4 * m.s[2];
  const uint64_t d3 = (d2 >> 26) + (uint64_t)h0 * m.r[3] + (uint64_t)h1 * m.r[2] + (uint64_t)h2 * m.r[1] + (uint64_t)h3 * m.r[0] + (uint64_t)h4 * m.s[3];
  const uint64_t d4 = (d3 >> 26) + (uint64_t)h0 * m.r[4] + (uint64_t)h1 * m.r[3] + (uint64_t)h2 * m.r[2] + (uint64_t)h3 * m.r[1] + (uint64_t)h4 * m.r[0];
  const uint32_t c4 = (uint32_t)(d4 >> 26);
  const uint64_t t = (uint64_t)((uint32_t)d0 & 0x3ffffff) + (uint64_t)c4 * 5u;
  h.l[0] = (uint32_t)t & 0x3ffffff;
  h.l[1] = ((uint32_t)d1 & 0x3ffffff) + (uint32_t)(t >> 26);
  h.l[2] = (uint32_t)d2 & 0x3ffffff;
  h.l[3] = (uint32_t)d3 & 0x3ffffff;
  h.l[4] = (uint32_t)d4 & 0x3ffffff;
}

// Full reduction mod p and tag = (h + s) mod 2^128, as 4 LE words.
__device__ __forceinline__ void p26_finish(P26 h, const uint32_t (&s)[4], uint32_t (&tag)[4]) {
  uint32_t c;
  c = h.l[0] >> 26; h.l[0] &= 0x3ffffff; h.l[1] += c;
  c = h.l[1] >> 26; h.l[1] &= 0x3ffffff; h.l[2] += c;
  c = h.l[2] >> 26; h.l[2] &= 0x3ffffff; h.l[3] += c;
  c = h.l[3] >> 26; h.l[3] &= 0x3ffffff; h.l[4] += c;
  c = h.l[4] >> 26; h.l[4] &= 0x3ffffff; h.l[0] += c * 5;
  c = h.l[0] >> 26; h.l[0] &= 0x3ffffff; h.l[1] += c;
  c = h.l[1] >> 26; h.l[1] &= 0x3ffffff; h.l[2] += c;
  uint32_t g0, g1, g2, g3, g4;
  g0 = h.l[0] + 5; c = g0 >> 26; g0 &= 0x3ffffff;
  g1 = h.l[1] + c; c = g1 >> 26; g1 &= 0x3ffffff;
  g2 = h.l[2] + c; c = g2 >> 26; g2 &= 0x3ffffff;
  g3 = h.l[3] + c; c = g3 >> 26; g3 &= 0x3ffffff;
  g4 = h.l[4] + c - (1u << 26);
  bool use_g = (g4 >> 31) == 0;
  uint32_t f0 = use_g ? g0 : h.l[0], f1 = use_g ? g1 : h.l[1], f2 = use_g ? g2 : h.l[2];
  uint32_t f3 = use_g ? g3 : h.l[3], f4 = use_g ? g4 : h.l[4];
  uint32_t w0 = f0 | (f1 << 26), w1 = (f1 >> 6) | (f2 << 20), w2 = (f2 >> 12) | (f3 << 14),
           w3 = (f3 >> 18) | (f4 << 8);
  uint64_t t = (uint64_t)w0 + s[0];
  tag[0] = (uint32_t)t;
  t = (uint64_t)w1 + s[1] + (t >> 32);
  tag[1] = (uint32_t)t;
  t = (uint64_t)w2 + s[2] + (t >> 32);
  tag[2] = (uint32_t)t;
  t = (uint64_t)w3 + s[3] + (t >> 32);
  tag[3] = (uint32_t)t;
}

}  // namespace mq
