// mq_resident.hip — per-packet Aead / HeaderProtection calls without a kernel launch per call.
//
// The reference's call sites are synchronous and per packet: Aead::seal_in_place
// (transmit.rs:713-718), open_in_place (recv.rs:416-421) and HeaderProtection::mask
// (transmit.rs:729, recv.rs:370) through rustcrypto.rs:38-220. Launching a kernel per call (r02:
// a batch of one) costs 30-40 us; here one resident workgroup per device (4 waves, one per SIMD)
// polls a mailbox in pinned host memory (mq_resident.h) and serves each call with all its lanes
// on ONE packet:
//   ChaCha20-Poly1305: keystream blocks on quads of lanes (a column per lane), the MAC as a 64-way
//     interleaved Horner on wave 0 (multiplier r^64, lane j's final multiplier r^(j + 1) from a
//     DPP prefix product), lanes summed in 64-bit limbs;
//   AES-128-GCM: CTR block b on thread b through the wide T-table (built once when the kernel
//     starts), GHASH on wave 0 as a 64-way Horner with the bit-holed product (multiplier H^64,
//     final H^(64-j); the host precomputes H^1 .. H^64 per context), lanes XOR-reduced;
//   header protection: one block on wave 0.
// A request runs in two halves around the packet's arrival: the polling wave reads the request
// header (key material, nonce, lengths — stamped slots, mq_resident.h) in its poll; the packet
// then streams host -> LDS by LDS-DMA while the first half runs on the header alone (keystream or
// CTR blocks, the one-time key and the powers of r, E_K(J0)); the second half (cipher XOR, MAC,
// verdict) follows the packet. Open verifies before it decrypts (a failed packet is never written
// back). Memory ordering: the host writes the packet, then the header slots, slot 0 last; the wave
// polls with system-scope 8-B loads (vector memory, never the scalar cache) and takes a
// system-scope acquire fence once the header is complete, before the packet's loads; after the
// results a system-scope release fence precedes `done`. The kernel leaves when the host asks (stop
// slot), or after `idle` ticks without a request (or `life` ticks in all) — an exit claimed with a
// Dekker-style handshake on `state` / slot 0, so a request posted meanwhile is either served or
// finds the kernel gone (the host then relaunches it).
#include "mq_aes.h"
#include "mq_opts.h"
#include "mq_resident.h"

#include <atomic>
#include <chrono>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

namespace mq {

__device__ __forceinline__ uint32_t ld_sys_sc(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys_sc(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint32_t uni(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }

// The resident workgroup: kResWaves waves, one per SIMD. Wave 0 polls; the others wait at the
// workgroup barrier (no issue slots) and join for the copies and the keystream.
constexpr int kResWaves = 4, kResThreads = 64 * kResWaves;

// LDS: the request header, the packet, the open keystream, the GHASH powers, scratch
__shared__ __attribute__((aligned(16))) uint32_t s_hdr[kResHdrSlots];
__shared__ __attribute__((aligned(16))) uint8_t s_pkt[kResMaxPkt + 64];
__shared__ __attribute__((aligned(16))) uint32_t s_ks[kResMaxPkt / 4];  // open: keystream until the tag verifies
__shared__ __attribute__((aligned(16))) uint32_t s_hpow[64 * 4];        // AES: H^1 .. H^64 of the request
__shared__ __attribute__((aligned(16))) uint32_t s_scr[16];             // [12]: open verdict
__shared__ uint32_t s_cmd[2];                                           // wave 0 -> all: leave?, seq

// Header polls: a ring of kResPolls polls in flight, each an LDS-DMA of the header slots (lane l
// loads slots 2l, 2l + 1: 16 B, kPollLanes lanes) into its own 512-B LDS slot, reissued as soon as
// it has been looked at, so host memory is sampled every ~RTT / kResPolls. Polls land in LDS, not
// registers: no in-flight destination register can be copied or reused by the compiler, and each
// look waits only for the oldest poll (vmcnt(kResPolls - 1): kResPolls - 1 later polls were issued
// after it, other memory operations only make the wait longer). Polls may be served out of order;
// each is judged on its own stamps.
constexpr int kResPolls = 8;
constexpr int kPollLanes = (int)(kHwStop + 2) / 2;  // slots 0 .. kHwStop (| kHwStop + 1)
__shared__ __attribute__((aligned(16))) uint64_t s_ring[kResPolls][64];

__device__ __forceinline__ void poll_issue(const ResArea* area, uint32_t k, int lane) {
  if (lane < kPollLanes)
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)((const uint8_t*)area->hdr + 16 * lane),
                                     (__attribute__((address_space(3))) void*)&s_ring[k][0], 16, 0,
                                     17 /* sc0 sc1: system coherent */);
}
// this lane's slot of poll k (slots past kHwStop + 1 read as garbage: never looked at)
__device__ __forceinline__ uint64_t poll_read(uint32_t k, int lane) {
  static_assert(kResPolls == 8, "vmcnt(7) below");
  uint64_t v;
  const uint32_t a = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint64_t*)&s_ring[k][lane];
  asm volatile("s_waitcnt vmcnt(7)\n\tds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a) : "memory");
  return v;
}

// Packet bytes host -> LDS: chunk c (16 B) of the mailbox's data area to s_pkt + 16c, by LDS-DMA
// (global_load_lds_dwordx4: lane-linear LDS destination, one instruction per wave per 64
// chunks) from waves 1..3 (wave 0's first half must not wait for them); completes at the next
// fenced barrier (s_waitcnt vmcnt(0)).
// (t: the thread's index among the loading threads, a multiple of 64 of them: kResThreads - 64)
// Mailbox bytes (host memory) -> LDS, system-coherent like the polls (sc0 sc1): the same mailbox
// lines were read by earlier requests, and a cached copy must never serve a new one. (Until late
// r05 these loads were cached and relied on wave 0's `buffer_inv` before the barrier, which waves
// 1..3 could pass before the invalidation had completed: one AES open of 12 000 resident calls
// failed its tag on stale packet bytes, gpurun_out/r05zd.)
__device__ __forceinline__ void dma_chunks(const uint8_t* src, uint8_t* dst, uint32_t nch, int t) {
  const uint32_t w = (uint32_t)t >> 6, lane = (uint32_t)t & 63;
  for (uint32_t b = 64 * w; b < nch; b += kResThreads - 64)  // wave-uniform
    if (b + lane < nch)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + 16u * (b + lane)),
                                       (__attribute__((address_space(3))) void*)(dst + 16u * b), 16, 0,
                                       17 /* sc0 sc1: system coherent */);
}

// the octet of a keystream word from a quad of lanes (chacha20_block4) to all lanes: word k of
// the block is ks[k >> 2] of quad lane k & 3 (wave 0's quad 0 holds block 0: the one-time key)
__device__ __forceinline__ void otk_from_quad(const uint32_t (&ks)[4], uint32_t (&otk)[8]) {
#pragma unroll
  for (int k = 0; k < 8; ++k) otk[k] = (uint32_t)__builtin_amdgcn_readlane((int)ks[k >> 2], k & 3);
}

// 64-bit lane sums of Poly1305 limbs -> the accumulator mod 2^130 - 5 in 26-bit limbs
__device__ __forceinline__ P26 p26_from_sums(const uint64_t (&s)[5]) {
  uint64_t t[5] = {s[0], s[1], s[2], s[3], s[4]};
  for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
    for (int l = 0; l < 4; ++l) {
      t[l + 1] += t[l] >> 26;
      t[l] &= 0x3ffffff;
    }
    t[0] += (t[4] >> 26) * 5;
    t[4] &= 0x3ffffff;
  }
  P26 h;
#pragma unroll
  for (int l = 0; l < 5; ++l) h.l[l] = (uint32_t)t[l];
  return h;
}

// 64-bit sum / 32-bit XOR over the 64 lanes of a wave by DPP (quad_perm, half- and row-mirror
// within each row of 16, then the four row results by readlane): ALU latency per step, where a
// __shfl_xor ladder waits on LDS six times
template <int CTRL>
__device__ __forceinline__ uint32_t dpp32(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xf, 0xf, false);
}
template <int CTRL>
__device__ __forceinline__ uint64_t dpp64(uint64_t x) {
  return ((uint64_t)dpp32<CTRL>((uint32_t)(x >> 32)) << 32) | dpp32<CTRL>((uint32_t)x);
}
__device__ __forceinline__ uint64_t rdl64(uint64_t x, int l) {
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(x >> 32), l) << 32) |
         (uint32_t)__builtin_amdgcn_readlane((int)x, l);
}
// Sum over the wave of Poly1305 limbs (< 2^27 per lane): 32-bit DPP sums inside each row of 16
// (< 2^31), the four row sums by readlane added in 64 bits
__device__ __forceinline__ uint64_t wave_sum_limb(uint32_t x) {
  x += dpp32<0xB1>(x);   // quad_perm [1,0,3,2]
  x += dpp32<0x4E>(x);   // quad_perm [2,3,0,1]
  x += dpp32<0x141>(x);  // row_half_mirror
  x += dpp32<0x140>(x);  // row_mirror: every lane holds its row's sum
  return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)x, 0) + (uint32_t)__builtin_amdgcn_readlane((int)x, 16) +
         (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)x, 32) + (uint32_t)__builtin_amdgcn_readlane((int)x, 48);
}
__device__ __forceinline__ uint32_t wave_xor_u32(uint32_t x) {
  x ^= dpp32<0xB1>(x);
  x ^= dpp32<0x4E>(x);
  x ^= dpp32<0x141>(x);
  x ^= dpp32<0x140>(x);
  return (uint32_t)__builtin_amdgcn_readlane((int)x, 0) ^ (uint32_t)__builtin_amdgcn_readlane((int)x, 16) ^
         (uint32_t)__builtin_amdgcn_readlane((int)x, 32) ^ (uint32_t)__builtin_amdgcn_readlane((int)x, 48);
}

// h = h * m mod 2^130 - 5 for ONE wave's latency: the five column sums are independent chains
// of v_mad_u64_u32 and the carries follow, where p26_mul (the tile kernels' throughput form)
// starts each column from the previous column's carry — a 25-multiply dependent chain. Same
// bounds (column sums < 2^58).
__device__ __forceinline__ void p26_mul_lat(P26& h, const P26m& m) {
  const uint64_t h0 = h.l[0], h1 = h.l[1], h2 = h.l[2], h3 = h.l[3], h4 = h.l[4];
  const uint64_t c0 = h0 * m.r[0] + h1 * m.s[3] + h2 * m.s[2] + h3 * m.s[1] + h4 * m.s[0];
  const uint64_t c1 = h0 * m.r[1] + h1 * m.r[0] + h2 * m.s[3] + h3 * m.s[2] + h4 * m.s[1];
  const uint64_t c2 = h0 * m.r[2] + h1 * m.r[1] + h2 * m.r[0] + h3 * m.s[3] + h4 * m.s[2];
  const uint64_t c3 = h0 * m.r[3] + h1 * m.r[2] + h2 * m.r[1] + h3 * m.r[0] + h4 * m.s[3];
  const uint64_t c4 = h0 * m.r[4] + h1 * m.r[3] + h2 * m.r[2] + h3 * m.r[1] + h4 * m.r[0];
  const uint64_t d1 = c1 + (c0 >> 26), d2 = c2 + (d1 >> 26), d3 = c3 + (d2 >> 26), d4 = c4 + (d3 >> 26);
  const uint32_t k4 = (uint32_t)(d4 >> 26);
  const uint64_t t = (uint64_t)((uint32_t)c0 & 0x3ffffff) + (uint64_t)k4 * 5u;
  h.l[0] = (uint32_t)t & 0x3ffffff;
  h.l[1] = ((uint32_t)d1 & 0x3ffffff) + (uint32_t)(t >> 26);
  h.l[2] = (uint32_t)d2 & 0x3ffffff;
  h.l[3] = (uint32_t)d3 & 0x3ffffff;
  h.l[4] = (uint32_t)d4 & 0x3ffffff;
}

// Poly1305 as a 64-way interleaved Horner on ONE wave (wave 0): the powers first (they need only
// the one-time key, so they run while the other waves make the keystream), then the blocks.
// Lane j takes the blocks whose last multiplier is r^(j + 1) (blocks 64k + 63 - j - z), so the
// powers are the inclusive prefix product of r over the lanes: row_shr 1, 2, 4, 8 inside each
// row of 16, then row_bcast15 / row_bcast31 across rows (DPP; lanes without a source multiply by
// one), six multiplies with no LDS round trip.
struct PolyPow { P26m m64, mj; };  // multiplier between rounds (r^64), lane j's last (r^(j + 1))
template <int CTRL, int ROWS>
__device__ __forceinline__ P26 p26_dpp(const P26& v) {
  P26 u;
#pragma unroll
  for (int l = 0; l < 5; ++l)
    u.l[l] = (uint32_t)__builtin_amdgcn_update_dpp(l == 0 ? 1 : 0, (int)v.l[l], CTRL, ROWS, 0xf, false);
  return u;
}
template <int CTRL, int ROWS>
__device__ __forceinline__ void p26_scan_step(P26& v) {
  p26_mul_lat(v, p26_mult(p26_dpp<CTRL, ROWS>(v)));
}
__device__ __forceinline__ PolyPow poly_powers(const uint32_t (&otk)[8]) {
  P26 v = p26_from_words(otk[0] & 0x0fffffffu, otk[1] & 0x0ffffffcu, otk[2] & 0x0ffffffcu, otk[3] & 0x0ffffffcu, 0);
  p26_scan_step<0x111, 0xf>(v);  // row_shr:1
  p26_scan_step<0x112, 0xf>(v);  // row_shr:2
  p26_scan_step<0x114, 0xf>(v);  // row_shr:4
  p26_scan_step<0x118, 0xf>(v);  // row_shr:8 -> r^(j % 16 + 1)
  p26_scan_step<0x142, 0xa>(v);  // row_bcast:15 into rows 1, 3
  p26_scan_step<0x143, 0xc>(v);  // row_bcast:31 into rows 2, 3 -> r^(j + 1)
  P26 e;
#pragma unroll
  for (int l = 0; l < 5; ++l) e.l[l] = (uint32_t)__builtin_amdgcn_readlane((int)v.l[l], 63);
  return PolyPow{p26_mult(e), p26_mult(v)};
}
// the tag of AAD||pad||C||pad||lens over the LDS packet (aad at 0, ciphertext at the aligned pay)
// (seal: ksw = the keystream words in s_ks, so the MAC reads plaintext ^ keystream without waiting
// for the keystream pass over the packet; open: nullptr, the packet holds the ciphertext)
__device__ __forceinline__ void poly_tag(uint32_t aad_len, uint32_t pay, uint32_t ct_len, const PolyPow& pw,
                                         const uint32_t (&otk)[8], int lane, const uint32_t* ksw, uint32_t (&tag)[4]) {
  const LdsSpace sp{s_pkt};
  const uint32_t A = (aad_len + 15) >> 4, T = (ct_len + 15) >> 4, nb = A + T + 1;
  const uint32_t K = (nb + 63) / 64;
  const int z = (int)(64 * K) - (int)nb;
  P26 acc;
#pragma unroll
  for (int l = 0; l < 5; ++l) acc.l[l] = 0;
#pragma unroll 1
  for (uint32_t k = 0; k < K; ++k) {
    const int i = (int)(64 * k) + 63 - lane - z;
    uint32_t m[4] = {0, 0, 0, 0};
    uint32_t hib = 1;
    if (i < 0) {
      hib = 0;
    } else if (i < (int)A) {
      load_words<4>(sp, 16u * (uint32_t)i, m);
      const int rem = (int)aad_len - 16 * i;
#pragma unroll
      for (int w = 0; w < 4; ++w) m[w] &= byte_mask(rem, w);
    } else if (i < (int)(A + T)) {
      const uint32_t o = 16u * (uint32_t)(i - (int)A);
      load_words<4>(sp, pay + o, m);
      if (ksw) {
#pragma unroll
        for (int w = 0; w < 4; ++w) m[w] ^= ksw[o / 4 + w];
      }
      const int rem = (int)(ct_len - o);
#pragma unroll
      for (int w = 0; w < 4; ++w) m[w] &= byte_mask(rem, w);
    } else {
      m[0] = aad_len; m[2] = ct_len;
    }
    const P26 x = p26_from_words(m[0], m[1], m[2], m[3], hib);
#pragma unroll
    for (int l = 0; l < 5; ++l) acc.l[l] += x.l[l];
    p26_mul_lat(acc, k + 1 < K ? pw.m64 : pw.mj);
  }
  uint64_t s[5];
#pragma unroll
  for (int l = 0; l < 5; ++l) s[l] = wave_sum_limb(acc.l[l]);
  const uint32_t sk[4] = {otk[4], otk[5], otk[6], otk[7]};
  p26_finish(p26_from_sums(s), sk, tag);
}

// ChaCha20 block on a quad of lanes (RFC 8439 §2.3): lane q of the quad holds column q of the
// state (words q, 4 + q, 8 + q, 12 + q), so a column round is one quarter-round per lane and a
// diagonal round one quarter-round after rotating rows 1..3 by 1..3 lanes (quad_perm DPP) — a
// quarter of the dependent chain of a block on one lane. ks[k] = keystream word 4k + q.
__device__ __forceinline__ void chacha20_block4(const uint32_t (&key)[8], uint32_t ctr, uint32_t n0, uint32_t n1,
                                                uint32_t n2, int q, uint32_t (&ks)[4]) {
  const uint32_t c0 = q == 0 ? 0x61707865u : q == 1 ? 0x3320646eu : q == 2 ? 0x79622d32u : 0x6b206574u;
  const uint32_t k0 = q == 0 ? key[0] : q == 1 ? key[1] : q == 2 ? key[2] : key[3];
  const uint32_t k1 = q == 0 ? key[4] : q == 1 ? key[5] : q == 2 ? key[6] : key[7];
  const uint32_t d0 = q == 0 ? ctr : q == 1 ? n0 : q == 2 ? n1 : n2;
  uint32_t a = c0, b = k0, c = k1, d = d0;
#pragma unroll 2
  for (int i = 0; i < 10; ++i) {
    MQ_QR(a, b, c, d)
    // diagonals: lane q takes b of lane q+1, c of q+2, d of q+3 (quad_perm [1,2,3,0], [2,3,0,1], [3,0,1,2])
    b = dpp32<0x39>(b); c = dpp32<0x4E>(c); d = dpp32<0x93>(d);
    MQ_QR(a, b, c, d)
    b = dpp32<0x93>(b); c = dpp32<0x4E>(c); d = dpp32<0x39>(d);
  }
  ks[0] = a + c0; ks[1] = b + k0; ks[2] = c + k1; ks[3] = d + d0;
}

// GHASH(AAD || C || lens) on ONE wave (lane j: blocks 64k + j - z, multiplier H^64, final
// H^(64 - j), lanes XOR-reduced), reflected basis (mq_aes.h); tag = that ^ E_K(J0)
// (ksw: as poly_tag)
__device__ __forceinline__ void ghash_tag(uint32_t aad_len, uint32_t pay, uint32_t P, const GfOp& m64,
                                          const GfOp& ml, const uint32_t (&ej0)[4], int lane, const uint32_t* ksw,
                                          uint32_t (&tag)[4]) {
  const LdsSpace sp{s_pkt};
  const uint32_t A = (aad_len + 15) >> 4, T = (P + 15) >> 4, nb = A + T + 1;
  const uint32_t K = (nb + 63) / 64;
  const int z = (int)(64 * K) - (int)nb;
  uint32_t acc[4] = {0, 0, 0, 0};
#pragma unroll 1
  for (uint32_t k = 0; k < K; ++k) {
    const int i = (int)(64 * k) + lane - z;
    uint32_t m[4] = {0, 0, 0, 0};
    if (i >= 0 && i < (int)A) {
      load_words<4>(sp, 16u * (uint32_t)i, m);
      const int rem = (int)aad_len - 16 * i;
#pragma unroll
      for (int w = 0; w < 4; ++w) m[w] = refl(m[w] & byte_mask(rem, w));
    } else if (i >= (int)A && i < (int)(A + T)) {
      const uint32_t o = 16u * (uint32_t)(i - (int)A);
      load_words<4>(sp, pay + o, m);
      if (ksw) {
#pragma unroll
        for (int w = 0; w < 4; ++w) m[w] ^= ksw[o / 4 + w];
      }
      const int rem = (int)(P - o);
#pragma unroll
      for (int w = 0; w < 4; ++w) m[w] = refl(m[w] & byte_mask(rem, w));
    } else if (i == (int)(A + T)) {
      const uint64_t ab = (uint64_t)aad_len * 8, cb = (uint64_t)P * 8;
      m[0] = brev((uint32_t)(ab >> 32)); m[1] = brev((uint32_t)ab);
      m[2] = brev((uint32_t)(cb >> 32)); m[3] = brev((uint32_t)cb);
    }
#pragma unroll
    for (int w = 0; w < 4; ++w) acc[w] ^= m[w];
    gf_mul(acc, k + 1 < K ? m64 : ml);
  }
#pragma unroll
  for (int w = 0; w < 4; ++w) tag[w] = bswap32(brev(wave_xor_u32(acc[w]))) ^ ej0[w];
}

// Stamps of a request's phases on wave 0 (ResCtl::phase): first half done, packet landed, second
// half done, decryption applied
struct ResT { uint64_t half1, landed, half2, applied; };

// the keystream pass of a request (waves 1..3): pw ^= s_ks over the P payload bytes
__device__ __forceinline__ void apply_ks(uint32_t* pw, uint32_t P, int t, int nt) {
  for (uint32_t w = (uint32_t)t; 4 * w < P; w += (uint32_t)nt) pw[w] ^= s_ks[w] & byte_mask((int)(P - 4 * w), 0);
}

// ChaCha20-Poly1305 seal / open of the LDS packet (aad at 0, body at the aligned pay). First half
// (header only, while the packet lands): wave 0 makes the Poly1305 key (block 0, on its quads) and
// the MAC's powers of r; waves 1..3 write keystream blocks 1.. to s_ks (one per quad, 48 per pass).
// Second half: seal runs the MAC (wave 0) over plaintext ^ s_ks and stores the tag, and its
// write-back applies s_ks (no pass over the packet, no barrier); open runs the MAC over the untouched ciphertext, verifies,
// and applies s_ks only if the tag matched. Returns MQ_* (workgroup-uniform).
__device__ int res_chacha(bool open, uint32_t aad_len, uint32_t pay, uint32_t body_len, int tid, ResT& t) {
  uint32_t key[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) key[k] = s_hdr[kHwKey + k];
  const uint32_t n0 = s_hdr[kHwNonce], n1 = s_hdr[kHwNonce + 1], n2 = s_hdr[kHwNonce + 2];
  const uint32_t P = open ? body_len - 16 : body_len;
  const uint32_t nblk = 1 + (P + 63) / 64;
  const int q = tid & 3;
  uint32_t* pw = (uint32_t*)(s_pkt + pay);
  constexpr uint32_t kQuads = (kResThreads - 64) / 4;
  uint32_t otk[8];
  PolyPow pp;
  if (tid < 64) {
    uint32_t ks[4];
    chacha20_block4(key, 0, n0, n1, n2, q, ks);
    otk_from_quad(ks, otk);
    pp = poly_powers(otk);
  } else {
#pragma unroll 1
    for (uint32_t b0 = 1; b0 < nblk; b0 += kQuads) {
      uint32_t ks[4];
      const uint32_t b = b0 + (uint32_t)((tid - 64) >> 2);
      chacha20_block4(key, b, n0, n1, n2, q, ks);
      if (b < nblk) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint32_t o = 64 * (b - 1) + 16 * k + 4 * q;  // payload byte offset of word 4k + q
          if (o < P) s_ks[o / 4] = ks[k];
        }
      }
    }
  }
  t.half1 = wall_clock64();
  __syncthreads();  // the packet has landed (vmcnt(0)); s_ks complete
  t.landed = wall_clock64();
  if (!open) {  // the packet keeps its plaintext: the write-back (wave 0) applies s_ks
    if (tid < 64) {
      uint32_t tag[4];
      poly_tag(aad_len, pay, P, pp, otk, tid, s_ks, tag);
      if (tid == 0) store_words<4>(LdsSpace{s_pkt}, pay + P, tag);
    }
    t.half2 = t.applied = wall_clock64();
    return MQ_OK;
  }
  if (tid < 64) {
    uint32_t tag[4], got[4];
    poly_tag(aad_len, pay, P, pp, otk, tid, nullptr, tag);
    load_words<4>(LdsSpace{s_pkt}, pay + P, got);
    if (tid == 0) s_scr[12] = (tag[0] ^ got[0]) | (tag[1] ^ got[1]) | (tag[2] ^ got[2]) | (tag[3] ^ got[3]);
  }
  __syncthreads();
  t.half2 = wall_clock64();
  if (s_scr[12]) return MQ_ERR_CRYPTO;  // rustcrypto.rs:156-163; nothing decrypted
  apply_ks(pw, P, tid, kResThreads);
  __syncthreads();
  t.applied = wall_clock64();
  return MQ_OK;
}

// AES-128-GCM seal / open of the LDS packet. First half: wave 0 makes E_K(J0), then — once the
// GHASH powers it loaded itself have landed — the GHASH multipliers (H^64, and H^(64 - lane));
// waves 1..3 write CTR blocks (one per thread, 192 per pass) to s_ks. Second half: as res_chacha.
__device__ int res_aes(bool open, uint32_t aad_len, uint32_t pay, uint32_t body_len, int tid, ResT& t) {
  const TwLane L = tw_lane();
  const RkLds key{s_hdr + kHwKey};
  const uint32_t nb0 = bswap32(s_hdr[kHwNonce]), nb1 = bswap32(s_hdr[kHwNonce + 1]), nb2 = bswap32(s_hdr[kHwNonce + 2]);
  const uint32_t P = open ? body_len - 16 : body_len;
  const uint32_t nblk = 1 + (P + 15) / 16;  // slot 0: E_K(J0), slot b >= 1: CTR block with counter b + 1
  uint32_t* pw = (uint32_t*)(s_pkt + pay);
  constexpr uint32_t kBlk = kResThreads - 64;
  uint32_t ej0[4];
  GfOp m64, ml;
  if (tid < 64) {
    uint32_t s[4] = {nb0, nb1, nb2, 1u};
    aes128_enc(key, L, s);
#pragma unroll
    for (int w = 0; w < 4; ++w) ej0[w] = bswap32(s[w]);
    // wave 0's only LDS-DMA is the GHASH powers (the packet is waves 1..3's): wait for it alone
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    uint32_t h[4], hl[4];
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      h[w] = brev(s_hpow[4 * 63 + w]);
      hl[w] = brev(s_hpow[4 * (63 - tid) + w]);
    }
    m64 = gf_prepare(h);
    ml = gf_prepare(hl);
  } else {
#pragma unroll 1
    for (uint32_t b0 = 1; b0 < nblk; b0 += kBlk) {
      const uint32_t b = b0 + (uint32_t)(tid - 64);
      uint32_t s[4] = {nb0, nb1, nb2, b + 1};
      aes128_enc(key, L, s);
      if (b < nblk) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint32_t o = 16 * (b - 1) + 4 * k;
          if (o < P) s_ks[o / 4] = bswap32(s[k]);
        }
      }
    }
  }
  t.half1 = wall_clock64();
  __syncthreads();  // the packet has landed; s_ks complete
  t.landed = wall_clock64();
  if (!open) {  // the packet keeps its plaintext: the write-back (wave 0) applies s_ks
    if (tid < 64) {
      uint32_t tag[4];
      ghash_tag(aad_len, pay, P, m64, ml, ej0, tid, s_ks, tag);
      if (tid == 0) store_words<4>(LdsSpace{s_pkt}, pay + P, tag);
    }
    t.half2 = t.applied = wall_clock64();
    return MQ_OK;
  }
  if (tid < 64) {
    uint32_t tag[4], got[4];
    ghash_tag(aad_len, pay, P, m64, ml, ej0, tid, nullptr, tag);
    load_words<4>(LdsSpace{s_pkt}, pay + P, got);
    if (tid == 0) s_scr[12] = (tag[0] ^ got[0]) | (tag[1] ^ got[1]) | (tag[2] ^ got[2]) | (tag[3] ^ got[3]);
  }
  __syncthreads();
  t.half2 = wall_clock64();
  if (s_scr[12]) return MQ_ERR_CRYPTO;  // rustcrypto.rs:85-91; nothing decrypted
  apply_ks(pw, P, tid, kResThreads);
  __syncthreads();
  t.applied = wall_clock64();
  return MQ_OK;
}

// HeaderProtection::mask from the header alone (sample and HP key material), wave 0
__device__ void res_hp(uint32_t suite, uint32_t& m0, uint32_t& m1) {
  const uint32_t smp[4] = {s_hdr[kHwSample], s_hdr[kHwSample + 1], s_hdr[kHwSample + 2], s_hdr[kHwSample + 3]};
  if (suite == MQ_SUITE_CHACHA20) {  // rustcrypto.rs:197-220
    uint32_t hk[8], blk[16];
#pragma unroll
    for (int k = 0; k < 8; ++k) hk[k] = s_hdr[kHwKey + k];
    chacha20_block(hk, smp[0], smp[1], smp[2], smp[3], blk);
    m0 = blk[0];
    m1 = blk[1] & 0xffu;
  } else {  // rustcrypto.rs:175-186
    uint32_t s[4] = {bswap32(smp[0]), bswap32(smp[1]), bswap32(smp[2]), bswap32(smp[3])};
    aes128_enc(RkLds{s_hdr + kHwKey}, tw_lane(), s);
    m0 = bswap32(s[0]);
    m1 = s[1] >> 24;
  }
}

}  // namespace mq

using namespace mq;

extern "C" __global__ __launch_bounds__(kResThreads) void mq_resident_kernel(ResArea* area, uint64_t idle_ticks,
                                                                             uint64_t life_ticks) {
  const int tid = (int)threadIdx.x, lane = tid & 63;
  const bool w0 = tid < 64;
  ResCtl* ctl = &area->ctl;
  build_tw(tid, kResThreads);  // the wide AES T-table, once per kernel
  __syncthreads();
  uint32_t done = uni(ld_sys_sc(&ctl->done));
  const uint64_t t0 = wall_clock64();
  uint64_t t_last = t0, t_seen = t0;
  const bool w0u = wave_id() == 0;  // wave-uniform: a scalar branch around the poll loop
  // wave 0's polls: kept in flight across loop iterations (and the request, see the end of the loop)
  uint32_t pos = 0;  // the ring's oldest poll (wave 0)
  if (w0u) {
#pragma unroll
    for (uint32_t k = 0; k < kResPolls; ++k) {
      poll_issue(area, k, lane);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_sleep(10);  // ~0.3 us apart
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  for (;;) {
    if (w0u) {  // wave 0 polls; waves 1..3 wait at the barrier below
      // A new request is one whose slot 0 carries another number than the last one served (`done`),
      // and it is complete when every slot it uses carries that number (the host writes slot 0
      // last, so a complete header usually comes in the first poll that sees slot 0). Any number
      // other than `done` is served, not just done + 1: a request the host gave up on (its 10-s
      // limit) is then simply superseded by the next one (r03 waited for done + 1 and never served
      // another request after such a timeout).
      uint32_t exp = done;
      uint32_t leave = 0;
      uint64_t hv = 0;
      // 0: nothing new, 1: a new request (slot 0), 2: stop, 3: idle
      auto test = [&](uint64_t v) -> uint32_t {
        if (__builtin_amdgcn_readlane((int)(uint32_t)v, kHwStop)) return 2;
        const uint32_t s0 = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), 0);
        if (s0 != done) {
          exp = s0;
          return 1;
        }
        return 0;
      };
      for (;;) {
        const uint64_t deadline = min(t_last + idle_ticks, t0 + life_ticks);
        uint32_t r = 0;
        do {
          hv = poll_read(pos, lane);
          r = test(hv);
          poll_issue(area, pos, lane);
          pos = (pos + 1) % kResPolls;
          if (!r && wall_clock64() > deadline) r = 3;
        } while (!r);
        const uint64_t now = wall_clock64();
        if (r == 2) { leave = 1; break; }
        if (r == 1) {
          const uint32_t n = res_hdr_words(((uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)hv, 0) >> 8) & 0xffu);
          if (!wave_any((uint32_t)lane < n && (uint32_t)(hv >> 32) != exp)) { t_seen = now; break; }
          t_last = now;  // a request is being written: no idle exit meanwhile
          continue;
        }
        // idle: claim the exit, then look once more; a request posted meanwhile is served first
        if (lane == 0) st_sys_sc(&ctl->state, kResExiting);
        wave_sync();
        if (uni(ld_sys_sc((const uint32_t*)&area->hdr[0] + 1)) == done) { leave = 1; break; }
        if (lane == 0) st_sys_sc(&ctl->state, kResRunning);
        t_last = now;
      }
      if (!leave) s_hdr[lane] = (uint32_t)hv;
      if (lane == 0) { s_cmd[0] = leave; s_cmd[1] = exp; }
      // The packet was written before the header; its loads are issued after this wave has seen the
      // header (they cannot pass it). Invalidate the vector caches for them, without a fence: a
      // system-scope acquire fence would wait for the ring's polls in flight (vmcnt(0)), up to a
      // round trip.
      asm volatile("buffer_inv sc0 sc1" ::: "memory");
    }
    // LDS-only barrier (the other waves' view of s_hdr / s_cmd): a __syncthreads() fence would also
    // wait for wave 0's polls in flight
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (s_cmd[0]) break;
    const uint32_t seq = s_cmd[1];
    const uint64_t t_hdr = wall_clock64();
    const uint32_t h0 = uni(s_hdr[kHwOp]), op = h0 & 0xffu, suite = (h0 >> 8) & 0xffu;
    const uint32_t aad_len = uni(s_hdr[kHwAad]), body_len = uni(s_hdr[kHwBody]), pay = uni(s_hdr[kHwPay]);
    const uint32_t tot = op == kResHp ? 0u : pay + body_len + (op == kResSeal ? 16u : 0u);
    const uint32_t nch = (tot + 15) / 16;
    const bool known = suite == MQ_SUITE_CHACHA20 || suite == MQ_SUITE_AES128GCM;
    const bool bad = !known || op > kResHp ||
                     (op != kResHp && (pay < aad_len || pay > aad_len + 15 || (pay & 15) || tot > kResMaxPkt ||
                                       (op == kResOpen && body_len < 16)));
    // the packet (and the GHASH powers) host -> LDS, landing during the first half
    if (!bad && op != kResHp) {
      if (!w0) dma_chunks(area->data, s_pkt, nch, tid - 64);  // waves 1..3: the packet
      else if (suite == MQ_SUITE_AES128GCM) dma_chunks((const uint8_t*)area->Hpow, (uint8_t*)s_hpow, 64, tid);
    }
    ResT t{t_hdr, t_hdr, t_hdr, t_hdr};
    int st = MQ_OK;
    uint32_t m0 = 0, m1 = 0;
    if (bad) {
      st = MQ_ERR_INVALID_ARG;  // the host checks these; never trust the mailbox
    } else if (op == kResHp) {
      if (w0) res_hp(suite, m0, m1);
      t.half1 = t.landed = t.half2 = t.applied = wall_clock64();
    } else if (suite == MQ_SUITE_CHACHA20) {
      st = res_chacha(op == kResOpen, aad_len, pay, body_len, tid, t);
    } else {
      st = res_aes(op == kResOpen, aad_len, pay, body_len, tid, t);
    }
    // The body back, by wave 0 alone (failed opens are not copied): its system-scope release
    // fence then orders every store before `done`. Waves 1..3 go on to the next barrier, which
    // wave 0 reaches only after this, so nothing overwrites the LDS packet meanwhile.
    if (!w0) continue;
    if (st == MQ_OK && op != kResHp) {
      uint4* dst = (uint4*)area->data;
      const uint32_t P = op == kResSeal ? body_len : 0u;  // seal: payload words still plaintext
#pragma unroll 1
      for (uint32_t c = pay / 16 + (uint32_t)lane; c < nch; c += 64) {
        uint4 v = *(const uint4*)(s_pkt + 16 * c);
        const uint32_t w0 = 4 * c - pay / 4;  // payload word of v.x (pay is 16-B aligned)
        if (4 * w0 + 16 <= P) {  // a whole payload chunk
          const uint4 k = *(const uint4*)(s_ks + w0);
          v.x ^= k.x; v.y ^= k.y; v.z ^= k.z; v.w ^= k.w;
        } else if (4 * w0 < P) {
          v.x ^= s_ks[w0] & byte_mask((int)(P - 4 * w0), 0);
          v.y ^= s_ks[w0 + 1] & byte_mask((int)(P - 4 * w0), 1);
          v.z ^= s_ks[w0 + 2] & byte_mask((int)(P - 4 * w0), 2);
          v.w ^= s_ks[w0 + 3] & byte_mask((int)(P - 4 * w0), 3);
        }
        dst[c] = v;
      }
    }
    const uint64_t t_wb = wall_clock64();
    if (tid == 0) {  // diagnostic stamps: they may land after `done`
      static_assert(kResPhases == 6, "phase stamps");
      st_sys(&ctl->phase[0], (uint32_t)(t_hdr - t_seen));
      st_sys(&ctl->phase[1], (uint32_t)(t.half1 - t_hdr));
      st_sys(&ctl->phase[2], (uint32_t)(t.landed - t.half1));
      st_sys(&ctl->phase[3], (uint32_t)(t.half2 - t.landed));
      st_sys(&ctl->phase[4], (uint32_t)(t.applied - t.half2));
      st_sys(&ctl->phase[5], (uint32_t)(t_wb - t.applied));
    }
    // system scope: the body before `done` — only when there is one: the fence waits for every
    // load in flight too (vmcnt counts stores and loads on gfx950), and after a mask (no packet,
    // no fenced barrier) the polls reissued at the hit are still in flight
    if (st == MQ_OK && op != kResHp) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    if (tid == 0) {  // done, status and the mask in one 16-B store
      typedef uint32_t v4u __attribute__((ext_vector_type(4)));
      const v4u out = {seq, (uint32_t)st, m0, m1};
      asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(&ctl->done), "v"(out) : "memory");
    }
    done = seq;
    t_last = wall_clock64();

  }
  __builtin_amdgcn_s_waitcnt(0);  // the ring's polls land before the wave ends
  if (tid == 0) st_sys_sc(&ctl->state, kResExited);
}

// ---- host ------------------------------------------------------------------------------------------
namespace {

struct Resident {
  int dev = -1;
  ResArea* host = nullptr;  // pinned, coherent, mapped
  ResArea* dptr = nullptr;
  hipStream_t stream = nullptr;
  uint32_t seq = 0;
  uint64_t hpow_uid = 0;  // the context whose GHASH powers the mailbox holds (0: none)
  bool launched = false;
  uint64_t idle = 0, life = 0;
  int khz = 100000;  // wall-clock rate
  uint32_t host_ns[3] = {0, 0, 0};  // last call: request written, waited for done, result copied
  std::vector<ResArea*> abandoned;  // mailboxes given up on a wedged kernel (still told to stop at exit)
  std::mutex mu;
};

// A device's servers (r05): kResLanes independent mailboxes, each with its own
// resident workgroup, so up to that many threads' per-packet calls run at once instead of one at
// a time behind one mutex. A lane's kernel holds one CU while it lives (it leaves after 2 ms
// without a call), so a device busy with per-packet calls from T threads holds min(T, lanes) CUs.
// MQ_RESIDENT_LANES (read once, 1..16) sets the count.
struct ResidentSet {
  std::vector<Resident*> lanes;
  std::atomic<uint32_t> last{0};  // the lane of the latest completed call (mq_resident_phases)
};
std::mutex g_res_mu;
std::vector<ResidentSet*> g_res;  // per device; never freed (the kernels may outlive static destructors)

uint32_t resident_lanes() {
  static const uint32_t k = [] {
    const char* e = std::getenv("MQ_RESIDENT_LANES");
    const unsigned long v = e ? std::strtoul(e, nullptr, 10) : 4ul;
    return (uint32_t)(v < 1 ? 1 : v > 16 ? 16 : v);
  }();
  return k;
}

void stop_all() {  // atexit: ask every resident kernel to leave (plain stores, no HIP call)
  for (ResidentSet* set : g_res) {
    if (!set) continue;
    for (Resident* r : set->lanes) {
      if (r->host) __atomic_store_n(&r->host->hdr[kHwStop], (uint64_t)1, __ATOMIC_SEQ_CST);
      for (ResArea* x : r->abandoned) __atomic_store_n(&x->hdr[kHwStop], (uint64_t)1, __ATOMIC_SEQ_CST);
    }
  }
}

ResidentSet* resident_set(int dev) {
  std::lock_guard<std::mutex> lk(g_res_mu);
  if ((size_t)dev >= g_res.size()) g_res.resize((size_t)dev + 1, nullptr);
  if (!g_res[(size_t)dev]) {
    static bool hooked = false;
    if (!hooked) {
      hooked = true;
      std::atexit(stop_all);
    }
    ResidentSet* set = new ResidentSet();
    for (uint32_t k = 0; k < resident_lanes(); ++k) {
      set->lanes.push_back(new Resident());
      set->lanes.back()->dev = dev;
    }
    g_res[(size_t)dev] = set;
  }
  return g_res[(size_t)dev];
}

uint32_t load_acq(const uint32_t* p) { return __atomic_load_n(p, __ATOMIC_ACQUIRE); }

// How long a call waits for the resident kernel: 10 s, or MQ_RESIDENT_TIMEOUT_US (mq_opts.h;
// tests force the timeout path with it)
std::chrono::microseconds resident_timeout() {
  const long v = opt(Opt::ResidentTimeoutUs);
  return std::chrono::microseconds(v >= 0 ? (unsigned long long)v : 10000000ull);
}

}  // namespace

// One call through the resident kernel of device `dev` (the caller holds a device guard on it).
// `q` is the context's request image with op, lengths and nonce / sample filled in; `uid`
// identifies the context (its GHASH powers are copied only when another context used the mailbox
// last); aad and body are the packet bytes. Returns MQ_OK when the call was served (*status = its
// result, out[0, out_len) = bytes [out_off, out_off + out_len) of the processed body when *status
// is MQ_OK, mask = the header-protection mask words), else an MQ_ERR_* of the transport.
int mq_resident_call(int dev, const ResReq& q, uint64_t uid, const uint8_t* aad, const uint8_t* body, uint8_t* out,
                     size_t out_off, size_t out_len, int* status, uint32_t* mask) {
  // a free lane, trying the thread's own first (a thread keeps its lane, and with it its context's
  // GHASH powers in the mailbox, while no other thread takes it); all busy: wait for the own lane
  ResidentSet* set = resident_set(dev);
  const uint32_t K = (uint32_t)set->lanes.size();
  const uint32_t home = (uint32_t)(std::hash<std::thread::id>()(std::this_thread::get_id()) % K);
  Resident* r = nullptr;
  uint32_t lane = home;
  std::unique_lock<std::mutex> lk;
  for (uint32_t k = 0; k < K && !r; ++k) {
    Resident* c = set->lanes[(home + k) % K];
    std::unique_lock<std::mutex> t(c->mu, std::try_to_lock);
    if (t.owns_lock()) {
      r = c;
      lane = (home + k) % K;
      lk = std::move(t);
    }
  }
  if (!r) {
    r = set->lanes[home];
    lk = std::unique_lock<std::mutex>(r->mu);
  }
  if (!r->host) {
    if (hipHostMalloc((void**)&r->host, sizeof(ResArea), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
      r->host = nullptr;
      return MQ_ERR_HIP;
    }
    std::memset(r->host, 0, sizeof(ResArea));
    if (hipHostGetDevicePointer((void**)&r->dptr, r->host, 0) != hipSuccess ||
        hipStreamCreateWithFlags(&r->stream, hipStreamNonBlocking) != hipSuccess)
      return MQ_ERR_HIP;
    int khz = 0;
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz <= 0) khz = 100000;
    r->khz = khz;
    const char* e = std::getenv("MQ_RESIDENT_IDLE_US");
    const uint64_t idle_us = e ? (uint64_t)std::strtoull(e, nullptr, 10) : 2000;  // 2 ms without a call
    r->idle = idle_us * (uint64_t)khz / 1000;
    r->life = 10ull * 1000 * (uint64_t)khz;  // 10 s, then leave at the next idle moment
  }
  const auto h0 = std::chrono::steady_clock::now();
  ResArea* a = r->host;
  const uint32_t pay = (q.aad_len + 15) & ~15u;  // the body 16-B aligned (mq_resident.h)
  const bool aead = q.op != kResHp;
  if (aead && (size_t)pay + q.body_len + 16 > kResMaxPkt) return MQ_ERR_INVALID_ARG;
  // the packet, and for an AES-128-GCM AEAD call the context's GHASH powers, before the header
  if (aead) {
    if (q.aad_len) std::memcpy(a->data, aad, q.aad_len);
    if (q.body_len) std::memcpy(a->data + pay, body, q.body_len);
    if (q.suite == MQ_SUITE_AES128GCM && r->hpow_uid != uid) {
      std::memcpy(a->Hpow, q.Hpow, sizeof a->Hpow);
      r->hpow_uid = uid;
    }
  }
  uint32_t w[kResHdrSlots];
  const uint32_t n = res_hdr_words(q.suite);
  w[kHwOp] = q.op | q.suite << 8;
  w[kHwAad] = q.aad_len;
  w[kHwBody] = q.body_len;
  w[kHwPay] = pay;
  for (int i = 0; i < 3; ++i) w[kHwNonce + i] = q.nonce[i];
  w[kHwNonce + 3] = 0;
  for (int i = 0; i < 4; ++i) w[kHwSample + i] = q.sample[i];
  if (q.suite == MQ_SUITE_AES128GCM) std::memcpy(w + kHwKey, aead ? q.aes_rk : q.hp_rk, 44 * 4);
  else std::memcpy(w + kHwKey, aead ? q.key : q.hp, 8 * 4);
  const uint32_t seq = ++r->seq;
  // slots 1 .. n-1, then slot 0: each one 8-B store (never torn), stores in program order (x86-64)
  for (uint32_t i = 1; i < n; ++i)
    __atomic_store_n(&a->hdr[i], (uint64_t)w[i] | (uint64_t)seq << 32, __ATOMIC_RELAXED);
  __atomic_store_n(&a->hdr[0], (uint64_t)w[0] | (uint64_t)seq << 32, __ATOMIC_SEQ_CST);
  const auto t0 = std::chrono::steady_clock::now();
  bool relaunched = false;
  for (uint32_t spins = 0;; ++spins) {
    if (load_acq(&a->ctl.done) == seq) break;
    if (!r->launched || __atomic_load_n(&a->ctl.state, __ATOMIC_SEQ_CST) == kResExited) {
      if (r->launched && hipStreamSynchronize(r->stream) != hipSuccess) return MQ_ERR_HIP;  // it has left
      if (load_acq(&a->ctl.done) == seq) break;  // served on its way out
      __atomic_store_n(&a->ctl.state, (uint32_t)kResRunning, __ATOMIC_SEQ_CST);
      __atomic_store_n(&a->hdr[kHwStop], (uint64_t)0, __ATOMIC_SEQ_CST);
      hipLaunchKernelGGL(mq_resident_kernel, dim3(1), dim3(kResThreads), 0, r->stream, r->dptr, r->idle, r->life);
      if (hipGetLastError() != hipSuccess) {
        __atomic_store_n(&a->ctl.state, (uint32_t)kResExited, __ATOMIC_SEQ_CST);
        return MQ_ERR_HIP;
      }
      r->launched = true;
      relaunched = true;
    }
    if ((spins & 1023) == 1023 && std::chrono::steady_clock::now() - t0 > resident_timeout()) {
      // Give up on this request, but leave no kernel behind that could still serve it (it would
      // write the mailbox while the next call fills it): ask the kernel to leave and
      // wait for its stream. A kernel not yet placed (every CU busy) starts, sees the stop slot and
      // leaves. If it served the request meanwhile, the call succeeds after all.
      __atomic_store_n(&a->hdr[kHwStop], (uint64_t)1, __ATOMIC_SEQ_CST);
      // The wait for the kernel to leave is bounded too: a kernel that cannot be
      // placed or is wedged would otherwise block this call forever. Past a second deadline the
      // mailbox is abandoned (poisoned): the old area and stream are left to that kernel, and the
      // next call starts over with a fresh area, stream and kernel.
      if (r->launched) {
        const auto t_stop = std::chrono::steady_clock::now();
        hipError_t q = hipErrorNotReady;
        while ((q = hipStreamQuery(r->stream)) == hipErrorNotReady &&
               std::chrono::steady_clock::now() - t_stop < resident_timeout())
          std::this_thread::yield();
        if (q == hipErrorNotReady) {
          r->abandoned.push_back(r->host);  // never freed: the kernel may still write it
          r->host = nullptr;
          r->dptr = nullptr;
          r->stream = nullptr;
          r->launched = false;
          r->seq = 0;
          r->hpow_uid = 0;
          return MQ_ERR_HIP;
        }
        if (q != hipSuccess) return MQ_ERR_HIP;
      }
      if (load_acq(&a->ctl.done) == seq) break;
      return MQ_ERR_HIP;  // the next call relaunches (state: exited) and supersedes this request
    }
  }
  const auto t1 = std::chrono::steady_clock::now();
  *status = (int)__atomic_load_n(&a->ctl.status, __ATOMIC_ACQUIRE);
  if (mask) {
    mask[0] = a->ctl.mask0;
    mask[1] = a->ctl.mask1;
  }
  if (*status == MQ_OK && out_len) std::memcpy(out, a->data + pay + out_off, out_len);
  const auto t2 = std::chrono::steady_clock::now();
  auto ns = [](std::chrono::steady_clock::duration d) {
    return (uint32_t)std::chrono::duration_cast<std::chrono::nanoseconds>(d).count();
  };
  r->host_ns[0] = ns(t0 - h0);
  r->host_ns[1] = relaunched ? 0u : ns(t1 - t0);
  r->host_ns[2] = ns(t2 - t1);
  set->last.store(lane, std::memory_order_relaxed);
  return MQ_OK;
}

// The device-side phases of device dev's last resident call in nanoseconds (ResCtl::phase), then
// the host's (request written, waited for done, result copied); returns the number written, 0
// before any call.
extern "C" int mq_resident_phases(int dev, uint32_t* ns, int n) {
  if (dev < 0 || !ns || n <= 0) return 0;
  ResidentSet* set = resident_set(dev);
  Resident* r = set->lanes[set->last.load(std::memory_order_relaxed) % set->lanes.size()];
  std::lock_guard<std::mutex> lk(r->mu);
  if (!r->host || !r->seq) return 0;
  int m = 0;
  for (; m < n && m < kResPhases; ++m)
    ns[m] = (uint32_t)((uint64_t)__atomic_load_n(&r->host->ctl.phase[m], __ATOMIC_ACQUIRE) * 1000000ull / (uint64_t)r->khz);
  for (int k = 0; m < n && k < 3; ++k, ++m) ns[m] = r->host_ns[k];
  return m;
}
