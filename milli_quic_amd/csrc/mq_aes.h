// mq_aes.h — AES-128 and GF(2^128) building blocks for gfx950 without AES / carry-less-multiply
// instructions, shared by the AES-128-GCM packet kernels (mq_aes.hip) and the batched Initial key
// derivation (mq_derive.hip):
//   * AES-128 rounds from T-tables in LDS (FIPS-197 §5.1). The packet tile kernels use a wide
//     table (T0 and T2 = ror(T0, 16), 32 replicas each, 64 KiB): one v_perm_b32 forms each
//     lookup address, every ds_read_b32 is bank-conflict-free, and a round column needs one
//     rotation. The one-block-per-lane kernels (HP pre-pass, key derivation) keep a small table
//     (T0 only, 8 replicas, 8 KiB) because they run too few rounds per workgroup to pay for more;
//   * GHASH multiplies by H^8 in the single-key tile kernels go through an LDS table of
//     (u x^(8q)) * H^8 for every byte position q and value u (64 KiB): 16 ds_read_b128 and XORs
//     per multiply, no reduction (r03; a nibble table of 8 KiB took 32 of each);
//   * GHASH multiplies in the bit-reflected polynomial basis with 32x32 carry-less products built
//     from integer v_mad_u64_u32 on bit-holed operands (4-bit spacing, <= 8 terms per output
//     position, so no carry reaches the next kept bit), Karatsuba 128 -> 64 -> 32 (9 products per
//     multiply), then the x^128 + x^7 + x^2 + x + 1 fold (SP 800-38D §6.3).
#pragma once
#include "mq_device.h"

namespace mq {

// FIPS-197 S-box (data table), used once per workgroup to build T0 in LDS.
__constant__ uint8_t kSbox[256] = {
    0x63, 0x7c, 0x77, 0x7b, 0xf2, 0x6b, 0x6f, 0xc5, 0x30, 0x01, 0x67, 0x2b, 0xfe, 0xd7, 0xab, 0x76,
    0xca, 0x82, 0xc9, 0x7d, 0xfa, 0x59, 0x47, 0xf0, 0xad, 0xd4, 0xa2, 0xaf, 0x9c, 0xa4, 0x72, 0xc0,
    0xb7, 0xfd, 0x93, 0x26, 0x36, 0x3f, 0xf7, 0xcc, 0x34, 0xa5, 0xe5, 0xf1, 0x71, 0xd8, 0x31, 0x15,
    0x04, 0xc7, 0x23, 0xc3, 0x18, 0x96, 0x05, 0x9a, 0x07, 0x12, 0x80, 0xe2, 0xeb, 0x27, 0xb2, 0x75,
    0x09, 0x83, 0x2c, 0x1a, 0x1b, 0x6e, 0x5a, 0xa0, 0x52, 0x3b, 0xd6, 0xb3, 0x29, 0xe3, 0x2f, 0x84,
    0x53, 0xd1, 0x00, 0xed, 0x20, 0xfc, 0xb1, 0x5b, 0x6a, 0xcb, 0xbe, 0x39, 0x4a, 0x4c, 0x58, 0xcf,
    0xd0, 0xef, 0xaa, 0xfb, 0x43, 0x4d, 0x33, 0x85, 0x45, 0xf9, 0x02, 0x7f, 0x50, 0x3c, 0x9f, 0xa8,
    0x51, 0xa3, 0x40, 0x8f, 0x92, 0x9d, 0x38, 0xf5, 0xbc, 0xb6, 0xda, 0x21, 0x10, 0xff, 0xf3, 0xd2,
    0xcd, 0x0c, 0x13, 0xec, 0x5f, 0x97, 0x44, 0x17, 0xc4, 0xa7, 0x7e, 0x3d, 0x64, 0x5d, 0x19, 0x73,
    0x60, 0x81, 0x4f, 0xdc, 0x22, 0x2a, 0x90, 0x88, 0x46, 0xee, 0xb8, 0x14, 0xde, 0x5e, 0x0b, 0xdb,
    0xe0, 0x32, 0x3a, 0x0a, 0x49, 0x06, 0x24, 0x5c, 0xc2, 0xd3, 0xac, 0x62, 0x91, 0x95, 0xe4, 0x79,
    0xe7, 0xc8, 0x37, 0x6d, 0x8d, 0xd5, 0x4e, 0xa9, 0x6c, 0x56, 0xf4, 0xea, 0x65, 0x7a, 0xae, 0x08,
    0xba, 0x78, 0x25, 0x2e, 0x1c, 0xa6, 0xb4, 0xc6, 0xe8, 0xdd, 0x74, 0x1f, 0x4b, 0xbd, 0x8b, 0x8a,
    0x70, 0x3e, 0xb5, 0x66, 0x48, 0x03, 0xf6, 0x0e, 0x61, 0x35, 0x57, 0xb9, 0x86, 0xc1, 0x1d, 0x9e,
    0xe1, 0xf8, 0x98, 0x11, 0x69, 0xd9, 0x8e, 0x94, 0x9b, 0x1e, 0x87, 0xe9, 0xce, 0x55, 0x28, 0xdf,
    0x8c, 0xa1, 0x89, 0x0d, 0xbf, 0xe6, 0x42, 0x68, 0x41, 0x99, 0x2d, 0x0f, 0xb0, 0x54, 0xbb, 0x16};

constexpr int kTReplicas = 8;
__shared__ uint32_t g_t0[256 * kTReplicas];

__device__ __forceinline__ void build_t0(int tid, int nthreads) {
  for (int e = tid; e < 256 * kTReplicas; e += nthreads) {
    const uint32_t s = kSbox[e / kTReplicas];
    const uint32_t s2 = ((s << 1) ^ ((s & 0x80) ? 0x11b : 0)) & 0xff;
    g_t0[e] = (s2 << 24) | (s << 16) | (s << 8) | (s2 ^ s);
  }
}

__device__ __forceinline__ uint32_t ror(uint32_t x, int r) { return (x >> r) | (x << (32 - r)); }

struct AesRk { uint32_t w[44]; };

__device__ __forceinline__ void load_rk(const uint32_t* src, AesRk& rk) {
#pragma unroll
  for (int i = 0; i < 11; ++i) {
    const uint4 v = *(const uint4*)(src + 4 * i);
    rk.w[4 * i] = v.x; rk.w[4 * i + 1] = v.y; rk.w[4 * i + 2] = v.z; rk.w[4 * i + 3] = v.w;
  }
}

// T0 lookup of byte k (0 = least significant) of s; `rb` = this lane's replica byte offset.
__device__ __forceinline__ uint32_t tlook(uint32_t s, int k, uint32_t rb) {
  const uint32_t idx = (s >> (8 * k)) & 0xff;
  return *(const uint32_t*)((const uint8_t*)g_t0 + idx * (4 * kTReplicas) + rb);
}

// AES-128 encryption of a block given as big-endian column words (FIPS-197 §5.1).
__device__ __forceinline__ void aes128_block(const AesRk& rk, uint32_t rb, uint32_t& s0, uint32_t& s1,
                                             uint32_t& s2, uint32_t& s3) {
#if MQ_PROF_SKIP & 16
  s0 ^= rk.w[0]; s1 ^= rk.w[41]; s2 ^= rk.w[42] ^ rb; s3 ^= rk.w[43];
  return;
#endif
  s0 ^= rk.w[0]; s1 ^= rk.w[1]; s2 ^= rk.w[2]; s3 ^= rk.w[3];
#pragma unroll
  for (int r = 1; r < 10; ++r) {
    const uint32_t t0 = tlook(s0, 3, rb) ^ ror(tlook(s1, 2, rb), 8) ^ ror(tlook(s2, 1, rb), 16) ^ ror(tlook(s3, 0, rb), 24) ^ rk.w[4 * r];
    const uint32_t t1 = tlook(s1, 3, rb) ^ ror(tlook(s2, 2, rb), 8) ^ ror(tlook(s3, 1, rb), 16) ^ ror(tlook(s0, 0, rb), 24) ^ rk.w[4 * r + 1];
    const uint32_t t2 = tlook(s2, 3, rb) ^ ror(tlook(s3, 2, rb), 8) ^ ror(tlook(s0, 1, rb), 16) ^ ror(tlook(s1, 0, rb), 24) ^ rk.w[4 * r + 2];
    const uint32_t t3 = tlook(s3, 3, rb) ^ ror(tlook(s0, 2, rb), 8) ^ ror(tlook(s1, 1, rb), 16) ^ ror(tlook(s2, 0, rb), 24) ^ rk.w[4 * r + 3];
    s0 = t0; s1 = t1; s2 = t2; s3 = t3;
  }
  // final round: SubBytes + ShiftRows (S[x] = byte 2 of T0[x]) + AddRoundKey
  auto fin = [&](uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t k) {
    return ((tlook(a, 3, rb) << 8) & 0xff000000u) ^ (tlook(b, 2, rb) & 0x00ff0000u) ^
           ((tlook(c, 1, rb) >> 8) & 0x0000ff00u) ^ ((tlook(d, 0, rb) >> 16) & 0x000000ffu) ^ k;
  };
  const uint32_t o0 = fin(s0, s1, s2, s3, rk.w[40]), o1 = fin(s1, s2, s3, s0, rk.w[41]),
                 o2 = fin(s2, s3, s0, s1, rk.w[42]), o3 = fin(s3, s0, s1, s2, rk.w[43]);
  s0 = o0; s1 = o1; s2 = o2; s3 = o3;
}

// ---- GHASH in the bit-reflected basis: bit i of word k = coefficient of x^(32k+i) --------------
__device__ __forceinline__ uint32_t brev(uint32_t x) { return __builtin_bitreverse32(x); }
// memory dword (little-endian load of 4 GCM bytes) <-> reflected word
__device__ __forceinline__ uint32_t refl(uint32_t le) { return brev(bswap32(le)); }

// operand prepared for repeated multiplication: 9 Karatsuba words x 4 bit-hole masks
struct GfOp { uint32_t y[9][4]; };

__device__ __forceinline__ void holes(uint32_t v, uint32_t (&o)[4]) {
  o[0] = v & 0x11111111u; o[1] = v & 0x22222222u; o[2] = v & 0x44444444u; o[3] = v & 0x88888888u;
}

__device__ __forceinline__ GfOp gf_prepare(const uint32_t (&b)[4]) {
  GfOp op;
  const uint32_t c0 = b[0] ^ b[2], c1 = b[1] ^ b[3];
  const uint32_t k[9] = {b[0], b[1], b[0] ^ b[1], b[2], b[3], b[2] ^ b[3], c0, c1, c0 ^ c1};
#pragma unroll
  for (int i = 0; i < 9; ++i) holes(k[i], op.y[i]);
  return op;
}

// 3-input XOR and bit select in one v_bitop3_b32 (gfx950): on this chip every VALU op other than
// add / xor / or / and issues at about half their rate (tools/ubench/ubench4.hip), so one bitop3
// replaces two of them profitably, not three.
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint32_t sel3(uint32_t m, uint32_t a, uint32_t b) {  // m ? a : b, bitwise
  return __builtin_amdgcn_bitop3_b32(m, a, b, 0xca);  // LUT index = 4 src0 + 2 src1 + src2
}
__device__ __forceinline__ uint64_t xor4_64(uint64_t a, uint64_t b, uint64_t c, uint64_t d) {
  const uint32_t lo = xor3((uint32_t)a, (uint32_t)b, (uint32_t)c) ^ (uint32_t)d;
  const uint32_t hi = xor3((uint32_t)(a >> 32), (uint32_t)(b >> 32), (uint32_t)(c >> 32)) ^ (uint32_t)(d >> 32);
  return (uint64_t)hi << 32 | lo;
}

// 32x32 -> 64 carry-less product with holes
__device__ __forceinline__ uint64_t bmul32(uint32_t x, const uint32_t (&y)[4]) {
  uint32_t xh[4];
  holes(x, xh);
  const uint64_t z0 = xor4_64((uint64_t)xh[0] * y[0], (uint64_t)xh[1] * y[3], (uint64_t)xh[2] * y[2], (uint64_t)xh[3] * y[1]);
  const uint64_t z1 = xor4_64((uint64_t)xh[0] * y[1], (uint64_t)xh[1] * y[0], (uint64_t)xh[2] * y[3], (uint64_t)xh[3] * y[2]);
  const uint64_t z2 = xor4_64((uint64_t)xh[0] * y[2], (uint64_t)xh[1] * y[1], (uint64_t)xh[2] * y[0], (uint64_t)xh[3] * y[3]);
  const uint64_t z3 = xor4_64((uint64_t)xh[0] * y[3], (uint64_t)xh[1] * y[2], (uint64_t)xh[2] * y[1], (uint64_t)xh[3] * y[0]);
  // keep bit class k of z_k: (z0 at 0x1.., z1 at 0x2..) and (z2 at 0x4.., z3 at 0x8..), then
  // the two halves by class 0|1 — three bit selects
  auto pick = [](uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    return sel3(0x33333333u, sel3(0x11111111u, a, b), sel3(0x44444444u, c, d));
  };
  const uint32_t lo = pick((uint32_t)z0, (uint32_t)z1, (uint32_t)z2, (uint32_t)z3);
  const uint32_t hi = pick((uint32_t)(z0 >> 32), (uint32_t)(z1 >> 32), (uint32_t)(z2 >> 32), (uint32_t)(z3 >> 32));
  return (uint64_t)hi << 32 | lo;
}

// 256-bit product p7..p0 -> a = p mod (x^128 + x^7 + x^2 + x + 1): x^(128+j) -> x^j + x^(j+1) +
// x^(j+2) + x^(j+7)
__device__ __forceinline__ void gf_fold(uint32_t p0, uint32_t p1, uint32_t p2, uint32_t p3, uint32_t p4,
                                        uint32_t p5, uint32_t p6, uint32_t p7, uint32_t (&a)[4]) {
  const uint32_t t = (p7 >> 31) ^ (p7 >> 30) ^ (p7 >> 25);
  a[0] = p0 ^ p4 ^ (p4 << 1) ^ (p4 << 2) ^ (p4 << 7) ^ t ^ (t << 1) ^ (t << 2) ^ (t << 7);
  a[1] = p1 ^ p5 ^ ((p5 << 1) | (p4 >> 31)) ^ ((p5 << 2) | (p4 >> 30)) ^ ((p5 << 7) | (p4 >> 25));
  a[2] = p2 ^ p6 ^ ((p6 << 1) | (p5 >> 31)) ^ ((p6 << 2) | (p5 >> 30)) ^ ((p6 << 7) | (p5 >> 25));
  a[3] = p3 ^ p7 ^ ((p7 << 1) | (p6 >> 31)) ^ ((p7 << 2) | (p6 >> 30)) ^ ((p7 << 7) | (p6 >> 25));
}

// a = a * b mod (x^128 + x^7 + x^2 + x + 1), b prepared
__device__ __forceinline__ void gf_mul(uint32_t (&a)[4], const GfOp& b) {
  const uint32_t c0 = a[0] ^ a[2], c1 = a[1] ^ a[3];
  // low half a1:a0 * b1:b0
  const uint64_t l0 = bmul32(a[0], b.y[0]), l1 = bmul32(a[1], b.y[1]), l2 = bmul32(a[0] ^ a[1], b.y[2]) ^ l0 ^ l1;
  // high half a3:a2 * b3:b2
  const uint64_t h0 = bmul32(a[2], b.y[3]), h1 = bmul32(a[3], b.y[4]), h2 = bmul32(a[2] ^ a[3], b.y[5]) ^ h0 ^ h1;
  // middle (a_lo ^ a_hi) * (b_lo ^ b_hi)
  const uint64_t m0 = bmul32(c0, b.y[6]), m1 = bmul32(c1, b.y[7]), m2 = bmul32(c0 ^ c1, b.y[8]) ^ m0 ^ m1;
  // 128-bit products as 4 words
  uint32_t L[4] = {(uint32_t)l0, (uint32_t)(l0 >> 32) ^ (uint32_t)l2, (uint32_t)(l2 >> 32) ^ (uint32_t)l1, (uint32_t)(l1 >> 32)};
  uint32_t H[4] = {(uint32_t)h0, (uint32_t)(h0 >> 32) ^ (uint32_t)h2, (uint32_t)(h2 >> 32) ^ (uint32_t)h1, (uint32_t)(h1 >> 32)};
  uint32_t M[4] = {(uint32_t)m0, (uint32_t)(m0 >> 32) ^ (uint32_t)m2, (uint32_t)(m2 >> 32) ^ (uint32_t)m1, (uint32_t)(m1 >> 32)};
#pragma unroll
  for (int i = 0; i < 4; ++i) M[i] ^= L[i] ^ H[i];
  // P = L + M x^64 + H x^128  (8 words)
  const uint32_t p0 = L[0], p1 = L[1], p2 = L[2] ^ M[0], p3 = L[3] ^ M[1];
  const uint32_t p4 = H[0] ^ M[2], p5 = H[1] ^ M[3], p6 = H[2], p7 = H[3];
  gf_fold(p0, p1, p2, p3, p4, p5, p6, p7, a);
}

// ---- tables of the packet tile kernels (mq_aes.hip): one static LDS block per workgroup --------
//  [0, 8 KiB)       single-key kernels: the half tables of H^1 and H^2 for the tags' final
//                   multiply (g_aes_fin holds H^3 .. H^7); multi-key kernels: unused
//  [8 KiB, 72 KiB)  wide T-table: row x (256 B) = 32 replicas of T0[x], then 32 replicas of
//                   T2[x] = ror(T0[x], 16). Lane l reads replica l & 31, so the 32 lanes of each
//                   ds_read_b32 lane group hit 32 distinct banks. The byte address of
//                   "row = byte k of s" is perm(s, 4 (l & 31) [+ 128 for T2]) — one v_perm_b32.
//  [72 KiB, ...)    round keys: per wave, the AEAD and HP key schedules of its 8 packets
//                   (kRkSlotBytes each; multi-key kernels), or one row's (single-key kernels)
constexpr uint32_t kGhBytes = 8192, kTwBytes = 65536;
constexpr uint32_t kRkSlotBytes = 2 * 176;  // aes_rk || hp_rk
__shared__ __attribute__((aligned(16))) uint32_t g_aes_lds[(kGhBytes + kTwBytes) / 4];
// multi-key tile kernels: per wave, the GHASH half table (gh_mul_half) of its tile's key
#ifndef MQ_AES_MULTI_WAVES
#define MQ_AES_MULTI_WAVES 12
#endif
constexpr uint32_t kGhHalfBytes = 4096, kAesMultiWaves = MQ_AES_MULTI_WAVES;
__shared__ __attribute__((aligned(16))) uint32_t g_aes_wtab[kAesMultiWaves * kGhHalfBytes / 4];
// single-key tile kernels: half tables of H^3 .. H^7 for the tag's final multiply (lane j of a
// packet multiplies by H^e, e = 1..8 blocks after its last one: H^1, H^2 in g_aes_lds's first
// 8 KiB, fin_table; a lane with e = 8 multiplies its last block by H^8 in the Horner loop instead)
constexpr uint32_t kFinTables = 5;
__shared__ __attribute__((aligned(16))) uint32_t g_aes_fin[kFinTables * kGhHalfBytes / 4];
// single-key tile kernels: the byte-position GHASH table of H^8 (gh_mul_tab8). Entry (q, u) at
// byte 4096 q + 16 u holds (u x^(8q)) * H^8 as 4 reflected words, q = byte position 0..15 of the
// operand (byte q = bits 8q..8q+7 of the reflected value: byte q & 3 of word q >> 2), u = its
// value; a * H^8 = XOR over q of entry (q, byte q of a). 16 reads of 16 B instead of the nibble
// table's 32 (and half the XORs); 64 KiB fit beside the T-table once the round keys of a
// single-key workgroup take one 352-B slot (g_aes_keys1) instead of the multi-key kernels' 33 KiB.
// (Placed at LDS address 0 — 64-KiB alignment — the table's row bases fold into the read offsets,
// but the T-table then sits above 64 KiB and every T-table lookup needs an add: C +5.8 %, r03ab.)
constexpr uint32_t kGh8Bytes = 65536;
__shared__ __attribute__((aligned(16))) uint32_t g_aes_gh8[kGh8Bytes / 4];

// final-multiply half table of H^(e1 + 1), e1 = 0..6
__device__ __forceinline__ const uint8_t* fin_table(uint32_t e1) {
  return e1 < 2 ? (const uint8_t*)g_aes_lds + kGhHalfBytes * e1 : (const uint8_t*)g_aes_fin + kGhHalfBytes * (e1 - 2);
}

__device__ __forceinline__ uint32_t xtime8(uint32_t s) { return ((s << 1) ^ ((s & 0x80) ? 0x11bu : 0u)) & 0xffu; }

__device__ __forceinline__ void build_tw(int tid, int nthreads) {
  uint4* tw = (uint4*)((uint8_t*)g_aes_lds + kGhBytes);
  for (int e = tid; e < 256 * 16; e += nthreads) {  // 16-B group e: row e >> 4, quarter e & 15
    const uint32_t s = kSbox[e >> 4], s2 = xtime8(s);
    const uint32_t t0 = (s2 << 24) | (s << 16) | (s << 8) | (s2 ^ s);
    const uint32_t v = (e & 8) ? ror(t0, 16) : t0;
    tw[e] = make_uint4(v, v, v, v);
  }
}

// this lane's replica byte offsets into a T-table row: T0 (r0) and T2 (r2)
struct TwLane { uint32_t r0, r2; };
__device__ __forceinline__ TwLane tw_lane() {
  const uint32_t r = (threadIdx.x & 31u) * 4u;
  return TwLane{r, r + 128u};
}
// T-table entry of row "byte k of s" from the half selected by rsel (L.r0: T0, L.r2: T2)
__device__ __forceinline__ uint32_t twl(uint32_t s, int k, uint32_t rsel) {
  const uint32_t addr = __builtin_amdgcn_perm(s, rsel, 0x0c0c0000u | ((4u + (uint32_t)k) << 8));
  return *(const uint32_t*)((const uint8_t*)g_aes_lds + kGhBytes + addr);
}

// Round-key sources: registers (SGPRs when wave-uniform) or an LDS key schedule (a per-lane
// pointer, so lanes of one wave may use different keys at no register cost). k(r) = the four
// words of round key r.
struct RkRegs {
  const AesRk& rk;
  __device__ __forceinline__ uint4 operator()(int r) const {
    return make_uint4(rk.w[4 * r], rk.w[4 * r + 1], rk.w[4 * r + 2], rk.w[4 * r + 3]);
  }
};
struct RkLds {
  const uint32_t* p;  // LDS
  __device__ __forceinline__ uint4 operator()(int r) const { return *(const uint4*)(p + 4 * r); }
};
__device__ __forceinline__ uint32_t u4at(const uint4& v, int q) { return q == 0 ? v.x : q == 1 ? v.y : q == 2 ? v.z : v.w; }

// One round from state s (rounds 1..9) through the wide table: all 16 lookups (and the key)
// are issued before any is consumed, so the LDS queue streams them.
template <class K>
__device__ __forceinline__ void aes_round(const K& key, int r, const TwLane& L, uint32_t (&s)[4]) {
  uint32_t l[16];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int q1 = (q + 1) & 3, q2 = (q + 2) & 3, q3 = (q + 3) & 3;
    l[4 * q] = twl(s[q], 3, L.r0); l[4 * q + 1] = twl(s[q2], 1, L.r2);
    l[4 * q + 2] = twl(s[q1], 2, L.r0); l[4 * q + 3] = twl(s[q3], 0, L.r2);
  }
  const uint4 kr = key(r);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int q = 0; q < 4; ++q) s[q] = l[4 * q] ^ l[4 * q + 1] ^ ror(l[4 * q + 2] ^ l[4 * q + 3], 8) ^ u4at(kr, q);
}

// final round: SubBytes + ShiftRows (S[x] from T2 byte 3, T0 byte 2, T0 byte 1, T2 byte 0) +
// AddRoundKey
template <class K>
__device__ __forceinline__ void aes_final(const K& key, const TwLane& L, uint32_t (&s)[4]) {
  uint32_t l[16];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int q1 = (q + 1) & 3, q2 = (q + 2) & 3, q3 = (q + 3) & 3;
    l[4 * q] = twl(s[q], 3, L.r2); l[4 * q + 1] = twl(s[q1], 2, L.r0);
    l[4 * q + 2] = twl(s[q2], 1, L.r0); l[4 * q + 3] = twl(s[q3], 0, L.r2);
  }
  const uint4 kr = key(10);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int q = 0; q < 4; ++q)
    s[q] = (__builtin_amdgcn_perm(l[4 * q], l[4 * q + 1], 0x07020c0cu) |
            __builtin_amdgcn_perm(l[4 * q + 2], l[4 * q + 3], 0x0c0c0500u)) ^ u4at(kr, q);
}

// AES-128 encryption of a block of big-endian column words with the wide table:
// T1[x] = ror(T0[x], 8) and T3[x] = ror(T2[x], 8), so each output column is
// T0[a] ^ T2[c] ^ ror(T0[b] ^ T2[d], 8) ^ k.
template <class K>
__device__ __forceinline__ void aes128_enc(const K& key, const TwLane& L, uint32_t (&s)[4]) {
#if MQ_PROF_SKIP & 16
  {
    const uint4 z = key(0);
    s[0] ^= z.x; s[1] ^= z.y; s[2] ^= z.z ^ L.r0; s[3] ^= z.w;
    return;
  }
#endif
  const uint4 k0 = key(0);
  s[0] ^= k0.x; s[1] ^= k0.y; s[2] ^= k0.z; s[3] ^= k0.w;
#pragma unroll
  for (int r = 1; r < 10; ++r) aes_round(key, r, L, s);
  aes_final(key, L, s);
}

__device__ __forceinline__ void aes128_block(const AesRk& rk, const TwLane& L, uint32_t& s0, uint32_t& s1,
                                             uint32_t& s2, uint32_t& s3) {
  uint32_t s[4] = {s0, s1, s2, s3};
  aes128_enc(RkRegs{rk}, L, s);
  s0 = s[0]; s1 = s[1]; s2 = s[2]; s3 = s[3];
}

// CTR caching (counter-mode AES with counters < 256): the input of block c of a packet is
// (nonce words n0..n2, counter c), so after AddRoundKey only byte 0 of column 3 depends on c.
// Round 1 therefore has three constant columns and one column with a single varying lookup
// (T2 of that byte, rotated), and round 2 — whose input differs only in column 0 — has one
// varying lookup per column. The per-packet constants below replace 27 of the block's 176
// lookups and most of two rounds of VALU work.
struct AesCtrCache {
  uint32_t k0;      // round-1 column 0 without its varying term
  uint32_t d[4];    // round-2 columns without their varying terms
  uint32_t x;       // low byte of round key word 3 (xored with the counter's low byte)
};

template <class K>
__device__ __forceinline__ AesCtrCache ctr_cache(const K& key, const TwLane& L, const uint32_t (&nb)[3]) {
  const uint4 r0 = key(0), r1 = key(1), r2 = key(2);
  const uint32_t s0 = nb[0] ^ r0.x, s1 = nb[1] ^ r0.y, s2 = nb[2] ^ r0.z, s3 = r0.w;
  AesCtrCache c;
  c.x = r0.w & 0xffu;
  // round 1 (column q = T0[b3 s_q] ^ T2[b1 s_q+2] ^ ror8(T0[b2 s_q+1] ^ T2[b0 s_q+3]) ^ k);
  // byte 0 of s3 (the counter's) only enters column 0
  c.k0 = twl(s0, 3, L.r0) ^ twl(s2, 1, L.r2) ^ ror(twl(s1, 2, L.r0), 8) ^ r1.x;
  const uint32_t k1 = twl(s1, 3, L.r0) ^ twl(s3, 1, L.r2) ^ ror(twl(s2, 2, L.r0) ^ twl(s0, 0, L.r2), 8) ^ r1.y;
  const uint32_t k2 = twl(s2, 3, L.r0) ^ twl(s0, 1, L.r2) ^ ror(twl(s3, 2, L.r0) ^ twl(s1, 0, L.r2), 8) ^ r1.z;
  const uint32_t k3 = twl(s3, 3, L.r0) ^ twl(s1, 1, L.r2) ^ ror(twl(s0, 2, L.r0) ^ twl(s2, 0, L.r2), 8) ^ r1.w;
  // round 2 with t1..t3 = k1..k3 constant: every column has one term from t0
  c.d[0] = twl(k2, 1, L.r2) ^ ror(twl(k1, 2, L.r0) ^ twl(k3, 0, L.r2), 8) ^ r2.x;
  c.d[1] = twl(k1, 3, L.r0) ^ twl(k3, 1, L.r2) ^ ror(twl(k2, 2, L.r0), 8) ^ r2.y;
  c.d[2] = twl(k2, 3, L.r0) ^ ror(twl(k3, 2, L.r0) ^ twl(k1, 0, L.r2), 8) ^ r2.z;
  c.d[3] = twl(k3, 3, L.r0) ^ twl(k1, 1, L.r2) ^ ror(twl(k2, 0, L.r2), 8) ^ r2.w;
  return c;
}

// state after round 2 of the CTR block with counter `ctr` (< 256)
__device__ __forceinline__ void ctr_round2(const AesCtrCache& c, const TwLane& L, uint32_t ctr, uint32_t (&s)[4]) {
  const uint32_t t0 = c.k0 ^ ror(twl(ctr ^ c.x, 0, L.r2), 8);
  s[0] = c.d[0] ^ twl(t0, 3, L.r0);
  s[1] = c.d[1] ^ ror(twl(t0, 0, L.r2), 8);
  s[2] = c.d[2] ^ twl(t0, 1, L.r2);
  s[3] = c.d[3] ^ ror(twl(t0, 2, L.r0), 8);
}

// CTR block with counter `ctr` (< 256) from the cache: rounds 3..10
template <class K>
__device__ __forceinline__ void aes128_ctr1(const K& key, const TwLane& L, const AesCtrCache& c, uint32_t ctr,
                                            uint32_t (&s)[4]) {
#if MQ_PROF_SKIP & 16
  s[0] = c.d[0] ^ ctr; s[1] = c.d[1]; s[2] = c.d[2] ^ L.r0; s[3] = c.d[3];
  return;
#endif
  ctr_round2(c, L, ctr, s);
#pragma unroll
  for (int r = 3; r < 10; ++r) aes_round(key, r, L, s);
  aes_final(key, L, s);
}

// a = x^i * h (reflected basis), 0 <= i < 128: shift into 8 words, then fold
__device__ __forceinline__ void gf_mul_xi(const uint32_t (&h)[4], uint32_t i, uint32_t (&a)[4]) {
  const uint32_t r = i & 31u, q = i >> 5;
  uint32_t sh[5];
  sh[0] = h[0] << r;
#pragma unroll
  for (int k = 1; k < 4; ++k) sh[k] = r ? ((h[k] << r) | (h[k - 1] >> (32u - r))) : h[k];
  sh[4] = r ? h[3] >> (32u - r) : 0u;
  uint32_t p[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    uint32_t v = 0;
#pragma unroll
    for (int t = 0; t < 4; ++t)
      if (k - t >= 0 && k - t <= 4) v = (q == (uint32_t)t) ? sh[k - t] : v;
    p[k] = v;
  }
  gf_fold(p[0], p[1], p[2], p[3], p[4], p[5], p[6], p[7], a);
}

// byte-position GHASH table for multiplier h (reflected words), built by the whole workgroup:
// basis entries (q, 1 << b) = x^(8q+b) h first, then every other entry as the XOR of its bits'
// basis entries. Ends with a workgroup barrier.
__device__ __forceinline__ void build_gh8(const uint32_t (&h)[4], int tid, int nthreads) {
  uint4* gh = (uint4*)g_aes_gh8;
  for (int i = tid; i < 128; i += nthreads) {
    uint32_t a[4];
    gf_mul_xi(h, (uint32_t)i, a);
    gh[(i >> 3) * 256 + (1 << (i & 7))] = make_uint4(a[0], a[1], a[2], a[3]);
  }
  __syncthreads();
  for (int e = tid; e < 4096; e += nthreads) {
    const int q = e >> 8, u = e & 255;
    if (u != 0 && (u & (u - 1)) == 0) continue;  // basis entry
    uint4 acc = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int b = 0; b < 8; ++b)
      if ((u >> b) & 1) {
        const uint4 x = gh[q * 256 + (1 << b)];
        acc.x ^= x.x; acc.y ^= x.y; acc.z ^= x.z; acc.w ^= x.w;
      }
    gh[e] = acc;
  }
  __syncthreads();
}

__device__ __forceinline__ uint32_t byte_of(uint32_t x, int m) {
  return m == 0 ? (x & 0xffu) : (m == 3 ? (x >> 24) : __builtin_amdgcn_ubfe(x, 8 * m, 8));
}

// a = a * H^8 through the GHASH table: nibble 2m of word w sits (times 16) in byte m of
// (a[w] << 4) & 0xf0f0f0f0, nibble 2m+1 in byte m of a[w] & 0xf0f0f0f0 — each a ready byte offset
// of its entry within its position's 256-B row. The 32 reads go in 8 groups of 4 with at most two
// groups in flight: group g's addresses take a fake dependency (empty asm) on the accumulator
// after group g - 2, because the scheduler would otherwise issue all 32 at once (128 VGPRs) and
// the 4-waves/SIMD streaming kernels would spill.
__device__ __forceinline__ void gh_group(const uint32_t (&a)[4], int g, uint4 (&e)[4], const uint32_t* dep,
                                         const uint8_t* t) {
  const int w = g >> 1, mb = 2 * (g & 1);
  const uint32_t lo = (a[w] << 4) & 0xf0f0f0f0u, hi = a[w] & 0xf0f0f0f0u;
  uint32_t ad[4] = {byte_of(lo, mb), byte_of(hi, mb), byte_of(lo, mb + 1), byte_of(hi, mb + 1)};
  if (dep)
    asm volatile("" : "+v"(ad[0]), "+v"(ad[1]), "+v"(ad[2]), "+v"(ad[3]) : "v"(dep[0]), "v"(dep[1]), "v"(dep[2]), "v"(dep[3]));
  e[0] = *(const uint4*)(t + ad[0]);
  e[1] = *(const uint4*)(t + 256 + ad[1]);
  e[2] = *(const uint4*)(t + 512 + ad[2]);
  e[3] = *(const uint4*)(t + 768 + ad[3]);
}
__device__ __forceinline__ void gh_fold(uint32_t (&r)[4], const uint4 (&e)[4]) {
  r[0] = xor3(r[0], e[0].x, e[1].x); r[1] = xor3(r[1], e[0].y, e[1].y);
  r[2] = xor3(r[2], e[0].z, e[1].z); r[3] = xor3(r[3], e[0].w, e[1].w);
  r[0] = xor3(r[0], e[2].x, e[3].x); r[1] = xor3(r[1], e[2].y, e[3].y);
  r[2] = xor3(r[2], e[2].z, e[3].z); r[3] = xor3(r[3], e[2].w, e[3].w);
}
// a = a * H^8 through the byte-position table: word w's four bytes, scaled by the 16-B entry size,
// read rows 4w .. 4w + 3. Words go in groups of 4 reads with at most two groups in flight (the
// empty asm ties group w's addresses to the accumulator after group w - 2), as in gh_mul_half.
__device__ __forceinline__ void gh_group8(const uint32_t (&a)[4], int w, uint4 (&e)[4], const uint32_t* dep) {
  const uint32_t x = a[w];
  uint32_t ad[4] = {(x << 4) & 0xff0u, (x >> 4) & 0xff0u, (x >> 12) & 0xff0u, (x >> 20) & 0xff0u};
  if (dep)
    asm volatile("" : "+v"(ad[0]), "+v"(ad[1]), "+v"(ad[2]), "+v"(ad[3]) : "v"(dep[0]), "v"(dep[1]), "v"(dep[2]), "v"(dep[3]));
  const uint8_t* t = (const uint8_t*)g_aes_gh8 + 16384u * (uint32_t)w;
  e[0] = *(const uint4*)(t + ad[0]);
  e[1] = *(const uint4*)(t + 4096 + ad[1]);
  e[2] = *(const uint4*)(t + 8192 + ad[2]);
  e[3] = *(const uint4*)(t + 12288 + ad[3]);
}
__device__ __forceinline__ void gh_mul_tab8(uint32_t (&a)[4]) {
  uint32_t r[4] = {0, 0, 0, 0};
  uint4 e0[4], e1[4];
  gh_group8(a, 0, e0, nullptr);
  gh_group8(a, 1, e1, nullptr);
  gh_fold(r, e0);
  gh_group8(a, 2, e0, r);
  gh_fold(r, e1);
  gh_group8(a, 3, e1, r);
  gh_fold(r, e0);
  gh_fold(r, e1);
  a[0] = r[0]; a[1] = r[1]; a[2] = r[2]; a[3] = r[3];
}

// ---- per-wave GHASH half table (multi-key kernels, waves whose packets share one key) -----------
// Entry (p, v) of the wave's 4 KiB, p = 0..15, v = 0..15, at byte 256 p + 16 v: (v x^(4p)) * H^8 —
// the low 16 nibble positions of the full table. a * H^8 = T(a_hi) x^64 + T(a_lo): the high
// half's nibbles read the same entries and one fold (x^64 mod the GCM polynomial) shifts their
// sum up before the low half's entries are added. 12 such tables fit beside the T-table where 12
// full ones would not. Built by the wave without branches or LDS reads: lane l takes position
// l / 4 and the four values whose top two bits are l % 4 — basis x^(4p+b) H for b = 0..3 (one
// multiply by x^(4p), then three by x), the top-bit part by selects, the four entries by XOR.
__device__ __forceinline__ void gf_mul_x(uint32_t (&a)[4]) {  // a * x
  const uint32_t c = a[3] >> 31;
  a[3] = __builtin_amdgcn_alignbit(a[3], a[2], 31);
  a[2] = __builtin_amdgcn_alignbit(a[2], a[1], 31);
  a[1] = __builtin_amdgcn_alignbit(a[1], a[0], 31);
  a[0] = (a[0] << 1) ^ (c ? 0x87u : 0u);
}
__device__ __forceinline__ void build_gh_half(uint8_t* tab, const uint32_t (&h)[4], int lane) {
  const uint32_t p = (uint32_t)lane >> 2, vh = (uint32_t)lane & 3u;
  uint32_t b0[4], b1[4], b2[4], b3[4];
  gf_mul_xi(h, 4u * p, b0);
#pragma unroll
  for (int q = 0; q < 4; ++q) b1[q] = b0[q];
  gf_mul_x(b1);
#pragma unroll
  for (int q = 0; q < 4; ++q) b2[q] = b1[q];
  gf_mul_x(b2);
#pragma unroll
  for (int q = 0; q < 4; ++q) b3[q] = b2[q];
  gf_mul_x(b3);
  uint32_t hi[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) hi[q] = ((vh & 1u) ? b2[q] : 0u) ^ ((vh & 2u) ? b3[q] : 0u);
  uint4* e = (uint4*)(tab + 256u * p + 64u * vh);  // entries (p, 4 vh .. 4 vh + 3)
  e[0] = make_uint4(hi[0], hi[1], hi[2], hi[3]);
  e[1] = make_uint4(hi[0] ^ b0[0], hi[1] ^ b0[1], hi[2] ^ b0[2], hi[3] ^ b0[3]);
  e[2] = make_uint4(hi[0] ^ b1[0], hi[1] ^ b1[1], hi[2] ^ b1[2], hi[3] ^ b1[3]);
  e[3] = make_uint4(hi[0] ^ b0[0] ^ b1[0], hi[1] ^ b0[1] ^ b1[1], hi[2] ^ b0[2] ^ b1[2], hi[3] ^ b0[3] ^ b1[3]);
  wave_sync();
}
__device__ __forceinline__ void gh_mul_half(uint32_t (&a)[4], const uint8_t* tab) {
  auto row = [tab](int g) { return tab + 256u * (8 * ((g >> 1) & 1) + 4 * (g & 1)); };
  uint32_t r[4] = {0, 0, 0, 0};
  uint4 e0[4], e1[4];
  gh_group(a, 4, e0, nullptr, row(4));  // words 2, 3 first: T(a_hi)
  gh_group(a, 5, e1, nullptr, row(5));
  gh_fold(r, e0);
  gh_group(a, 6, e0, r, row(6));
  gh_fold(r, e1);
  gh_group(a, 7, e1, r, row(7));
  gh_fold(r, e0);
  gh_group(a, 0, e0, r, row(0));  // words 0, 1 in flight during the x^64 fold
  gh_fold(r, e1);
  gh_group(a, 1, e1, r, row(1));
  uint32_t s[4];
  gf_fold(0u, 0u, r[0], r[1], r[2], r[3], 0u, 0u, s);  // T(a_hi) * x^64
  gh_fold(s, e0);
  gh_group(a, 2, e0, s, row(2));
  gh_fold(s, e1);
  gh_group(a, 3, e1, s, row(3));
  gh_fold(s, e0);
  gh_fold(s, e1);
  a[0] = s[0]; a[1] = s[1]; a[2] = s[2]; a[3] = s[3];
}

}  // namespace mq
