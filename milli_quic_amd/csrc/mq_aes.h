// mq_aes.h — AES-128 and GF(2^128) building blocks for gfx950 without AES / carry-less-multiply
// instructions, shared by the AES-128-GCM packet kernels (mq_aes.hip) and the batched Initial key
// derivation (mq_derive.hip):
//   * AES-128 rounds from one T-table (T0, 1 KiB) in LDS replicated kTReplicas x per workgroup
//     (entry x, replica lane & 7 -> fewer bank conflicts), T1..T3 by rotation (FIPS-197 §5.1);
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
constexpr int kAesWaves = 4;  // waves (tiles) per workgroup sharing one T-table
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

// 32x32 -> 64 carry-less product with holes
__device__ __forceinline__ uint64_t bmul32(uint32_t x, const uint32_t (&y)[4]) {
  uint32_t xh[4];
  holes(x, xh);
  const uint64_t z0 = (uint64_t)xh[0] * y[0] ^ (uint64_t)xh[1] * y[3] ^ (uint64_t)xh[2] * y[2] ^ (uint64_t)xh[3] * y[1];
  const uint64_t z1 = (uint64_t)xh[0] * y[1] ^ (uint64_t)xh[1] * y[0] ^ (uint64_t)xh[2] * y[3] ^ (uint64_t)xh[3] * y[2];
  const uint64_t z2 = (uint64_t)xh[0] * y[2] ^ (uint64_t)xh[1] * y[1] ^ (uint64_t)xh[2] * y[0] ^ (uint64_t)xh[3] * y[3];
  const uint64_t z3 = (uint64_t)xh[0] * y[3] ^ (uint64_t)xh[1] * y[2] ^ (uint64_t)xh[2] * y[1] ^ (uint64_t)xh[3] * y[0];
  return (z0 & 0x1111111111111111ull) | (z1 & 0x2222222222222222ull) | (z2 & 0x4444444444444444ull) |
         (z3 & 0x8888888888888888ull);
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
  // fold x^(128+j) -> x^j + x^(j+1) + x^(j+2) + x^(j+7)
  const uint32_t t = (p7 >> 31) ^ (p7 >> 30) ^ (p7 >> 25);
  a[0] = p0 ^ p4 ^ (p4 << 1) ^ (p4 << 2) ^ (p4 << 7) ^ t ^ (t << 1) ^ (t << 2) ^ (t << 7);
  a[1] = p1 ^ p5 ^ ((p5 << 1) | (p4 >> 31)) ^ ((p5 << 2) | (p4 >> 30)) ^ ((p5 << 7) | (p4 >> 25));
  a[2] = p2 ^ p6 ^ ((p6 << 1) | (p5 >> 31)) ^ ((p6 << 2) | (p5 >> 30)) ^ ((p6 << 7) | (p5 >> 25));
  a[3] = p3 ^ p7 ^ ((p7 << 1) | (p6 >> 31)) ^ ((p7 << 2) | (p6 >> 30)) ^ ((p7 << 7) | (p6 >> 25));
}

}  // namespace mq
