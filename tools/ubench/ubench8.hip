// ubench8 — AES-128 CTR keystream on gfx950: the product's wide T-table (LDS lookups, CTR round
// caching, mq_aes.h) against a BITSLICED AES with no LDS at all (reference
// src/crypto/rustcrypto.rs:38-94 calls aes 0.8.4, whose software backend is a fixsliced AES).
//
// Bitsliced: each lane encrypts 32 counter blocks at once; the state is 128 bit planes (uint32:
// bit k = block k), plane 8i + b = bit (7 - b) of byte i. SubBytes is the Boyar-Peralta circuit
// (113 gates: 32 AND, 77 XOR, 4 XNOR; verified against the FIPS-197 table for all 256 inputs
// below), ShiftRows is register renaming, MixColumns is XORs of planes (xtime = a plane shift with
// feedback into bits 4, 3, 1, 0), AddRoundKey XORs 0 / ~0 masks (round-key bits, wave-uniform:
// scalar loads). All ten rounds run in full (the T-table path caches rounds 1-2 of its CTR
// blocks; the same could save about a tenth here). The output keystream is transposed back to
// bytes (four 32 x 32 bit transposes) as the product would need it.
//
// Both kernels produce every keystream byte, fold it into a checksum per lane, and (mode "check")
// write the first 32 blocks of lane 0 so the host can compare them with a byte-wise FIPS-197 AES.
// Timing: best of 5 runs of NB blocks, blocks/s and the equivalent GiB/s of 16-B blocks.
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 ubench8.hip -o ubench8
#include "../../milli_quic_amd/csrc/mq_aes.h"

#include <cstdio>
#include <cstring>
#include <vector>

using namespace mq;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

// ---- T-table (product code path) -----------------------------------------------------------------
template <int WAVES>
__global__ __launch_bounds__(64 * WAVES) void ttab_ctr(const uint32_t* __restrict__ rkg, uint32_t iters,
                                                     uint32_t* __restrict__ out, uint32_t* __restrict__ chk) {
  build_tw(threadIdx.x, blockDim.x);
  __syncthreads();
  const TwLane L = tw_lane();
  AesRk rk;
  load_rk(rkg, rk);
  const uint32_t gl = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t nb[3] = {0x00112233u, 0x44556677u, 0x8899aabbu};
  const AesCtrCache cc = ctr_cache(RkRegs{rk}, L, nb);
  uint32_t acc = 0;
  for (uint32_t it = 0; it < iters; ++it) {
    uint32_t s[4];
    const uint32_t ctr = (gl + it) & 255u;  // < 256: the cached rounds apply
    aes128_ctr1(RkRegs{rk}, L, cc, ctr, s);
    acc ^= s[0] ^ (s[1] << 1) ^ (s[2] << 2) ^ (s[3] << 3);
    if (out && gl == 0 && it < 32) {
      for (int q = 0; q < 4; ++q) out[4 * it + q] = s[q];
    }
  }
  chk[gl] = acc;
}

// ---- bitsliced -------------------------------------------------------------------------------------
// Boyar-Peralta S-box on planes u[0] (MSB) .. u[7] (LSB), in place
__device__ __forceinline__ void sbox_bp(uint32_t (&u)[8]) {
  const uint32_t U0 = u[0], U1 = u[1], U2 = u[2], U3 = u[3], U4 = u[4], U5 = u[5], U6 = u[6], U7 = u[7];
  const uint32_t T1 = U0 ^ U3, T2 = U0 ^ U5, T3 = U0 ^ U6, T4 = U3 ^ U5, T5 = U4 ^ U6, T6 = T1 ^ T5, T7 = U1 ^ U2;
  const uint32_t T8 = U7 ^ T6, T9 = U7 ^ T7, T10 = T6 ^ T7, T11 = U1 ^ U5, T12 = U2 ^ U5, T13 = T3 ^ T4;
  const uint32_t T14 = T6 ^ T11, T15 = T5 ^ T11, T16 = T5 ^ T12, T17 = T9 ^ T16, T18 = U3 ^ U7, T19 = T7 ^ T18;
  const uint32_t T20 = T1 ^ T19, T21 = U6 ^ U7, T22 = T7 ^ T21, T23 = T2 ^ T22, T24 = T2 ^ T10, T25 = T20 ^ T17;
  const uint32_t T26 = T3 ^ T16, T27 = T1 ^ T12;
  const uint32_t M1 = T13 & T6, M2 = T23 & T8, M3 = T14 ^ M1, M4 = T19 & U7, M5 = M4 ^ M1, M6 = T3 & T16;
  const uint32_t M7 = T22 & T9, M8 = T26 ^ M6, M9 = T20 & T17, M10 = M9 ^ M6, M11 = T1 & T15, M12 = T4 & T27;
  const uint32_t M13 = M12 ^ M11, M14 = T2 & T10, M15 = M14 ^ M11, M16 = M3 ^ M2, M17 = M5 ^ T24, M18 = M8 ^ M7;
  const uint32_t M19 = M10 ^ M15, M20 = M16 ^ M13, M21 = M17 ^ M15, M22 = M18 ^ M13, M23 = M19 ^ T25;
  const uint32_t M24 = M22 ^ M23, M25 = M22 & M20, M26 = M21 ^ M25, M27 = M20 ^ M21, M28 = M23 ^ M25;
  const uint32_t M29 = M28 & M27, M30 = M26 & M24, M31 = M20 & M23, M32 = M27 & M31, M33 = M27 ^ M25;
  const uint32_t M34 = M21 & M22, M35 = M24 & M34, M36 = M24 ^ M25, M37 = M21 ^ M29, M38 = M32 ^ M33;
  const uint32_t M39 = M23 ^ M30, M40 = M35 ^ M36, M41 = M38 ^ M40, M42 = M37 ^ M39, M43 = M37 ^ M38;
  const uint32_t M44 = M39 ^ M40, M45 = M42 ^ M41, M46 = M44 & T6, M47 = M40 & T8, M48 = M39 & U7;
  const uint32_t M49 = M43 & T16, M50 = M38 & T9, M51 = M37 & T17, M52 = M42 & T15, M53 = M45 & T27;
  const uint32_t M54 = M41 & T10, M55 = M44 & T13, M56 = M40 & T23, M57 = M39 & T19, M58 = M43 & T3;
  const uint32_t M59 = M38 & T22, M60 = M37 & T20, M61 = M42 & T1, M62 = M45 & T4, M63 = M41 & T2;
  const uint32_t L0 = M61 ^ M62, L1 = M50 ^ M56, L2 = M46 ^ M48, L3 = M47 ^ M55, L4 = M54 ^ M58, L5 = M49 ^ M61;
  const uint32_t L6 = M62 ^ L5, L7 = M46 ^ L3, L8 = M51 ^ M59, L9 = M52 ^ M53, L10 = M53 ^ L4, L11 = M60 ^ L2;
  const uint32_t L12 = M48 ^ M51, L13 = M50 ^ L0, L14 = M52 ^ M61, L15 = M55 ^ L1, L16 = M56 ^ L0;
  const uint32_t L17 = M57 ^ L1, L18 = M58 ^ L8, L19 = M63 ^ L4, L20 = L0 ^ L1, L21 = L1 ^ L7, L22 = L3 ^ L12;
  const uint32_t L23 = L18 ^ L2, L24 = L15 ^ L9, L25 = L6 ^ L10, L26 = L7 ^ L9, L27 = L8 ^ L10;
  const uint32_t L28 = L11 ^ L14, L29 = L11 ^ L17;
  u[0] = L6 ^ L24; u[1] = ~(L16 ^ L26); u[2] = ~(L19 ^ L28); u[3] = L6 ^ L21;
  u[4] = L20 ^ L22; u[5] = L25 ^ L29; u[6] = ~(L13 ^ L27); u[7] = ~(L6 ^ L23);
}

typedef uint32_t BsState[16][8];

__device__ __forceinline__ void bs_ark(BsState& x, const uint32_t* __restrict__ m) {  // m: 128 masks (uniform)
#pragma unroll
  for (int i = 0; i < 16; ++i)
#pragma unroll
    for (int b = 0; b < 8; ++b) x[i][b] ^= m[8 * i + b];
}

__device__ __forceinline__ void bs_shift_rows(BsState& x) {
  BsState y;
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int b = 0; b < 8; ++b) y[r + 4 * c][b] = x[r + 4 * ((c + r) & 3)][b];
#pragma unroll
  for (int i = 0; i < 16; ++i)
#pragma unroll
    for (int b = 0; b < 8; ++b) x[i][b] = y[i][b];
}

__device__ __forceinline__ void bs_xtime(const uint32_t (&v)[8], uint32_t (&o)[8]) {
  o[0] = v[1]; o[1] = v[2]; o[2] = v[3]; o[3] = v[4] ^ v[0];
  o[4] = v[5] ^ v[0]; o[5] = v[6]; o[6] = v[7] ^ v[0]; o[7] = v[0];
}

__device__ __forceinline__ void bs_mix_column(BsState& x, int c) {
  uint32_t t[8], a[4][8];
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int b = 0; b < 8; ++b) a[k][b] = x[k + 4 * c][b];
#pragma unroll
  for (int b = 0; b < 8; ++b) t[b] = xor3(a[0][b], a[1][b], a[2][b]) ^ a[3][b];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    uint32_t v[8], xt[8];
#pragma unroll
    for (int b = 0; b < 8; ++b) v[b] = a[k][b] ^ a[(k + 1) & 3][b];
    bs_xtime(v, xt);
#pragma unroll
    for (int b = 0; b < 8; ++b) x[k + 4 * c][b] = xor3(a[k][b], t[b], xt[b]);
  }
}

// 32 x 32 bit transpose of w (w[i] bit j <-> w[j] bit i), Hacker's Delight style
__device__ __forceinline__ void transpose32(uint32_t (&w)[32]) {
  uint32_t m = 0x0000FFFFu;
#pragma unroll
  for (int s = 16; s >= 1; s >>= 1, m ^= (m << s)) {
#pragma unroll
    for (int k = 0; k < 32; k = (k + s + 1) & ~s) {
      const uint32_t t = ((w[k] >> s) ^ w[k + s]) & m;
      w[k + s] ^= t;
      w[k] ^= t << s;
    }
  }
}

template <int WAVES>
__global__ __launch_bounds__(64 * WAVES) __attribute__((amdgpu_waves_per_eu(2))) void bs_ctr(const uint32_t* __restrict__ masks, uint32_t iters,
                                                   uint32_t* __restrict__ out, uint32_t* __restrict__ chk) {
  const uint32_t gl = blockIdx.x * blockDim.x + threadIdx.x;
  // input: nonce bytes 0..11, counter bytes 12..15 big-endian; counter = 32 * (group) + k
  const uint8_t nonce[12] = {0x00, 0x11, 0x22, 0x33, 0x44, 0x55, 0x66, 0x77, 0x88, 0x99, 0xaa, 0xbb};
  const uint32_t kpat[5] = {0xAAAAAAAAu, 0xCCCCCCCCu, 0xF0F0F0F0u, 0xFF00FF00u, 0xFFFF0000u};
  uint32_t acc = 0;
  for (uint32_t it = 0; it < iters; ++it) {
    const uint32_t base = 32u * (gl + it * 131u);  // counter of block 0 of this group (multiple of 32)
    BsState x;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const uint32_t byte = i < 12 ? nonce[i] : (base >> (8 * (15 - i))) & 0xffu;
#pragma unroll
      for (int b = 0; b < 8; ++b) x[i][b] = ((byte >> (7 - b)) & 1u) ? 0xFFFFFFFFu : 0u;
    }
#pragma unroll
    for (int j = 0; j < 5; ++j) x[15][7 - j] = kpat[j];  // the low 5 counter bits = block index
    bs_ark(x, masks);
#pragma unroll 1
    for (int r = 1; r < 10; ++r) {
#pragma unroll
      for (int i = 0; i < 16; ++i) sbox_bp(x[i]);
      bs_shift_rows(x);
#pragma unroll
      for (int c = 0; c < 4; ++c) bs_mix_column(x, c);
      bs_ark(x, masks + 128 * r);
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) sbox_bp(x[i]);
    bs_shift_rows(x);
    bs_ark(x, masks + 128 * 10);
    // back to bytes: word q of block k holds bytes 4q .. 4q + 3 (big-endian column word)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      uint32_t w[32];
#pragma unroll
      for (int bb = 0; bb < 4; ++bb)
#pragma unroll
        for (int b = 0; b < 8; ++b) w[8 * bb + b] = x[4 * q + bb][b];
      // w[p] bit k = bit (31 - p) of block k's word q; transpose32 maps w[i] bit j -> w[j] bit i,
      // so w[k] bit p = that word's bit (31 - p): one bit reversal gives the word
      transpose32(w);
#pragma unroll
      for (int k = 0; k < 32; ++k) {
        w[k] = __builtin_bitreverse32(w[k]);
        acc ^= w[k] + (uint32_t)k;
      }
      if (out && gl == 0 && it == 0) {
#pragma unroll
        for (int k = 0; k < 32; ++k) out[4 * k + q] = w[k];
      }
    }
  }
  chk[gl] = acc;
}

// ---- host ------------------------------------------------------------------------------------------
static uint8_t hs[256];
static uint8_t gm(uint8_t a, uint8_t b) { uint8_t r = 0; while (b) { if (b & 1) r ^= a; a = (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0)); b >>= 1; } return r; }
static void host_sbox() {
  for (int x = 0; x < 256; ++x) {
    uint8_t inv = 0;
    for (int y = 1; y < 256 && x; ++y) if (gm((uint8_t)x, (uint8_t)y) == 1) { inv = (uint8_t)y; break; }
    uint8_t s = inv, r = inv;
    for (int k = 0; k < 4; ++k) { r = (uint8_t)((r << 1) | (r >> 7)); s ^= r; }
    hs[x] = s ^ 0x63;
  }
}
static void host_expand(const uint8_t key[16], uint32_t rk[44]) {
  uint8_t rcon = 1;
  for (int i = 0; i < 4; ++i) rk[i] = (uint32_t)key[4 * i] << 24 | key[4 * i + 1] << 16 | key[4 * i + 2] << 8 | key[4 * i + 3];
  for (int i = 4; i < 44; ++i) {
    uint32_t t = rk[i - 1];
    if (i % 4 == 0) {
      t = (t << 8) | (t >> 24);
      t = (uint32_t)hs[t >> 24] << 24 | hs[(t >> 16) & 255] << 16 | hs[(t >> 8) & 255] << 8 | hs[t & 255];
      t ^= (uint32_t)rcon << 24;
      rcon = gm(rcon, 2);
    }
    rk[i] = rk[i - 4] ^ t;
  }
}
static void host_aes(const uint32_t rk[44], const uint8_t in[16], uint8_t out[16]) {
  uint8_t s[16];
  for (int i = 0; i < 16; ++i) s[i] = in[i] ^ (uint8_t)(rk[i / 4] >> (24 - 8 * (i % 4)));
  for (int r = 1; r <= 10; ++r) {
    uint8_t t[16];
    for (int c = 0; c < 4; ++c) for (int q = 0; q < 4; ++q) t[q + 4 * c] = hs[s[q + 4 * ((c + q) & 3)]];
    if (r < 10)
      for (int c = 0; c < 4; ++c) {
        uint8_t a0 = t[4 * c], a1 = t[4 * c + 1], a2 = t[4 * c + 2], a3 = t[4 * c + 3];
        s[4 * c] = gm(a0, 2) ^ gm(a1, 3) ^ a2 ^ a3; s[4 * c + 1] = a0 ^ gm(a1, 2) ^ gm(a2, 3) ^ a3;
        s[4 * c + 2] = a0 ^ a1 ^ gm(a2, 2) ^ gm(a3, 3); s[4 * c + 3] = gm(a0, 3) ^ a1 ^ a2 ^ gm(a3, 2);
      }
    else memcpy(s, t, 16);
    for (int i = 0; i < 16; ++i) s[i] ^= (uint8_t)(rk[4 * r + i / 4] >> (24 - 8 * (i % 4)));
  }
  memcpy(out, s, 16);
}

template <class F>
static double best_ms(F&& launch) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  double best = 1e30;
  for (int r = 0; r < 6; ++r) {
    (void)hipEventRecord(e0);
    launch();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (r > 0 && ms < best) best = ms;
  }
  return best;
}

int main() {
  host_sbox();
  uint8_t key[16];
  for (int i = 0; i < 16; ++i) key[i] = (uint8_t)(0x2b + 17 * i);
  uint32_t rk[44];
  host_expand(key, rk);
  std::vector<uint32_t> masks(11 * 128);
  for (int r = 0; r < 11; ++r)
    for (int i = 0; i < 16; ++i) {
      const uint8_t kb = (uint8_t)(rk[4 * r + i / 4] >> (24 - 8 * (i % 4)));
      for (int b = 0; b < 8; ++b) masks[128 * r + 8 * i + b] = ((kb >> (7 - b)) & 1) ? 0xFFFFFFFFu : 0u;
    }
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  uint32_t *d_rk, *d_masks, *d_out, *d_chk;
  CK(hipMalloc(&d_rk, sizeof rk));
  CK(hipMalloc(&d_masks, masks.size() * 4));
  CK(hipMalloc(&d_out, 4096));
  const size_t max_threads = (size_t)cus * 1024 * 4;
  CK(hipMalloc(&d_chk, max_threads * 4));
  CK(hipMemcpy(d_rk, rk, sizeof rk, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_masks, masks.data(), masks.size() * 4, hipMemcpyHostToDevice));

  // correctness: lane 0's blocks vs the host AES
  uint8_t nonce[12] = {0x00, 0x11, 0x22, 0x33, 0x44, 0x55, 0x66, 0x77, 0x88, 0x99, 0xaa, 0xbb};
  std::vector<uint32_t> got(128);
  int bad = 0;
  hipLaunchKernelGGL(ttab_ctr<16>, dim3(1), dim3(1024), 0, 0, d_rk, 32u, d_out, d_chk);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(got.data(), d_out, 512, hipMemcpyDeviceToHost));
  for (int it = 0; it < 32; ++it) {
    uint8_t in[16], want[16];
    memcpy(in, nonce, 12);
    in[12] = 0; in[13] = 0; in[14] = 0; in[15] = (uint8_t)it;
    host_aes(rk, in, want);
    for (int q = 0; q < 4; ++q) {
      const uint32_t w = (uint32_t)want[4 * q] << 24 | want[4 * q + 1] << 16 | want[4 * q + 2] << 8 | want[4 * q + 3];
      if (got[4 * it + q] != w) ++bad;
    }
  }
  printf("ttab check: %s\n", bad ? "MISMATCH" : "ok");
  int bad2 = 0;
  hipLaunchKernelGGL(bs_ctr<4>, dim3(1), dim3(256), 0, 0, d_masks, 1u, d_out, d_chk);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(got.data(), d_out, 512, hipMemcpyDeviceToHost));
  for (int k = 0; k < 32; ++k) {
    uint8_t in[16], want[16];
    memcpy(in, nonce, 12);
    in[12] = 0; in[13] = 0; in[14] = 0; in[15] = (uint8_t)k;  // gl 0, it 0: counter 0 + k
    host_aes(rk, in, want);
    for (int q = 0; q < 4; ++q) {
      const uint32_t w = (uint32_t)want[4 * q] << 24 | want[4 * q + 1] << 16 | want[4 * q + 2] << 8 | want[4 * q + 3];
      if (got[4 * k + q] != w) { if (bad2 < 3) printf("  bs block %d word %d got %08x want %08x\n", k, q, got[4 * k + q], w); ++bad2; }
    }
  }
  printf("bitsliced check: %s\n", bad2 ? "MISMATCH" : "ok");
  if (bad || bad2) return 1;

  // throughput: the same number of keystream blocks per kernel
  const uint32_t it_tt = 256;
  const double tt16 = best_ms([&] { hipLaunchKernelGGL(ttab_ctr<16>, dim3(cus), dim3(1024), 0, 0, d_rk, it_tt, (uint32_t*)nullptr, d_chk); });
  const double blocks_tt = (double)cus * 1024 * it_tt;
  printf("T-table (wide, CTR cache, 16 waves/CU): %.3f ms for %.0f blocks: %.2f Gblock/s = %.1f GiB/s of keystream\n",
         tt16, blocks_tt, blocks_tt / tt16 / 1e6, blocks_tt * 16 / (tt16 * 1e-3) / (1u << 30));
  for (int wgs_per_cu : {2, 3, 4}) {
    const uint32_t it_bs = 8;
    const double ms = best_ms([&] { hipLaunchKernelGGL(bs_ctr<4>, dim3(cus * wgs_per_cu), dim3(256), 0, 0, d_masks, it_bs, (uint32_t*)nullptr, d_chk); });
    const double blocks = (double)cus * wgs_per_cu * 256 * 32 * it_bs;
    printf("bitsliced (BP S-box, no LDS, 4-wave WGs x %d per CU): %.3f ms for %.0f blocks: %.2f Gblock/s = %.1f GiB/s of keystream\n",
           wgs_per_cu, ms, blocks, blocks / ms / 1e6, blocks * 16 / (ms * 1e-3) / (1u << 30));
  }
  return 0;
}
