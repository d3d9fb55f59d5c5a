// Poly1305 Horner step in three radices: instruction counts of the lean step, from
// the gfx950 code object, plus a CPU check of all three against 128-bit arithmetic.
//   p26  — the product's step (mq_device.h: radix 2^26, 5 limbs, general multiplier r^8)
//   p32c — radix 2^32 with a CLAMPED multiplier (r itself: r1..r3 multiples of 4, so 2^128 folds as
//          5/4 * r_i without leaving the integers; OpenSSL's 32-bit poly1305_blocks form)
//   p32g — radix 2^32 with a GENERAL multiplier (r^8 mod p: no clamping), product normalised and
//          re-aligned at bit 130 before the x5 fold
// Build + count (no GPU needed): tools/ubench/poly_radix.sh. Diagnostic only, not product code.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define HD __host__ __device__ __forceinline__

// ---- radix 2^26 (as mq_device.h p26_mul, block absorbed first) --------------------------------
struct P26 { uint32_t l[5]; };
struct P26m { uint32_t r[5], s[4]; };
HD void p26_absorb(P26& h, uint32_t t0, uint32_t t1, uint32_t t2, uint32_t t3, uint32_t hibit) {
  h.l[0] += t0 & 0x3ffffff;
  h.l[1] += ((t0 >> 26) | (t1 << 6)) & 0x3ffffff;
  h.l[2] += ((t1 >> 20) | (t2 << 12)) & 0x3ffffff;
  h.l[3] += ((t2 >> 14) | (t3 << 18)) & 0x3ffffff;
  h.l[4] += (t3 >> 8) | (hibit << 24);
}
HD void p26_mul(P26& h, const P26m& m) {
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

// ---- radix 2^32: h = h0..h3 + h4 * 2^128 (h4 small) -------------------------------------------
struct P32 { uint32_t w[5]; };
HD void p32_absorb(P32& h, uint32_t t0, uint32_t t1, uint32_t t2, uint32_t t3, uint32_t hibit) {
  uint64_t c = (uint64_t)h.w[0] + t0; h.w[0] = (uint32_t)c;
  c = (c >> 32) + h.w[1] + t1; h.w[1] = (uint32_t)c;
  c = (c >> 32) + h.w[2] + t2; h.w[2] = (uint32_t)c;
  c = (c >> 32) + h.w[3] + t3; h.w[3] = (uint32_t)c;
  h.w[4] += (uint32_t)(c >> 32) + hibit;
}
// partial reduction of d0..d3 (64-bit column sums) and top word h4: c = h4 >> 2 folds as 5c
HD void p32_carry(P32& h, uint64_t d0, uint64_t d1, uint64_t d2, uint64_t d3, uint32_t h4) {
  d1 += d0 >> 32; d2 += d1 >> 32; d3 += d2 >> 32;
  h4 += (uint32_t)(d3 >> 32);
  const uint32_t c = (h4 >> 2) + (h4 & ~3u);  // 5 * (h4 >> 2)
  h4 &= 3u;
  uint64_t t = (uint64_t)(uint32_t)d0 + c; h.w[0] = (uint32_t)t;
  t = (t >> 32) + (uint32_t)d1; h.w[1] = (uint32_t)t;
  t = (t >> 32) + (uint32_t)d2; h.w[2] = (uint32_t)t;
  t = (t >> 32) + (uint32_t)d3; h.w[3] = (uint32_t)t;
  h.w[4] = h4 + (uint32_t)(t >> 32);
}
// clamped multiplier r (r0 < 2^28, r1..r3 < 2^28 and = 0 mod 4), s_i = r_i + (r_i >> 2)
struct P32c { uint32_t r[4], s[3]; };
HD void p32c_mul(P32& h, const P32c& m) {
  const uint32_t h0 = h.w[0], h1 = h.w[1], h2 = h.w[2], h3 = h.w[3], h4 = h.w[4];
  const uint64_t d0 = (uint64_t)h0 * m.r[0] + (uint64_t)h1 * m.s[2] + (uint64_t)h2 * m.s[1] + (uint64_t)h3 * m.s[0];
  const uint64_t d1 = (uint64_t)h0 * m.r[1] + (uint64_t)h1 * m.r[0] + (uint64_t)h2 * m.s[2] + (uint64_t)h3 * m.s[1] + (uint64_t)h4 * m.s[0];
  const uint64_t d2 = (uint64_t)h0 * m.r[2] + (uint64_t)h1 * m.r[1] + (uint64_t)h2 * m.r[0] + (uint64_t)h3 * m.s[2] + (uint64_t)h4 * m.s[1];
  const uint64_t d3 = (uint64_t)h0 * m.r[3] + (uint64_t)h1 * m.r[2] + (uint64_t)h2 * m.r[1] + (uint64_t)h3 * m.r[0] + (uint64_t)h4 * m.s[2];
  p32_carry(h, d0, d1, d2, d3, h4 * m.r[0]);
}
// general multiplier b = b0..b3 + b4 * 2^128 (b4 <= 3: a reduced element)
struct P32g { uint32_t b[5]; };
HD void p32g_mul(P32& h, const P32g& m) {
  // schoolbook columns k = 0..8 of sum h_i b_j 2^(32(i+j)), as 64-bit sums with carries kept apart
  uint64_t c[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  uint32_t hi[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};  // carries out of the 64-bit column sums
#pragma unroll
  for (int i = 0; i < 5; ++i)
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      const uint64_t p = (uint64_t)h.w[i] * m.b[j];
      const uint64_t s = c[i + j] + p;
      hi[i + j] += s < p;
      c[i + j] = s;
    }
  // normalise into 32-bit words w0..w8 (value < 2^262)
  uint32_t w[9];
  uint64_t carry = 0;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const uint64_t lo = (c[k] & 0xffffffffu) + (carry & 0xffffffffu);
    w[k] = (uint32_t)lo;
    carry = (c[k] >> 32) + ((uint64_t)hi[k] << 32) + (carry >> 32) + (lo >> 32);
  }
  // split at bit 130: L = w0..w4 (low 2 bits of w4), H = bits 130.. ; result L + 5 H (partial)
  uint32_t H[5];
#pragma unroll
  for (int k = 0; k < 4; ++k) H[k] = (w[4 + k] >> 2) | (w[5 + k] << 30);
  H[4] = w[8] >> 2;
  uint64_t t = (uint64_t)w[0] + (uint64_t)H[0] * 5u; h.w[0] = (uint32_t)t;
  t = (t >> 32) + w[1] + (uint64_t)H[1] * 5u; h.w[1] = (uint32_t)t;
  t = (t >> 32) + w[2] + (uint64_t)H[2] * 5u; h.w[2] = (uint32_t)t;
  t = (t >> 32) + w[3] + (uint64_t)H[3] * 5u; h.w[3] = (uint32_t)t;
  uint32_t h4 = (uint32_t)(t >> 32) + (w[4] & 3u) + H[4] * 5u;
  // second fold: without it h4 grows by ~b4 per step (the product's bits >= 130 carry h4 * b)
  const uint32_t c2 = (h4 >> 2) + (h4 & ~3u);
  h4 &= 3u;
  t = (uint64_t)h.w[0] + c2; h.w[0] = (uint32_t)t;
  t = (t >> 32) + h.w[1]; h.w[1] = (uint32_t)t;
  t = (t >> 32) + h.w[2]; h.w[2] = (uint32_t)t;
  t = (t >> 32) + h.w[3]; h.w[3] = (uint32_t)t;
  h.w[4] = h4 + (uint32_t)(t >> 32);
}

// ---- kernels: the lean loop over n blocks (counted from the code object) -----------------------
#define LOOP_BODY(ABSORB, MUL)                                                                     \
  for (uint32_t i = 0; i < n; ++i) {                                                              \
    const uint4 v = blk[i * 64u + threadIdx.x];                                                   \
    ABSORB(h, v.x, v.y, v.z, v.w, 1u);                                                            \
    MUL(h, m);                                                                                    \
  }
extern "C" __global__ void k_p26(const uint4* blk, uint32_t n, P26m m, uint32_t* out) {
  P26 h{};
  asm volatile("; LOOP_START p26");
  LOOP_BODY(p26_absorb, p26_mul)
  asm volatile("; LOOP_END p26");
  for (int k = 0; k < 5; ++k) out[threadIdx.x * 5 + k] = h.l[k];
}
extern "C" __global__ void k_p32c(const uint4* blk, uint32_t n, P32c m, uint32_t* out) {
  P32 h{};
  asm volatile("; LOOP_START p32c");
  LOOP_BODY(p32_absorb, p32c_mul)
  asm volatile("; LOOP_END p32c");
  for (int k = 0; k < 5; ++k) out[threadIdx.x * 5 + k] = h.w[k];
}
extern "C" __global__ void k_p32g(const uint4* blk, uint32_t n, P32g m, uint32_t* out) {
  P32 h{};
  asm volatile("; LOOP_START p32g");
  LOOP_BODY(p32_absorb, p32g_mul)
  asm volatile("; LOOP_END p32g");
  for (int k = 0; k < 5; ++k) out[threadIdx.x * 5 + k] = h.w[k];
}

// ---- CPU check: the forms run on the host; poly_radix.sh recomputes every result with Python ints ----
static uint64_t rng_state = 0x9e3779b97f4a7c15ull;
static uint32_t rnd() { rng_state ^= rng_state << 13; rng_state ^= rng_state >> 7; rng_state ^= rng_state << 17; return (uint32_t)rng_state; }
static void put(const char* tag, const uint32_t* w, int n) {
  std::printf("%s", tag);
  for (int k = 0; k < n; ++k) std::printf(" %u", w[k]);
  std::printf("\n");
}

int main() {
  for (int trial = 0; trial < 200; ++trial) {
    // clamped r (RFC 8439 2.5) and a general multiplier g (random, reduced: g4 <= 3)
    const uint32_t r[4] = {rnd() & 0x0fffffffu, rnd() & 0x0ffffffcu, rnd() & 0x0ffffffcu, rnd() & 0x0ffffffcu};
    const uint32_t g[5] = {rnd(), rnd(), rnd(), rnd(), rnd() & 3u};
    P26m m26{}, g26{};
    auto limbs26 = [](const uint32_t* w, int nw, uint32_t (&l)[5]) {
      for (int i = 0; i < 5; ++i) {
        const int bit = 26 * i, wi = bit / 32, sh = bit % 32;
        uint64_t v = (uint64_t)(wi < nw ? w[wi] : 0u) >> sh;
        if (wi + 1 < nw) v |= (uint64_t)w[wi + 1] << (32 - sh);
        l[i] = (uint32_t)(v & 0x3ffffff);
      }
    };
    limbs26(r, 4, m26.r);
    limbs26(g, 5, g26.r);
    for (int i = 0; i < 4; ++i) { m26.s[i] = m26.r[i + 1] * 5; g26.s[i] = g26.r[i + 1] * 5; }
    P32c mc{{r[0], r[1], r[2], r[3]}, {r[1] + (r[1] >> 2), r[2] + (r[2] >> 2), r[3] + (r[3] >> 2)}};
    P32g mg{{g[0], g[1], g[2], g[3], g[4]}};
    P26 h26{}, h26g{};
    P32 h32c{}, h32g{};
    put("T r", r, 4);
    put("T g", g, 5);
    for (int b = 0; b < 40; ++b) {
      const uint32_t t[4] = {rnd(), rnd(), rnd(), rnd()};
      put("B", t, 4);
      p26_absorb(h26, t[0], t[1], t[2], t[3], 1); p26_mul(h26, m26);
      p26_absorb(h26g, t[0], t[1], t[2], t[3], 1); p26_mul(h26g, g26);
      p32_absorb(h32c, t[0], t[1], t[2], t[3], 1); p32c_mul(h32c, mc);
      p32_absorb(h32g, t[0], t[1], t[2], t[3], 1); p32g_mul(h32g, mg);
    }
    put("H p26", h26.l, 5);
    put("H p26g", h26g.l, 5);
    put("H p32c", h32c.w, 5);
    put("H p32g", h32g.w, 5);
  }
  return 0;
}
