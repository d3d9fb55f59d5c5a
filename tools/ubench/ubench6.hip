// Streaming AES-128-GCM seal prototype (gfx950): the product's octet layout (r02: the first cut of the streaming design; r02 measured 1.41 ms
// for 16 waves/CU single blocks, 3.34 ms for block pairs (spills), 1.42 ms for 12 waves/CU pairs) (8 packets x 8 lanes
// per wave, CTR block b on lane b % 8) but WITHOUT LDS packet images — each lane loads its 16-B
// plaintext block straight from HBM into VGPRs (prefetched one iteration ahead), XORs the
// keystream, stores the ciphertext and absorbs it into its GHASH accumulator at once. LDS holds
// only the wide T-table and the GHASH table (72 KiB), so one 16-wave workgroup per CU fits
// (4 waves/SIMD if <= 128 VGPRs) instead of 8 waves with 10-KiB images. Timing only (synthetic
// keys, no HP, no tag store): does the occupancy pay for the HBM-direct access?
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 ubench6.hip -o ubench6
#include "../../milli_quic_amd/csrc/mq_aes.h"

#include <cstdio>
#include <vector>

using namespace mq;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

typedef uint4 __attribute__((aligned(4))) uint4u;

template <int WAVES, bool PAIR>
__global__ __launch_bounds__(64 * WAVES) void proto_seal(uint8_t* __restrict__ arena, uint32_t n, const uint32_t* __restrict__ rkg,
                                                   const uint32_t* __restrict__ h8g, uint32_t plen, uint32_t aad) {
  build_tw(threadIdx.x, blockDim.x);
  uint32_t h8[4] = {h8g[0], h8g[1], h8g[2], h8g[3]};
  build_gh(h8, threadIdx.x, blockDim.x);
  const TwLane L = tw_lane();
  AesRk rk;
  load_rk(rkg, rk);
  const uint32_t lane = threadIdx.x & 63, p = lane >> 3, j = lane & 7, w = threadIdx.x >> 6;
  const uint32_t tiles = n / 8;
  for (uint32_t t = blockIdx.x * WAVES + w; t < tiles; t += gridDim.x * WAVES) {
    const uint32_t pi = t * 8 + p;
    const uint64_t pay = (uint64_t)pi * plen + aad;
    const uint32_t P = plen - aad - 16, nblk = 1 + (P + 15) / 16;
    uint32_t nb[3] = {0x01020304u, pi, pi * 7u};
    const AesCtrCache cc = ctr_cache(RkRegs{rk}, L, nb);
    uint32_t acc[4] = {0, 0, 0, 0};
    const uint32_t iters = (nblk + 7) / 8;
    auto ld = [&](uint32_t b) -> uint4 {
      if (b >= 1 && b < nblk) return *(const uint4u*)(arena + pay + 16ull * (b - 1));
      return make_uint4(0, 0, 0, 0);
    };
    auto use = [&](uint32_t b, const uint32_t (&s)[4], uint4 v) {
      if (b >= 1 && b < nblk) {
        const uint32_t rem = P - 16 * (b - 1);
        uint32_t c[4] = {v.x ^ bswap32(s[0]), v.y ^ bswap32(s[1]), v.z ^ bswap32(s[2]), v.w ^ bswap32(s[3])};
        uint8_t* dst = arena + pay + 16ull * (b - 1);
        if (rem >= 16) {
          *(uint4u*)dst = make_uint4(c[0], c[1], c[2], c[3]);
        } else {
          for (uint32_t k = 0; k < rem; ++k) dst[k] = (uint8_t)(c[k >> 2] >> (8 * (k & 3)));
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[q] ^= refl(c[q] & byte_mask((int)rem, q));
      }
      gh_mul_tab(acc);
    };
    {
      uint4 v0 = ld(j);
      for (uint32_t it = 0; it < iters; ++it) {
        const uint32_t b = j + 8 * it;
        const uint4 n0 = ld(b + 8);
        uint32_t a[4];
        aes128_ctr1(RkRegs{rk}, L, cc, b == 0 ? 1u : b + 1, a);
        use(b, a, v0);
        v0 = n0;
      }
    }
    // octet reduction and a tag store by lane 0 (keeps the work live)
    uint32_t y[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) y[q] = oct_xor(acc[q]);
    if (j == 0) *(uint4u*)(arena + pay + P) = make_uint4(y[0], y[1], y[2], y[3]);
  }
}

template <int WAVES, bool PAIR>
static int run(const char* name, uint8_t* arena, uint32_t n, const uint32_t* rk, const uint32_t* h8, int cus) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float best = 1e9;
  for (int r = 0; r < 12; ++r) {
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL((proto_seal<WAVES, PAIR>), dim3(cus), dim3(64 * WAVES), 0, 0, arena, n, rk, h8, 1200u, 20u);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (r >= 2 && ms < best) best = ms;
  }
  printf("%-28s %.4f ms  %.1f GiB/s (2L per packet)\n", name, best, 2.0 * 1200 * n / (best * 1e-3) / (1u << 30));
  return 0;
}

int main() {
  const uint32_t n = 1u << 20;
  uint8_t* arena;
  uint32_t *rk, *h8;
  CK(hipMalloc(&arena, (size_t)n * 1200 + 64));
  CK(hipMemset(arena, 0x5a, (size_t)n * 1200 + 64));
  std::vector<uint32_t> hrk(44), hh(4);
  for (int i = 0; i < 44; ++i) hrk[i] = 0x9e3779b9u * (i + 1);
  for (int i = 0; i < 4; ++i) hh[i] = 0x85ebca6bu * (i + 3);
  CK(hipMalloc(&rk, 44 * 4));
  CK(hipMalloc(&h8, 16));
  CK(hipMemcpy(rk, hrk.data(), 44 * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(h8, hh.data(), 16, hipMemcpyHostToDevice));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  run<16, false>("16 waves/CU, single block", arena, n, rk, h8, cus);
  run<8, false>("8 waves/CU, single block", arena, n, rk, h8, cus);
  return 0;
}
