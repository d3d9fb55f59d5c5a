// VALU issue cost per wave-instruction on gfx950 for the ops the ChaCha20 rounds and the
// Poly1305 Horner steps are made of: 8 independent chains per lane (throughput) or 1 chain
// (dependent-issue latency), at 1 or 4 waves per SIMD. Timing only.
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 ubench7.hip -o ubench7
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int kIters = 2048;

// OP(x, y): x = op(x, y, ...), one instruction
#define OP_ADD(x, y) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(y))
#define OP_XOR(x, y) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x) : "v"(y))
#define OP_ALIGN(x, y) asm volatile("v_alignbit_b32 %0, %0, %0, 20" : "+v"(x))
#define OP_PERM(x, y) asm volatile("v_perm_b32 %0, %0, %0, %1" : "+v"(x) : "v"(y))
#define OP_ADD3(x, y) asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(x) : "v"(y))
#define OP_XAD(x, y) asm volatile("v_xad_u32 %0, %0, %1, %1" : "+v"(x) : "v"(y))
#define OP_MULLO(x, y) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x) : "v"(y))
#define OP_MULHI(x, y) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x) : "v"(y))
#define OP_MAD24(x, y) asm volatile("v_mad_u32_u24 %0, %0, %1, %1" : "+v"(x) : "v"(y))
#define OP_MULHI24(x, y) asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(x) : "v"(y))
#define OP_LSHLADD(x, y) asm volatile("v_lshl_add_u32 %0, %0, 3, %1" : "+v"(x) : "v"(y))

template <int CHAINS>
struct Regs { uint32_t v[CHAINS]; };

#define KERNEL32(NAME, OP)                                                                  \
  template <int CHAINS>                                                                     \
  __global__ void NAME(uint32_t* out, uint32_t seed) {                                      \
    uint32_t r[CHAINS];                                                                     \
    const uint32_t y = seed ^ threadIdx.x;                                                  \
    _Pragma("unroll") for (int c = 0; c < CHAINS; ++c) r[c] = threadIdx.x * (c + 3);        \
    for (int i = 0; i < kIters; ++i) {                                                      \
      _Pragma("unroll") for (int u = 0; u < 8 / CHAINS * 4; ++u)                            \
        _Pragma("unroll") for (int c = 0; c < CHAINS; ++c) OP(r[c], y);                     \
    }                                                                                       \
    uint32_t s = 0;                                                                         \
    _Pragma("unroll") for (int c = 0; c < CHAINS; ++c) s ^= r[c];                           \
    if (s == 0x12345678u) out[0] = s;                                                       \
  }

KERNEL32(k_add, OP_ADD)
KERNEL32(k_xor, OP_XOR)
KERNEL32(k_align, OP_ALIGN)
KERNEL32(k_perm, OP_PERM)
KERNEL32(k_add3, OP_ADD3)
KERNEL32(k_xad, OP_XAD)
KERNEL32(k_mullo, OP_MULLO)
KERNEL32(k_mulhi, OP_MULHI)
KERNEL32(k_mad24, OP_MAD24)
KERNEL32(k_mulhi24, OP_MULHI24)
KERNEL32(k_lshladd, OP_LSHLADD)

// 64-bit results
template <int CHAINS>
__global__ void k_mad64(uint32_t* out, uint32_t seed) {
  uint64_t r[CHAINS];
  const uint32_t y = seed ^ threadIdx.x;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) r[c] = threadIdx.x * (c + 3);
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int u = 0; u < 8 / CHAINS * 4; ++u)
#pragma unroll
      for (int c = 0; c < CHAINS; ++c)
        asm volatile("v_mad_u64_u32 %0, s[40:41], %1, %1, %0" : "+v"(r[c]) : "v"(y) : "s40", "s41");
  }
  uint64_t s = 0;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) s ^= r[c];
  if (s == 0x12345678u) out[0] = (uint32_t)s;
}

template <int CHAINS>
__global__ void k_fma64(uint32_t* out, uint32_t seed) {
  double r[CHAINS];
  const double y = 1.0 + 1e-9 * (seed ^ threadIdx.x);
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) r[c] = threadIdx.x * (c + 3);
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int u = 0; u < 8 / CHAINS * 4; ++u)
#pragma unroll
      for (int c = 0; c < CHAINS; ++c) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(r[c]) : "v"(y));
  }
  double s = 0;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) s += r[c];
  if (s == 1.2345) out[0] = 1;
}

typedef void (*Kern)(uint32_t*, uint32_t);

static int run(const char* name, Kern k8, Kern k1, int cus, uint32_t* out) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double clk = 2.4e9;
  printf("%-18s", name);
  for (int chains : {8, 1}) {
    Kern k = chains == 8 ? k8 : k1;
    for (int wps : {1, 4}) {  // waves per SIMD
      float best = 1e9;
      for (int r = 0; r < 5; ++r) {
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(k, dim3(cus * wps), dim3(256), 0, 0, out, 7u);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r >= 1 && ms < best) best = ms;
      }
      // per SIMD: wps waves x kIters x 32 instructions
      const double inst = (double)wps * kIters * 32;
      printf("  ch%d w%d %6.2f cyc", chains, wps, best * 1e-3 * clk / inst);
    }
  }
  printf("\n");
  return 0;
}

#define RUN(NAME, K) run(NAME, K<8>, K<1>, cus, out)

int main() {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  uint32_t* out;
  CK(hipMalloc(&out, 64));
  hipLaunchKernelGGL(k_add<8>, dim3(cus), dim3(256), 0, 0, out, 7u);  // warm-up
  CK(hipDeviceSynchronize());
  printf("cycles per wave-instruction per SIMD at 2.4 GHz (ch = independent chains per lane, w = waves/SIMD)\n");
  RUN("v_add_u32", k_add);
  RUN("v_xor_b32", k_xor);
  RUN("v_alignbit_b32", k_align);
  RUN("v_perm_b32", k_perm);
  RUN("v_add3_u32", k_add3);
  RUN("v_xad_u32", k_xad);
  RUN("v_lshl_add_u32", k_lshladd);
  RUN("v_mul_lo_u32", k_mullo);
  RUN("v_mul_hi_u32", k_mulhi);
  RUN("v_mad_u32_u24", k_mad24);
  RUN("v_mul_hi_u32_u24", k_mulhi24);
  RUN("v_mad_u64_u32", k_mad64);
  RUN("v_fma_f64", k_fma64);
  return 0;
}
