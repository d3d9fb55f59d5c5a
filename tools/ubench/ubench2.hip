// Streaming shapes for one-packet-per-lane kernels (1M x 1200-B packets):
//  - "pieces": a wave-instruction covers 1024/PIECE packets with PIECE contiguous bytes each;
//  - "lds": 64-B pieces through an LDS transpose so each lane ends up with its own packet's
//    64-B window (what the ChaCha20-Poly1305 kernel needs), then the reverse for the store.
// Build: hipcc --offload-arch=gfx950 -O3 -o ubench2 ubench2.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int L = 1200;
constexpr int STEPS = 18;  // 18 x 64 B = 1152 B per packet streamed

template <int PIECE, int OFF>
__global__ __launch_bounds__(256) void k_pieces(const uint8_t* __restrict__ in, uint8_t* __restrict__ out, int npkt) {
  constexpr int LPP = PIECE / 16;        // lanes per piece
  constexpr int PPI = 64 / LPP;          // packets per instruction
  constexpr int NI = 64 / PPI;           // instructions per 64 packets per PIECE step
  int lane = threadIdx.x & 63;
  int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  size_t p0 = (size_t)wave * 64;
  if (p0 >= (size_t)npkt) return;
  for (int s = 0; s < STEPS * 64 / PIECE; ++s) {
    u32x4 v[NI];
#pragma unroll
    for (int k = 0; k < NI; ++k) {
      size_t p = p0 + k * PPI + lane / LPP;
      const uint8_t* src = in + p * L + OFF + (size_t)s * PIECE + 16 * (lane % LPP);
      __builtin_memcpy(&v[k], src, 16);
    }
#pragma unroll
    for (int k = 0; k < NI; ++k) {
      size_t p = p0 + k * PPI + lane / LPP;
      uint8_t* dst = out + p * L + OFF + (size_t)s * PIECE + 16 * (lane % LPP);
      __builtin_memcpy(dst, &v[k], 16);
    }
  }
}

// LDS transpose staging: per wave 64 rows x 80 B (64 B window + 16 B pad).
template <int OFF>
__global__ __launch_bounds__(256) void k_lds(const uint8_t* __restrict__ in, uint8_t* __restrict__ out, int npkt) {
  __shared__ u32x4 lds[4][64 * 5];
  int lane = threadIdx.x & 63;
  int w = threadIdx.x >> 6;
  int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  size_t p0 = (size_t)wave * 64;
  if (p0 >= (size_t)npkt) return;
  u32x4* row = &lds[w][0];
  for (int s = 0; s < STEPS; ++s) {
    u32x4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      size_t p = p0 + k * 16 + lane / 4;
      __builtin_memcpy(&v[k], in + p * L + OFF + (size_t)s * 64 + 16 * (lane % 4), 16);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) row[(k * 16 + lane / 4) * 5 + (lane % 4)] = v[k];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    u32x4 d[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) d[c] = row[lane * 5 + c];
#pragma unroll
    for (int c = 0; c < 4; ++c) d[c] ^= (u32x4){0x01010101u, 0x02020202u, 0x03030303u, (uint32_t)s};
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int c = 0; c < 4; ++c) row[lane * 5 + c] = d[c];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = row[(k * 16 + lane / 4) * 5 + (lane % 4)];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      size_t p = p0 + k * 16 + lane / 4;
      __builtin_memcpy(out + p * L + OFF + (size_t)s * 64 + 16 * (lane % 4), &v[k], 16);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

template <typename F>
float timeit(F f, hipEvent_t e0, hipEvent_t e1) {
  f();
  hipEventRecord(e0);
  for (int i = 0; i < 5; ++i) f();
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms / 5;
}

int main() {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int npkt = 1 << 20;
  size_t bytes = (size_t)npkt * L;
  uint8_t *a, *b;
  CK(hipMalloc(&a, bytes + 256));
  CK(hipMalloc(&b, bytes + 256));
  CK(hipMemset(a, 1, bytes));
  CK(hipMemset(b, 0, bytes));
  double moved = 2.0 * npkt * STEPS * 64;
  dim3 grid(npkt / 256), blk(256);
  float ms;
#define RUN(name, ...) ms = timeit([&] { hipLaunchKernelGGL(__VA_ARGS__, grid, blk, 0, 0, a, b, npkt); }, e0, e1); \
  printf("%-28s %.3f ms  %.0f GB/s\n", name, ms, moved / (ms * 1e-3) / 1e9);
  RUN("pieces 16B aligned", (k_pieces<16, 0>));
  RUN("pieces 64B aligned", (k_pieces<64, 0>));
  RUN("pieces 64B +12", (k_pieces<64, 12>));
  RUN("pieces 128B aligned", (k_pieces<128, 0>));
  RUN("pieces 128B +12", (k_pieces<128, 12>));
  RUN("pieces 256B aligned", (k_pieces<256, 0>));
  RUN("lds 64B aligned", (k_lds<0>));
  RUN("lds 64B +12", (k_lds<12>));
  CK(hipDeviceSynchronize());
  printf("done\n");
  return 0;
}
