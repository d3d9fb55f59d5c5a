// Streaming shapes with software prefetch (next step's loads issued before this step's stores),
// 1M x 1200-B packets, one wave = 64 packets.
//   MODE 0: per-lane (lane = packet), 64 B per step as 4 x 16 B
//   MODE 1: 64-B pieces (4 lanes per piece, 16 packets per instruction)
//   MODE 2: contiguous (wave's 76.8-KB span read 1 KiB per instruction) — upper bound
// plus an ALU load of `alu` dependent ARX ops per step to emulate ChaCha work.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int L = 1200;
constexpr int STEPS = 18;

template <int MODE>
__device__ __forceinline__ size_t addr(size_t p0, int lane, int s, int k) {
  if (MODE == 0) return (p0 + lane) * L + (size_t)s * 64 + 16 * k;
  if (MODE == 1) return (p0 + k * 16 + lane / 4) * L + (size_t)s * 64 + 16 * (lane % 4);
  return p0 * L + ((size_t)s * 4 + k) * 1024 + 16 * lane;
}

template <int MODE>
__global__ __launch_bounds__(256) void k_stream(const uint8_t* __restrict__ in, uint8_t* __restrict__ out, int npkt, int alu) {
  int lane = threadIdx.x & 63;
  int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  size_t p0 = (size_t)wave * 64;
  if (p0 >= (size_t)npkt) return;
  u32x4 cur[4], nxt[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) __builtin_memcpy(&cur[k], in + addr<MODE>(p0, lane, 0, k), 16);
  uint32_t x = lane, y = 7;
  for (int s = 0; s < STEPS; ++s) {
    if (s + 1 < STEPS) {
#pragma unroll
      for (int k = 0; k < 4; ++k) __builtin_memcpy(&nxt[k], in + addr<MODE>(p0, lane, s + 1, k), 16);
    }
    for (int i = 0; i < alu; ++i) { x += y; y ^= x; y = (y << 7) | (y >> 25); }
#pragma unroll
    for (int k = 0; k < 4; ++k) { u32x4 v = cur[k]; v.x ^= y; __builtin_memcpy(out + addr<MODE>(p0, lane, s, k), &v, 16); }
#pragma unroll
    for (int k = 0; k < 4; ++k) cur[k] = nxt[k];
  }
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
  for (int alu : {0, 100, 300}) {
    for (int mode = 0; mode < 3; ++mode) {
      auto launch = [&] {
        if (mode == 0) hipLaunchKernelGGL(k_stream<0>, grid, blk, 0, 0, a, b, npkt, alu);
        if (mode == 1) hipLaunchKernelGGL(k_stream<1>, grid, blk, 0, 0, a, b, npkt, alu);
        if (mode == 2) hipLaunchKernelGGL(k_stream<2>, grid, blk, 0, 0, a, b, npkt, alu);
      };
      launch();
      CK(hipEventRecord(e0));
      for (int i = 0; i < 5; ++i) launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ms /= 5;
      printf("alu %3d mode %d (%s): %.3f ms  %.0f GB/s\n", alu, mode,
             mode == 0 ? "per-lane" : mode == 1 ? "64B pieces" : "contiguous", ms, moved / (ms * 1e-3) / 1e9);
    }
  }
  CK(hipDeviceSynchronize());
  printf("done\n");
  return 0;
}
