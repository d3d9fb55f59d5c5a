// Lane-per-packet streaming microbenchmark (gfx950): each lane walks its own 1200-B packet in
// 64-B steps (4 x 16-B global loads to VGPRs, one ChaCha20 block, XOR, 4 x 16-B stores), the
// access pattern of a packet-per-lane ChaCha20 kernel without LDS staging. Variants: memory
// only, compute only, both; n packets at a 1200-B stride.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__device__ __forceinline__ uint32_t rotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
#define QR(a, b, c, d) a += b; d ^= a; d = rotl(d, 16); c += d; b ^= c; b = rotl(b, 12); a += b; d ^= a; d = rotl(d, 8); c += d; b ^= c; b = rotl(b, 7);

__device__ __forceinline__ void block(const uint32_t* key, uint32_t ctr, uint32_t n0, uint32_t n1, uint32_t n2, uint32_t (&o)[16]) {
  uint32_t x0 = 0x61707865u, x1 = 0x3320646eu, x2 = 0x79622d32u, x3 = 0x6b206574u;
  uint32_t x4 = key[0], x5 = key[1], x6 = key[2], x7 = key[3], x8 = key[4], x9 = key[5], x10 = key[6], x11 = key[7];
  uint32_t x12 = ctr, x13 = n0, x14 = n1, x15 = n2;
#pragma unroll 2
  for (int i = 0; i < 10; ++i) {
    QR(x0, x4, x8, x12) QR(x1, x5, x9, x13) QR(x2, x6, x10, x14) QR(x3, x7, x11, x15)
    QR(x0, x5, x10, x15) QR(x1, x6, x11, x12) QR(x2, x7, x8, x13) QR(x3, x4, x9, x14)
  }
  o[0] = x0 + 0x61707865u; o[1] = x1 + 0x3320646eu; o[2] = x2 + 0x79622d32u; o[3] = x3 + 0x6b206574u;
  o[4] = x4 + key[0]; o[5] = x5 + key[1]; o[6] = x6 + key[2]; o[7] = x7 + key[3];
  o[8] = x8 + key[4]; o[9] = x9 + key[5]; o[10] = x10 + key[6]; o[11] = x11 + key[7];
  o[12] = x12 + ctr; o[13] = x13 + n0; o[14] = x14 + n1; o[15] = x15 + n2;
}

template <int MODE>  // 0 memory only, 1 compute only, 2 both
__global__ __launch_bounds__(256) void k_stream(uint8_t* arena, uint32_t n, const uint32_t* __restrict__ keyp, uint32_t* sink) {
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  uint32_t key[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) key[k] = keyp[k];
  uint4* pk = (uint4*)(arena + (size_t)p * 1200);
  uint32_t acc = 0;
  for (uint32_t s = 0; s < 18; ++s) {
    uint32_t ks[16];
    if (MODE != 0) block(key, s + 1, p, 7, 9, ks);
    else {
#pragma unroll
      for (int k = 0; k < 16; ++k) ks[k] = s * 0x9e3779b9u + k;
    }
    if (MODE != 1) {
      uint4 d[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) d[q] = pk[4 * s + q];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        d[q].x ^= ks[4 * q]; d[q].y ^= ks[4 * q + 1]; d[q].z ^= ks[4 * q + 2]; d[q].w ^= ks[4 * q + 3];
        pk[4 * s + q] = d[q];
      }
    } else {
#pragma unroll
      for (int k = 0; k < 16; ++k) acc ^= ks[k];
    }
  }
  if (MODE == 1 && acc == 0x12345678u) sink[0] = acc;
}

// MODE 3 (both) / 4 (memory only): per 64-B step the wave loads the step's segment of all 64
// packets with 4 LDS-DMA instructions (lane l of instruction q: packet 16q + l/4, 16-B part l%4,
// so 4 lanes read 64 contiguous bytes), each lane reads its packet's 64 B from LDS, XORs, writes
// them back to LDS, and the wave stores the segment with 4 quad-coalesced 16-B stores.
template <int MODE>
__global__ __launch_bounds__(256) void k_stage(uint8_t* arena, uint32_t n, const uint32_t* __restrict__ keyp, uint32_t* sink) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[4][4096];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint8_t* my = lds[w];
  const uint32_t p0 = (blockIdx.x * blockDim.x + (threadIdx.x & ~63));  // wave's first packet
  const uint32_t p = p0 + lane;
  if (p0 >= n) return;
  uint32_t key[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) key[k] = keyp[k];
  for (uint32_t s = 0; s < 18; ++s) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t pp = p0 + 16 * q + (lane >> 2);
      const uint8_t* src = arena + (size_t)pp * 1200 + 64 * s + 16 * (lane & 3);
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)(my + 1024 * q), 16, 0, 0);
    }
    uint32_t ks[16];
    if (MODE == 3) block(key, s + 1, p, 7, 9, ks);
    else {
#pragma unroll
      for (int k = 0; k < 16; ++k) ks[k] = s * 0x9e3779b9u + k;
    }
    __builtin_amdgcn_s_waitcnt(0);  // vmcnt(0) & lgkmcnt(0)
    __builtin_amdgcn_wave_barrier();
    uint4 d[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) d[i] = *(const uint4*)(my + 64 * lane + 16 * i);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      d[i].x ^= ks[4 * i]; d[i].y ^= ks[4 * i + 1]; d[i].z ^= ks[4 * i + 2]; d[i].w ^= ks[4 * i + 3];
      *(uint4*)(my + 64 * lane + 16 * i) = d[i];
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t pp = p0 + 16 * q + (lane >> 2);
      *(uint4*)(arena + (size_t)pp * 1200 + 64 * s + 16 * (lane & 3)) = *(const uint4*)(my + 1024 * q + 16 * lane);
    }
    __builtin_amdgcn_wave_barrier();
  }
}

// MODE 5 (both) / 6 (memory only): as 3/4 with 128-B steps (two ChaCha blocks per lane per
// step, 8 LDS-DMA instructions: lane l of instruction q = packet 8q + l/8, part l%8), double-
// buffered: step s+1's DMA is issued before step s is processed.
template <int MODE>
__global__ __launch_bounds__(128) void k_stage2(uint8_t* arena, uint32_t n, const uint32_t* __restrict__ keyp, uint32_t* sink) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[2][2][8192];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint32_t p0 = (blockIdx.x * blockDim.x + (threadIdx.x & ~63));
  const uint32_t p = p0 + lane;
  if (p0 >= n) return;
  uint32_t key[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) key[k] = keyp[k];
  auto issue = [&](uint32_t s) {
    uint8_t* my = lds[w][s & 1];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const uint32_t pp = p0 + 8 * q + (lane >> 3);
      const uint8_t* src = arena + (size_t)pp * 1200 + 128 * s + 16 * (lane & 7);
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)(my + 1024 * q), 16, 0, 0);
    }
  };
  issue(0);
  for (uint32_t s = 0; s < 9; ++s) {
    uint8_t* my = lds[w][s & 1];
    uint32_t ks[32];
    if (MODE == 5) {
      uint32_t a[16], b[16];
      block(key, 2 * s + 1, p, 7, 9, a);
      block(key, 2 * s + 2, p, 7, 9, b);
#pragma unroll
      for (int k = 0; k < 16; ++k) { ks[k] = a[k]; ks[16 + k] = b[k]; }
    } else {
#pragma unroll
      for (int k = 0; k < 32; ++k) ks[k] = s * 0x9e3779b9u + k;
    }
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    if (s + 1 < 9) issue(s + 1);  // next step lands while this one is processed
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      uint4 d = *(const uint4*)(my + 128 * lane + 16 * ((i + lane) & 7));
      const int k = 4 * ((i + lane) & 7);
      d.x ^= ks[k]; d.y ^= ks[k + 1]; d.z ^= ks[k + 2]; d.w ^= ks[k + 3];
      *(uint4*)(my + 128 * lane + 16 * ((i + lane) & 7)) = d;
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const uint32_t pp = p0 + 8 * q + (lane >> 3);
      *(uint4*)(arena + (size_t)pp * 1200 + 128 * s + 16 * (lane & 7)) = *(const uint4*)(my + 1024 * q + 16 * lane);
    }
    __builtin_amdgcn_wave_barrier();
  }
}

template <int MODE>
float run(uint8_t* arena, uint32_t n, const uint32_t* key, uint32_t* sink) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  auto kern = MODE >= 5 ? k_stage2<MODE> : (MODE >= 3 ? k_stage<MODE> : k_stream<MODE>);
  const int bs = MODE >= 5 ? 128 : 256;
  hipLaunchKernelGGL(kern, dim3((n + bs - 1) / bs), dim3(bs), 0, 0, arena, n, key, sink);
  hipDeviceSynchronize();
  float best = 1e9;
  for (int r = 0; r < 5; ++r) {
    hipEventRecord(e0);
    hipLaunchKernelGGL(kern, dim3((n + bs - 1) / bs), dim3(bs), 0, 0, arena, n, key, sink);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) best = ms;
  }
  return best;
}

int main() {
  const uint32_t n = 1u << 20;
  uint8_t* arena; uint32_t *key, *sink;
  CK(hipMalloc(&arena, (size_t)n * 1200 + 4096));
  CK(hipMalloc(&key, 64)); CK(hipMalloc(&sink, 64));
  CK(hipMemset(arena, 1, (size_t)n * 1200));
  CK(hipMemset(key, 3, 64));
  const double bytes = (double)n * 18 * 64 * 2;  // read + write
  float m0 = run<0>(arena, n, key, sink), m1 = run<1>(arena, n, key, sink), m2 = run<2>(arena, n, key, sink);
  printf("memory only : %.3f ms  %.0f GB/s (R+W)\n", m0, bytes / m0 / 1e6);
  printf("compute only: %.3f ms\n", m1);
  printf("both        : %.3f ms  %.0f GB/s (R+W)\n", m2, bytes / m2 / 1e6);
  float m4 = run<4>(arena, n, key, sink), m3 = run<3>(arena, n, key, sink);
  printf("staged mem  : %.3f ms  %.0f GB/s (R+W)\n", m4, bytes / m4 / 1e6);
  printf("staged both : %.3f ms  %.0f GB/s (R+W)\n", m3, bytes / m3 / 1e6);
  float m6 = run<6>(arena, n, key, sink), m5 = run<5>(arena, n, key, sink);
  const double b2 = (double)n * 9 * 128 * 2;
  printf("128B dbuf mem : %.3f ms  %.0f GB/s (R+W)\n", m6, b2 / m6 / 1e6);
  printf("128B dbuf both: %.3f ms  %.0f GB/s (R+W)\n", m5, b2 / m5 / 1e6);
  return 0;
}
