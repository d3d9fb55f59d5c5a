// Micro-benchmarks that size the design of the packet-protection kernels on gfx950:
//  (1) integer ALU rates: v_mad_u64_u32 (Poly1305 limb products), v_mul_lo_u32, plain add/xor/rotate;
//  (2) HBM streaming shapes: coalesced copy vs one-packet-per-lane copy at 1200-B stride.
// Build: hipcc --offload-arch=gfx950 -O3 -o ubench ubench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void k_mad64(uint32_t* out, uint32_t a0, int iters) {
  uint32_t a = a0 + threadIdx.x;
  uint64_t acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = a + i;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = (uint64_t)(uint32_t)acc[i] * (uint64_t)(a + i) + acc[i];
  }
  uint64_t s = 0;
  for (int i = 0; i < 8; ++i) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s ^ (uint32_t)(s >> 32);
}

__global__ void k_mullo(uint32_t* out, uint32_t a0, int iters) {
  uint32_t a = a0 + threadIdx.x;
  uint32_t acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = a + i;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = acc[i] * (a + 2 * i + 1);
  }
  uint32_t s = 0;
  for (int i = 0; i < 8; ++i) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__device__ __forceinline__ uint32_t rotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

__global__ void k_arx(uint32_t* out, uint32_t a0, int iters) {
  uint32_t x[8];
  for (int i = 0; i < 8; ++i) x[i] = a0 + threadIdx.x * 7 + i;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      x[i] += x[i + 4]; x[i + 4] ^= x[i]; x[i + 4] = rotl(x[i + 4], 7);
    }
  }
  uint32_t s = 0;
  for (int i = 0; i < 8; ++i) s ^= x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_copy_coalesced(const uint4* __restrict__ in, uint4* __restrict__ out, size_t n16) {
  size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) out[i] = in[i];
}

// One packet per lane: lane copies its own L-byte packet in 16-B pieces (aligned).
__global__ void k_copy_perlane(const uint8_t* __restrict__ in, uint8_t* __restrict__ out, int npkt, int L) {
  int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= npkt) return;
  const uint4* src = (const uint4*)(in + (size_t)p * L);
  uint4* dst = (uint4*)(out + (size_t)p * L);
  for (int i = 0; i < L / 16; ++i) dst[i] = src[i];
}

// One packet per lane, 64-B steps (4 x 16B loads) with 4-byte (not 16-byte) alignment, as a
// payload window starting at floor4(payload_start) would be.
__global__ void k_copy_perlane_u4(const uint8_t* __restrict__ in, uint8_t* __restrict__ out, int npkt, int L) {
  int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= npkt) return;
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  const uint8_t* src = in + (size_t)p * L + 12;
  uint8_t* dst = out + (size_t)p * L + 12;
  for (int i = 0; i < (L - 64) / 64; ++i) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      u32x4 v;
      __builtin_memcpy(&v, src + 64 * i + 16 * k, 16);
      __builtin_memcpy(dst + 64 * i + 16 * k, &v, 16);
    }
  }
}

int main() {
  int dev = 0;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, dev));
  printf("device %s CUs %d clock %d kHz\n", prop.gcnArchName, prop.multiProcessorCount, prop.clockRate);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  uint32_t* dout;
  int blocks = 256 * 32, threads = 256;
  CK(hipMalloc(&dout, (size_t)blocks * threads * 4));
  float ms;
  const int iters = 2048;
  double lanes = (double)blocks * threads;
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(k_mad64, dim3(blocks), dim3(threads), 0, 0, dout, 3u, iters);
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_mad64, dim3(blocks), dim3(threads), 0, 0, dout, 3u, iters);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
    printf("mad_u64_u32: %.3f ms, %.2f T lane-ops/s\n", ms, lanes * iters * 8 / (ms * 1e-3) / 1e12);
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_mullo, dim3(blocks), dim3(threads), 0, 0, dout, 3u, iters);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
    printf("mul_lo_u32: %.3f ms, %.2f T lane-ops/s\n", ms, lanes * iters * 8 / (ms * 1e-3) / 1e12);
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_arx, dim3(blocks), dim3(threads), 0, 0, dout, 3u, iters);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
    printf("arx (add,xor,rot): %.3f ms, %.2f T lane-ops/s (3 ops per step)\n", ms, lanes * iters * 12 / (ms * 1e-3) / 1e12);
  }
  const int npkt = 1 << 20, L = 1200;
  size_t bytes = (size_t)npkt * L;
  uint8_t *a, *b;
  CK(hipMalloc(&a, bytes + 256));
  CK(hipMalloc(&b, bytes + 256));
  CK(hipMemset(a, 1, bytes));
  CK(hipMemset(b, 0, bytes));
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_copy_coalesced, dim3(256 * 8), dim3(256), 0, 0, (const uint4*)a, (uint4*)b, bytes / 16);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
    printf("copy coalesced: %.3f ms, %.1f GB/s (R+W)\n", ms, 2.0 * bytes / (ms * 1e-3) / 1e9);
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_copy_perlane, dim3(npkt / 256), dim3(256), 0, 0, a, b, npkt, L);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
    printf("copy per-lane 16B-aligned: %.3f ms, %.1f GB/s (R+W)\n", ms, 2.0 * bytes / (ms * 1e-3) / 1e9);
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_copy_perlane_u4, dim3(npkt / 256), dim3(256), 0, 0, a, b, npkt, L);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
    printf("copy per-lane 4B-aligned 64B steps: %.3f ms, %.1f GB/s (R+W of 1088/1200 B)\n", ms, 2.0 * npkt * 1088 / (ms * 1e-3) / 1e9);
  }
  CK(hipDeviceSynchronize());
  printf("done\n");
  return 0;
}
