// mq_partition.hip — stable device-side partition of a mixed batch by cipher suite, so that each
// suite kernel sees wave-uniform work ("descriptor-only partition by suite").
// Output: list[0..c0) = AES-128-GCM descriptor indices, list[n..n+c1) = everything else
// (ChaCha20 rows and invalid key ids, which the ChaCha kernel rejects with a status);
// counts[0] = c0, counts[1] = c1. Descriptor order is preserved inside each list, so tiles of
// adjacent packets stay adjacent in HBM.
#include "mq_device.h"

using namespace mq;

namespace {
constexpr int kPartThreads = 256;
constexpr int kPartItems = 4;  // descriptors per thread
constexpr int kPartBlock = kPartThreads * kPartItems;

__device__ __forceinline__ bool is_aes(const KeyRow* kt, uint32_t n_rows, const mq_pkt_desc* desc,
                                       uint32_t i) {
  const uint32_t k = desc[i].key_id;
  return k < n_rows && kt[k].suite == MQ_SUITE_AES128GCM;
}
}  // namespace

extern "C" __global__ __launch_bounds__(kPartThreads) void mq_part_count_kernel(
    const KeyRow* __restrict__ kt, uint32_t n_rows, const mq_pkt_desc* __restrict__ desc, uint32_t n,
    uint32_t* __restrict__ block_counts) {
  __shared__ uint32_t s_aes;
  if (threadIdx.x == 0) s_aes = 0;
  __syncthreads();
  uint32_t mine = 0;
  for (int k = 0; k < kPartItems; ++k) {
    const uint32_t i = blockIdx.x * kPartBlock + k * kPartThreads + threadIdx.x;
    if (i < n && is_aes(kt, n_rows, desc, i)) ++mine;
  }
  atomicAdd(&s_aes, mine);
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t lo = blockIdx.x * kPartBlock;
    const uint32_t cnt = n - lo < (uint32_t)kPartBlock ? n - lo : (uint32_t)kPartBlock;
    block_counts[2 * blockIdx.x] = s_aes;
    block_counts[2 * blockIdx.x + 1] = cnt - s_aes;
  }
}

// Single workgroup: exclusive scan of the per-block counts (in place) and the two totals.
extern "C" __global__ __launch_bounds__(1024) void mq_part_scan_kernel(uint32_t* __restrict__ block_counts,
                                                                        uint32_t nblocks,
                                                                        uint32_t* __restrict__ counts) {
  __shared__ uint32_t s_tot[2][1024];
  const uint32_t per = (nblocks + 1023) / 1024;
  const uint32_t lo = threadIdx.x * per, hi = min(lo + per, nblocks);
  uint32_t a = 0, b = 0;
  for (uint32_t k = lo; k < hi; ++k) { a += block_counts[2 * k]; b += block_counts[2 * k + 1]; }
  s_tot[0][threadIdx.x] = a;
  s_tot[1][threadIdx.x] = b;
  __syncthreads();
  for (uint32_t d = 1; d < 1024; d <<= 1) {
    uint32_t x0 = threadIdx.x >= d ? s_tot[0][threadIdx.x - d] : 0u;
    uint32_t x1 = threadIdx.x >= d ? s_tot[1][threadIdx.x - d] : 0u;
    __syncthreads();
    s_tot[0][threadIdx.x] += x0;
    s_tot[1][threadIdx.x] += x1;
    __syncthreads();
  }
  uint32_t ra = s_tot[0][threadIdx.x] - a, rb = s_tot[1][threadIdx.x] - b;
  for (uint32_t k = lo; k < hi; ++k) {
    const uint32_t ca = block_counts[2 * k], cb = block_counts[2 * k + 1];
    block_counts[2 * k] = ra;
    block_counts[2 * k + 1] = rb;
    ra += ca;
    rb += cb;
  }
  if (threadIdx.x == 1023) { counts[0] = s_tot[0][1023]; counts[1] = s_tot[1][1023]; }
}

extern "C" __global__ __launch_bounds__(kPartThreads) void mq_part_scatter_kernel(
    const KeyRow* __restrict__ kt, uint32_t n_rows, const mq_pkt_desc* __restrict__ desc, uint32_t n,
    const uint32_t* __restrict__ block_offsets, uint32_t* __restrict__ list) {
  __shared__ uint32_t s_wave[kPartThreads / kWave][2];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t base_a = block_offsets[2 * blockIdx.x], base_b = block_offsets[2 * blockIdx.x + 1];
  for (int k = 0; k < kPartItems; ++k) {
    const uint32_t i = blockIdx.x * kPartBlock + k * kPartThreads + threadIdx.x;
    const bool in = i < n;
    const bool aes = in && is_aes(kt, n_rows, desc, i);
    const uint64_t ma = __ballot(aes), mb = __ballot(in && !aes);
    const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    if (lane == 0) { s_wave[wave][0] = __popcll(ma); s_wave[wave][1] = __popcll(mb); }
    __syncthreads();
    uint32_t pa = base_a, pb = base_b, ta = 0, tb = 0;
    for (int w = 0; w < kPartThreads / kWave; ++w) {
      if (w < wave) { pa += s_wave[w][0]; pb += s_wave[w][1]; }
      ta += s_wave[w][0];
      tb += s_wave[w][1];
    }
    if (aes) list[pa + __popcll(ma & below)] = i;
    else if (in) list[n + pb + __popcll(mb & below)] = i;
    base_a += ta;
    base_b += tb;
    __syncthreads();
  }
}

hipError_t mq_launch_partition(const KeyRow* kt, uint32_t n_rows, const mq_pkt_desc* desc, uint32_t n,
                               uint32_t* list, uint32_t* block_counts, uint32_t* counts,
                               hipStream_t s) {
  const uint32_t nblocks = (n + kPartBlock - 1) / kPartBlock;
  if (nblocks == 0) return hipMemsetAsync(counts, 0, 2 * sizeof(uint32_t), s);
  hipLaunchKernelGGL(mq_part_count_kernel, dim3(nblocks), dim3(kPartThreads), 0, s, kt, n_rows, desc, n,
                     block_counts);
  hipLaunchKernelGGL(mq_part_scan_kernel, dim3(1), dim3(1024), 0, s, block_counts, nblocks, counts);
  hipLaunchKernelGGL(mq_part_scatter_kernel, dim3(nblocks), dim3(kPartThreads), 0, s, kt, n_rows, desc, n,
                     block_counts, list);
  return hipGetLastError();
}

size_t mq_partition_workspace(uint32_t n) {
  const size_t nblocks = (n + kPartBlock - 1) / kPartBlock;
  // list (2n indices) + block counts (2 per block) + 2 totals, 256-B aligned pieces
  auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
  return al(sizeof(uint32_t) * 2 * (size_t)n) + al(sizeof(uint32_t) * 2 * nblocks) + 256;
}
