// mq_partition.hip — device-side partition of a mixed batch ("descriptor-only
// partition by suite"), refined by packet length so that each tile's eight packets need about the
// same number of keystream iterations and MAC blocks.
//
// Output: list[0..c0) = AES-128-GCM descriptor indices, list[cap..cap+c1) = everything else
// (ChaCha20 rows and invalid key ids, which the ChaCha kernel rejects with a status); counts[0] =
// c0, counts[1] = c1, cap = mq_partition_list_cap(n). Inside each suite list the packets are
// grouped by 64-B length class, longest class first (the tail of the grid then runs the short
// tiles); inside a class the order is the descriptor order per wave of 64 descriptors. Every class
// starts on a tile boundary, and a long class puts only as many packets in a tile as fit the
// LDS image at its longest length; the rest of the tile's entries are holes (kListHole), which
// the tile kernels skip. Packets are independent and processed in place, so
// the order changes nothing but the tile composition: a tile runs as long as its longest packet,
// and a uniformly mixed 64-1350-B batch otherwise pays for 8 x its maximum in nearly every tile.
//
// Counting sort in three launches: per-block class histograms (class-major), one exclusive scan of
// the histograms, scatter.
#include "mq_tile.h"

using namespace mq;

namespace {
constexpr int kPartThreads = 256;
constexpr int kPartItems = 16;  // descriptors per thread
constexpr int kPartBlock = kPartThreads * kPartItems;
constexpr uint32_t kLenClasses = 32;  // per suite: min(len / 64, 31), longest first
constexpr uint32_t kClasses = 2 * kLenClasses;
constexpr uint32_t kBudgetChunks = kDataBudget / 16;

// class = suite * kLenClasses + (31 - length bucket); suite 0 = AES-128-GCM, 1 = the rest
__device__ __forceinline__ uint32_t part_class(const KeyRow* kt, uint32_t n_rows, const mq_pkt_desc& d) {
  const bool aes = d.key_id < n_rows && kt[d.key_id].suite == MQ_SUITE_AES128GCM;
  const uint32_t b = min(d.len >> 6, kLenClasses - 1);
  return (aes ? 0u : kLenClasses) + (kLenClasses - 1 - b);
}

// Packets per tile of a class: as many as fit the LDS image budget at the class's longest
// length and worst alignment (4b + 5 chunks), so the class's tiles stay on the staged path;
// classes that would need fewer than kMinPpt per tile (and the open-ended last one) keep 8 and
// take the direct path.
constexpr uint32_t kMinPpt = 5;
__device__ __forceinline__ uint32_t class_ppt(uint32_t c) {
  const uint32_t b = kLenClasses - 1 - (c % kLenClasses);
  if (b == kLenClasses - 1) return kPktsPerTile;
  const uint32_t x = kBudgetChunks / (4 * b + 5);
  return x >= kPktsPerTile ? kPktsPerTile : (x >= kMinPpt ? x : kPktsPerTile);
}
}  // namespace

// Entries of one suite's list: every class segment is whole tiles of 8 entries, holes included.
uint32_t mq_partition_list_cap(uint32_t n) {
  const uint64_t c = ((uint64_t)n * kPktsPerTile + kMinPpt - 1) / kMinPpt + kPktsPerTile * kLenClasses;
  return (uint32_t)((c + kPktsPerTile - 1) & ~(uint64_t)(kPktsPerTile - 1));
}

extern "C" __global__ __launch_bounds__(kPartThreads) void mq_part_count_kernel(
    const KeyRow* __restrict__ kt, uint32_t n_rows, const mq_pkt_desc* __restrict__ desc, uint32_t n,
    uint32_t nblocks, uint32_t* __restrict__ hist) {
  __shared__ uint32_t s_cnt[kClasses];
  if (threadIdx.x < kClasses) s_cnt[threadIdx.x] = 0;
  __syncthreads();
  for (int k = 0; k < kPartItems; ++k) {
    const uint32_t i = blockIdx.x * kPartBlock + k * kPartThreads + threadIdx.x;
    if (i < n) atomicAdd(&s_cnt[part_class(kt, n_rows, desc[i])], 1u);
  }
  __syncthreads();
  if (threadIdx.x < kClasses) hist[(size_t)threadIdx.x * nblocks + blockIdx.x] = s_cnt[threadIdx.x];
}

// Single workgroup: per class, the exclusive scan of its per-block counts (in place: the rank of
// the block's first packet inside the class); then the class segments (whole tiles) are laid out
// suite by suite: seg[c] = first list entry of class c (suite 1 starts at `cap`), counts[s] =
// entries of suite s's list, holes included.
extern "C" __global__ __launch_bounds__(1024) void mq_part_scan_kernel(uint32_t* __restrict__ hist,
                                                                        uint32_t nblocks, uint32_t cap,
                                                                        uint32_t* __restrict__ counts,
                                                                        uint32_t* __restrict__ seg) {
  __shared__ uint32_t s_tot[kClasses];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (uint32_t c = wave; c < kClasses; c += 1024 / kWave) {
    uint32_t* h = hist + (size_t)c * nblocks;
    uint32_t carry = 0;
    for (uint32_t k0 = 0; k0 < nblocks; k0 += kWave) {
      const uint32_t k = k0 + lane;
      const uint32_t v = k < nblocks ? h[k] : 0u;
      uint32_t x = v;  // inclusive wave scan
#pragma unroll
      for (int d = 1; d < kWave; d <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, d, kWave);
        if (lane >= d) x += y;
      }
      if (k < nblocks) h[k] = carry + x - v;
      carry += (uint32_t)__shfl((int)x, kWave - 1, kWave);
    }
    if (lane == 0) s_tot[c] = carry;
  }
  __syncthreads();
  if (threadIdx.x < 2) {
    const uint32_t s = threadIdx.x;
    uint32_t e = 0;
    for (uint32_t c = s * kLenClasses; c < (s + 1) * kLenClasses; ++c) {
      seg[c] = s * cap + e;
      const uint32_t ppt = class_ppt(c);
      e += kPktsPerTile * ((s_tot[c] + ppt - 1) / ppt);
    }
    counts[s] = e;
  }
}

extern "C" __global__ __launch_bounds__(kPartThreads) void mq_part_scatter_kernel(
    const KeyRow* __restrict__ kt, uint32_t n_rows, const mq_pkt_desc* __restrict__ desc, uint32_t n,
    uint32_t nblocks, const uint32_t* __restrict__ hist, const uint32_t* __restrict__ seg,
    uint32_t* __restrict__ list) {
  __shared__ uint32_t s_rank[kClasses];
  const int lane = threadIdx.x & 63;
  if (threadIdx.x < kClasses) s_rank[threadIdx.x] = hist[(size_t)threadIdx.x * nblocks + blockIdx.x];
  __syncthreads();
  const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  for (int k = 0; k < kPartItems; ++k) {
    const uint32_t i = blockIdx.x * kPartBlock + k * kPartThreads + threadIdx.x;
    const bool in = i < n;
    const uint32_t c = in ? part_class(kt, n_rows, desc[i]) : 0u;
    // lanes of this wave with the same class (6 ballots), rank among them = peers below
    uint64_t peers = __ballot(in);
#pragma unroll
    for (int bit = 0; bit < 6; ++bit) {
      const uint64_t b = __ballot((c >> bit) & 1u);
      peers &= ((c >> bit) & 1u) ? b : ~b;
    }
    const uint32_t rank = (uint32_t)__popcll(peers & below);
    uint32_t base = 0;
    if (in && rank == 0) base = atomicAdd(&s_rank[c], (uint32_t)__popcll(peers));
    // the leader (lowest lane of the peer group) hands its base to the group
    const int leader = in ? __ffsll((unsigned long long)peers) - 1 : lane;
    base = (uint32_t)__shfl((int)base, leader, kWave);
    if (in) {
      const uint32_t r = base + rank, ppt = class_ppt(c);
      list[seg[c] + kPktsPerTile * (r / ppt) + r % ppt] = i;
    }
  }
}

hipError_t mq_launch_partition(const KeyRow* kt, uint32_t n_rows, const mq_pkt_desc* desc, uint32_t n,
                               uint32_t* list, uint32_t* hist, uint32_t* counts, hipStream_t s) {
  const uint32_t nblocks = (n + kPartBlock - 1) / kPartBlock;
  if (nblocks == 0) return hipMemsetAsync(counts, 0, 2 * sizeof(uint32_t), s);
  const uint32_t cap = mq_partition_list_cap(n);
  uint32_t* seg = counts + 2;
  hipError_t e = hipMemsetAsync(list, 0xff, sizeof(uint32_t) * 2 * (size_t)cap, s);  // holes
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(mq_part_count_kernel, dim3(nblocks), dim3(kPartThreads), 0, s, kt, n_rows, desc, n,
                     nblocks, hist);
  hipLaunchKernelGGL(mq_part_scan_kernel, dim3(1), dim3(1024), 0, s, hist, nblocks, cap, counts, seg);
  hipLaunchKernelGGL(mq_part_scatter_kernel, dim3(nblocks), dim3(kPartThreads), 0, s, kt, n_rows, desc, n,
                     nblocks, hist, seg, list);
  return hipGetLastError();
}

// list (2 x cap entries) | class histograms (kClasses per block) | 2 totals + kClasses segment
// starts, 256-B aligned pieces
static size_t part_align(size_t b) { return (b + 255) & ~(size_t)255; }

size_t mq_partition_workspace(uint32_t n) {
  const size_t nblocks = (n + kPartBlock - 1) / kPartBlock;
  return part_align(sizeof(uint32_t) * 2 * (size_t)mq_partition_list_cap(n)) +
         part_align(sizeof(uint32_t) * kClasses * nblocks) + part_align(sizeof(uint32_t) * (2 + kClasses));
}

// offsets of the pieces inside the partition workspace
void mq_partition_layout(uint32_t n, size_t* hist_off, size_t* counts_off) {
  const size_t nblocks = (n + kPartBlock - 1) / kPartBlock;
  *hist_off = part_align(sizeof(uint32_t) * 2 * (size_t)mq_partition_list_cap(n));
  *counts_off = *hist_off + part_align(sizeof(uint32_t) * kClasses * nblocks);
}
