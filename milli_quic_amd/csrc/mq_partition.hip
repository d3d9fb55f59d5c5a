// mq_partition.hip — device-side partition of a mixed batch ("descriptor-only
// partition by suite"), refined by packet length so that each tile's eight packets need about the
// same number of keystream iterations and MAC blocks.
//
// Output: list[0..c0) = AES-128-GCM descriptor indices, list[cap..cap+c1) = everything else
// (ChaCha20 rows and invalid key ids, which the ChaCha kernel rejects with a status); counts[0] =
// c0, counts[1] = c1, cap = mq_partition_list_cap(n). Inside each suite list the packets are
// grouped by 64-B length class, longest class first (the tail of the grid then runs the short
// tiles); inside a class the order is the descriptor order per wave of 64 descriptors. Every class
// starts on a tile boundary, and a long ChaCha class puts only as many packets in a tile as fit
// the LDS image at its longest length; the rest of the tile's entries are holes (kListHole), which
// the tile kernels skip. Packets are independent and processed in place, so
// the order changes nothing but the tile composition: a tile runs as long as its longest packet,
// and a uniformly mixed 64-1350-B batch otherwise pays for 8 x its maximum in nearly every tile.
//
// AES packets are further split by key: the batch's majority AES key (Boyer-Moore vote; in a
// server's mix the 1-RTT key of the busiest path) goes first in the AES list, so its tiles are
// key-uniform and the multi-key AES kernels run their GHASH through the LDS table of that key's
// H^8 (counts[2] = its row, or 0xFFFFFFFF). With no majority the vote's candidate is just some
// key: results are the same, only fewer tiles use the table.
//
// Launches: per-block votes, one vote reduction, per-block class histograms (class-major), one
// exclusive scan of the histograms, scatter.
#include "mq_tile.h"

using namespace mq;

namespace {
constexpr int kPartThreads = 256;
constexpr int kPartItems = 16;  // descriptors per thread
constexpr int kPartBlock = kPartThreads * kPartItems;
constexpr uint32_t kLenClasses = 32;  // per group: min(len / 64, 31), longest first
constexpr uint32_t kGroups = 3;       // AES with the hot key, other AES (both: list 0), the rest (list 1)
constexpr uint32_t kClasses = kGroups * kLenClasses;
constexpr uint32_t kBudgetChunks = kDataBudget / 16;
constexpr uint32_t kNoKey = 0xFFFFFFFFu;

__device__ __forceinline__ bool is_aes(const KeyRow* kt, uint32_t n_rows, const mq_pkt_desc& d) {
  return d.key_id < n_rows && kt[d.key_id].suite == MQ_SUITE_AES128GCM;
}

// class = group * kLenClasses + (31 - length bucket)
__device__ __forceinline__ uint32_t part_class(const KeyRow* kt, uint32_t n_rows, uint32_t hot,
                                               const mq_pkt_desc& d) {
  const uint32_t g = is_aes(kt, n_rows, d) ? (d.key_id == hot ? 0u : 1u) : 2u;
  const uint32_t b = min(d.len >> 6, kLenClasses - 1);
  return g * kLenClasses + (kLenClasses - 1 - b);
}

// Boyer-Moore majority pairs (candidate, count); combining any partition of the input in any
// order keeps the majority element if there is one
__device__ __forceinline__ uint2 vote_join(uint2 a, uint2 b) {
  if (a.x == b.x) return make_uint2(a.x, a.y + b.y);
  return a.y >= b.y ? make_uint2(a.x, a.y - b.y) : make_uint2(b.x, b.y - a.y);
}

__device__ __forceinline__ uint2 block_vote(uint2 v) {  // 256 threads
  __shared__ uint2 s_v[kPartThreads];
  s_v[threadIdx.x] = v;
  __syncthreads();
  for (int d = kPartThreads / 2; d > 0; d >>= 1) {
    if ((int)threadIdx.x < d) s_v[threadIdx.x] = vote_join(s_v[threadIdx.x], s_v[threadIdx.x + d]);
    __syncthreads();
  }
  return s_v[0];
}

// Packets per tile of a class: AES tiles stream from HBM (no LDS image), so always 8. ChaCha
// tiles take as many as fit the LDS image budget at the class's longest length and worst
// alignment (4b + 5 chunks), so the class's tiles stay on the staged path; classes that would
// need fewer than kMinPpt per tile (and the open-ended last one) keep 8 and take the direct path.
constexpr uint32_t kMinPpt = 5;
__device__ __forceinline__ uint32_t class_ppt(uint32_t c) {
  if (c < 2 * kLenClasses) return kPktsPerTile;  // groups 0 and 1: AES
  const uint32_t b = kLenClasses - 1 - (c % kLenClasses);
  if (b == kLenClasses - 1) return kPktsPerTile;
  const uint32_t x = kBudgetChunks / (4 * b + 5);
  return x >= kPktsPerTile ? kPktsPerTile : (x >= kMinPpt ? x : kPktsPerTile);
}
}  // namespace

// Entries of one suite's list: every class segment is whole tiles of 8 entries, holes included.
// A class of c packets at p <= 8 per tile takes 8 * ceil(c / p) < 8c / kMinPpt + 8 entries, so a
// list of n packets spread over its classes needs at most 8n / kMinPpt + 8 per class. List 0 holds
// two class groups (hot AES key, other AES keys: 2 * kLenClasses classes), list 1 one; the cap
// covers the larger.
uint32_t mq_partition_list_cap(uint32_t n) {
  const uint64_t c = ((uint64_t)n * kPktsPerTile + kMinPpt - 1) / kMinPpt + kPktsPerTile * 2 * kLenClasses;
  return (uint32_t)((c + kPktsPerTile - 1) & ~(uint64_t)(kPktsPerTile - 1));
}

extern "C" __global__ __launch_bounds__(kPartThreads) void mq_part_vote_kernel(
    const KeyRow* __restrict__ kt, uint32_t n_rows, const mq_pkt_desc* __restrict__ desc, uint32_t n,
    uint2* __restrict__ votes) {
  uint2 v = make_uint2(kNoKey, 0u);
  for (int k = 0; k < kPartItems; ++k) {
    const uint32_t i = blockIdx.x * kPartBlock + k * kPartThreads + threadIdx.x;
    if (i < n) {
      const mq_pkt_desc d = desc[i];
      if (is_aes(kt, n_rows, d)) v = vote_join(v, make_uint2(d.key_id, 1u));
    }
  }
  v = block_vote(v);
  if (threadIdx.x == 0) votes[blockIdx.x] = v;
}

// Single workgroup: the batch's vote; meta[0] = the hot key row (kNoKey if no AES packet)
extern "C" __global__ __launch_bounds__(kPartThreads) void mq_part_vote_reduce_kernel(
    const uint2* __restrict__ votes, uint32_t nblocks, uint32_t* __restrict__ meta) {
  uint2 v = make_uint2(kNoKey, 0u);
  for (uint32_t k = threadIdx.x; k < nblocks; k += kPartThreads) v = vote_join(v, votes[k]);
  v = block_vote(v);
  if (threadIdx.x == 0) meta[0] = v.y ? v.x : kNoKey;
}

extern "C" __global__ __launch_bounds__(kPartThreads) void mq_part_count_kernel(
    const KeyRow* __restrict__ kt, uint32_t n_rows, const mq_pkt_desc* __restrict__ desc, uint32_t n,
    uint32_t nblocks, const uint32_t* __restrict__ hot_p, uint32_t* __restrict__ hist) {
  __shared__ uint32_t s_cnt[kClasses];
  if (threadIdx.x < kClasses) s_cnt[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t hot = *hot_p;
  for (int k = 0; k < kPartItems; ++k) {
    const uint32_t i = blockIdx.x * kPartBlock + k * kPartThreads + threadIdx.x;
    if (i < n) atomicAdd(&s_cnt[part_class(kt, n_rows, hot, desc[i])], 1u);
  }
  __syncthreads();
  if (threadIdx.x < kClasses) hist[(size_t)threadIdx.x * nblocks + blockIdx.x] = s_cnt[threadIdx.x];
}

// Single workgroup: per class, the exclusive scan of its per-block counts (in place: the rank of
// the block's first packet inside the class); then the class segments (whole tiles) are laid out
// list by list (groups 0 and 1: list 0, group 2: list 1 at `cap`): seg[c] = first list entry of
// class c, counts[s] = entries of list s, holes included.
// Latency-bound work (a few thousand counts): each wave owns kClasses / 16 classes and issues
// all their loads before any scan (4 consecutive blocks per lane per 256-block chunk), so the
// kernel waits on memory once instead of once per class (r01: 26 us per partition, rocprof).
constexpr int kScanWaves = 16, kClassesPerWave = kClasses / kScanWaves;
static_assert(kClasses % kScanWaves == 0, "classes per scan wave");
extern "C" __global__ __launch_bounds__(64 * kScanWaves) void mq_part_scan_kernel(uint32_t* __restrict__ hist,
                                                                                 uint32_t nblocks, uint32_t cap,
                                                                                 uint32_t* __restrict__ counts,
                                                                                 uint32_t* __restrict__ seg) {
  __shared__ uint32_t s_tot[kClasses];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t carry[kClassesPerWave];
#pragma unroll
  for (int q = 0; q < kClassesPerWave; ++q) carry[q] = 0;
  for (uint32_t k0 = 0; k0 < nblocks; k0 += 4 * kWave) {  // one chunk for n <= 2^20 descriptors
    uint32_t v[kClassesPerWave][4];
#pragma unroll
    for (int q = 0; q < kClassesPerWave; ++q) {
      const uint32_t* h = hist + (size_t)(wave + kScanWaves * q) * nblocks;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const uint32_t k = k0 + 4 * lane + e;
        v[q][e] = k < nblocks ? h[k] : 0u;
      }
    }
#pragma unroll
    for (int q = 0; q < kClassesPerWave; ++q) {
      uint32_t* h = hist + (size_t)(wave + kScanWaves * q) * nblocks;
      const uint32_t lsum = v[q][0] + v[q][1] + v[q][2] + v[q][3];
      const uint32_t incl = wave_incl_scan(lsum);
      uint32_t run = carry[q] + incl - lsum;  // exclusive prefix of this lane's first block
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const uint32_t k = k0 + 4 * lane + e;
        if (k < nblocks) h[k] = run;
        run += v[q][e];
      }
      carry[q] += (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    }
  }
  if (lane == 0) {
#pragma unroll
    for (int q = 0; q < kClassesPerWave; ++q) s_tot[wave + kScanWaves * q] = carry[q];
  }
  __syncthreads();
  if (threadIdx.x < 2) {
    const uint32_t s = threadIdx.x;
    const uint32_t c0 = s == 0 ? 0u : 2 * kLenClasses, c1 = s == 0 ? 2 * kLenClasses : kClasses;
    uint32_t e = 0;
    for (uint32_t c = c0; c < c1; ++c) {
      seg[c] = s * cap + e;
      const uint32_t ppt = class_ppt(c);
      e += kPktsPerTile * ((s_tot[c] + ppt - 1) / ppt);
    }
    // mq_partition_list_cap bounds e; the clamp only keeps a broken bound from running a suite
    // kernel over the other list
    counts[s] = min(e, cap);
  }
}

extern "C" __global__ __launch_bounds__(kPartThreads) void mq_part_scatter_kernel(
    const KeyRow* __restrict__ kt, uint32_t n_rows, const mq_pkt_desc* __restrict__ desc, uint32_t n,
    uint32_t nblocks, const uint32_t* __restrict__ hot_p, const uint32_t* __restrict__ hist,
    const uint32_t* __restrict__ seg, uint32_t* __restrict__ list) {
  __shared__ uint32_t s_rank[kClasses];
  const uint32_t hot = *hot_p;
  const int lane = threadIdx.x & 63;
  if (threadIdx.x < kClasses) s_rank[threadIdx.x] = hist[(size_t)threadIdx.x * nblocks + blockIdx.x];
  __syncthreads();
  const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  for (int k = 0; k < kPartItems; ++k) {
    const uint32_t i = blockIdx.x * kPartBlock + k * kPartThreads + threadIdx.x;
    const bool in = i < n;
    const uint32_t c = in ? part_class(kt, n_rows, hot, desc[i]) : 0u;
    // lanes of this wave with the same class (7 ballots), rank among them = peers below
    uint64_t peers = __ballot(in);
#pragma unroll
    for (int bit = 0; bit < 7; ++bit) {
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
  uint32_t* hot = counts + 2;  // meta: counts[0..1] | hot row | pad | seg[kClasses]
  uint32_t* seg = counts + 4;
  uint2* votes = (uint2*)(hist + (size_t)kClasses * nblocks);
  hipError_t e = hipMemsetAsync(list, 0xff, sizeof(uint32_t) * 2 * (size_t)cap, s);  // holes
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(mq_part_vote_kernel, dim3(nblocks), dim3(kPartThreads), 0, s, kt, n_rows, desc, n, votes);
  hipLaunchKernelGGL(mq_part_vote_reduce_kernel, dim3(1), dim3(kPartThreads), 0, s, votes, nblocks, hot);
  hipLaunchKernelGGL(mq_part_count_kernel, dim3(nblocks), dim3(kPartThreads), 0, s, kt, n_rows, desc, n,
                     nblocks, hot, hist);
  hipLaunchKernelGGL(mq_part_scan_kernel, dim3(1), dim3(64 * kScanWaves), 0, s, hist, nblocks, cap, counts, seg);
  hipLaunchKernelGGL(mq_part_scatter_kernel, dim3(nblocks), dim3(kPartThreads), 0, s, kt, n_rows, desc, n,
                     nblocks, hot, hist, seg, list);
  return hipGetLastError();
}

// list (2 x cap entries) | class histograms (kClasses per block) + votes (2 words per block) |
// meta (2 totals, hot row, pad, kClasses segment starts), 256-B aligned pieces
static size_t part_align(size_t b) { return (b + 255) & ~(size_t)255; }

size_t mq_partition_workspace(uint32_t n) {
  const size_t nblocks = (n + kPartBlock - 1) / kPartBlock;
  return part_align(sizeof(uint32_t) * 2 * (size_t)mq_partition_list_cap(n)) +
         part_align(sizeof(uint32_t) * (kClasses + 2) * nblocks) + part_align(sizeof(uint32_t) * (4 + kClasses));
}

// offsets of the pieces inside the partition workspace
void mq_partition_layout(uint32_t n, size_t* hist_off, size_t* counts_off) {
  const size_t nblocks = (n + kPartBlock - 1) / kPartBlock;
  *hist_off = part_align(sizeof(uint32_t) * 2 * (size_t)mq_partition_list_cap(n));
  *counts_off = *hist_off + part_align(sizeof(uint32_t) * (kClasses + 2) * nblocks);
}
