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
// AES packets are further split by key, so that the multi-key AES kernels find key-uniform
// tiles (they then multiply through a GHASH table of that key's H^8 instead of the bit-holed
// product): the batch's majority AES key (Boyer-Moore vote over a 4096-descriptor sample; in a
// server's mix the 1-RTT key of the busiest path; counts[2] = its row, or 0xFFFFFFFF) goes
// first, by length class; then, when
// the key table is small enough for one counter per (row, 128-B length class) in the workspace
// ("keyed" layout), every other AES key's packets follow key by key, each key's segment longest
// class first and padded to whole tiles. Otherwise the other keys share length classes as the
// majority key does. With no majority the vote's candidate is just some key: results are the
// same either way, only the tile composition changes.
//
// Launches: fill + sliced sample vote (mq_part_init_kernel); class counts and, keyed, per-(row,
// class) counts and ranks, with the lists' layout by the last block (mq_part_count_kernel);
// scatter from the count kernel's per-packet codes. (r02 start: eight operations with a full vote
// pass, ~126 us per mixed 2^20-packet partition.)
#include "mq_tile.h"
#include "mq_opts.h"

#include <cstdlib>

using namespace mq;

namespace {
// 1024-thread blocks of 4 descriptors per thread: 16 waves per CU hide the latency of the
// dependent loads and atomics (r02: 256 x 16 ran one wave per SIMD)
constexpr int kPartThreads = 1024;
constexpr int kPartItems = 4;  // descriptors per thread
constexpr int kPartBlock = kPartThreads * kPartItems;
constexpr uint32_t kLenClasses = 32;  // per group: min(len / 64, 31), longest first
constexpr uint32_t kGroups = 3;       // AES with the hot key, other AES (both: list 0), the rest (list 1)
constexpr uint32_t kClasses = kGroups * kLenClasses;
constexpr uint32_t kBudgetChunks = kDataBudget / 16;
constexpr uint32_t kNoKey = 0xFFFFFFFFu;
constexpr uint32_t kKeyClasses = 16;  // keyed layout: per row, min(len / 128, 15), longest first
// skip_unkeyed (the receive composite's AEAD passes, mq_host.cpp): descriptors without a valid key
// row are in no list (their statuses are never written; mq_recv.hip reads only attempted ones).
// live (receive passes, may be null): a device word counting the pass's keyed descriptors; when it
// is 0 every kernel returns at once and the scan publishes empty lists, so a pass with nothing to
// open costs a few launches instead of four passes over the batch's descriptors (r04: ~110 us per
// empty pass, four such passes per receive batch, profiles/r04k2_kernel_trace_recv.csv).
__device__ __forceinline__ bool pass_empty(const uint32_t* live) { return live && *live == 0; }

// Diagnostic phase stamps (-DMQ_STAMPS build only, tools/part_count_stamps.py): thread 0 of each
// block records s_memrealtime (100 MHz, one clock for all XCDs) at phase boundaries into
// buf[row * 8 + slot]; count kernel rows 0 .. grid-1, scatter rows grid .. 2 grid-1.
#ifdef MQ_STAMPS
static __device__ uint64_t* mq_part_stamp_buf;
#define MQ_PSTAMP(row, slot)                                                        \
  do {                                                                              \
    __builtin_amdgcn_sched_barrier(0);                                              \
    uint64_t _t = __builtin_amdgcn_s_memrealtime();                                 \
    if (threadIdx.x == 0 && mq_part_stamp_buf) mq_part_stamp_buf[(size_t)(row) * 8 + (slot)] = _t; \
    __builtin_amdgcn_sched_barrier(0);                                              \
  } while (0)
#else
#define MQ_PSTAMP(row, slot) do { } while (0)
#endif

// What the partition reads of a descriptor: key row, length, and whether the row is AES-128-GCM.
// A thread's kPartItems descriptors are fetched together (fields first, then the rows' suites),
// so it waits on memory twice rather than twice per descriptor.
struct PartItem { uint32_t key, len, nch; bool aes; };  // nch: 16-B chunks of its LDS image
__device__ __forceinline__ void part_fetch(const KeyRow* __restrict__ kt, uint32_t n_rows,
                                           const mq_pkt_desc* __restrict__ desc, uint32_t n,
                                           PartItem (&it)[kPartItems]) {
  const uint32_t base = blockIdx.x * kPartBlock + threadIdx.x;
#pragma unroll
  for (int k = 0; k < kPartItems; ++k) {
    const uint32_t i = base + k * kPartThreads;
    it[k].key = i < n ? desc[i].key_id : 0xFFFFFFFFu;
    it[k].len = i < n ? desc[i].len : 0u;
    it[k].nch = i < n ? (((uint32_t)desc[i].offset & 15u) + it[k].len + 15u) >> 4 : 0u;
  }
#pragma unroll
  for (int k = 0; k < kPartItems; ++k) it[k].aes = it[k].key < n_rows && kt[it[k].key].suite == MQ_SUITE_AES128GCM;
}

// class = group * kLenClasses + (31 - length bucket)
__device__ __forceinline__ uint32_t part_class(uint32_t hot, const PartItem& x) {
  const uint32_t g = x.aes ? (x.key == hot ? 0u : 1u) : 2u;
  const uint32_t b = min(x.len >> 6, kLenClasses - 1);
  return g * kLenClasses + (kLenClasses - 1 - b);
}

// keyed layout: the bin of a non-majority AES packet (row-major, longest class first)
__device__ __forceinline__ uint32_t key_bin(const PartItem& x) {
  return x.key * kKeyClasses + (kKeyClasses - 1 - min(x.len >> 7, kKeyClasses - 1));
}
// Tables of at most kBinSlots bins (<= 128 rows) count in LDS per block, then one global atomic per
// bin of the block: a batch over 2 or 3 AES keys otherwise put every packet of a row on ONE global
// counter, 131k-350k atomics on one address per kernel (config C over 2 keys: 248 GiB/s,
// gpurun_out/r04zb; 741 with the LDS counts, r04zc). Larger tables keep the per-thread combining
// below (an LDS hash of bins measured C with 1024 keys 2.8 % and E 1.1 % slower, r04zc).
constexpr uint32_t kBinSlots = 2048;
__device__ __forceinline__ bool bins_in_lds(const uint32_t* bins, uint32_t n_rows) {
  return bins && n_rows * kKeyClasses <= kBinSlots;
}

// Boyer-Moore majority pairs (candidate, count); combining any partition of the input in any
// order keeps the majority element if there is one
__device__ __forceinline__ uint2 vote_join(uint2 a, uint2 b) {
  if (a.x == b.x) return make_uint2(a.x, a.y + b.y);
  return a.y >= b.y ? make_uint2(a.x, a.y - b.y) : make_uint2(b.x, b.y - a.y);
}

__device__ __forceinline__ uint2 block_vote(uint2 v) {  // kPartThreads threads: waves, then wave 0
  __shared__ uint2 s_v[kPartThreads / kWave];
#pragma unroll
  for (int d = kWave / 2; d > 0; d >>= 1)
    v = vote_join(v, make_uint2((uint32_t)__shfl_xor((int)v.x, d, kWave), (uint32_t)__shfl_xor((int)v.y, d, kWave)));
  if ((threadIdx.x & (kWave - 1)) == 0) s_v[threadIdx.x / kWave] = v;
  __syncthreads();
  v = (threadIdx.x & (kWave - 1)) < kPartThreads / kWave ? s_v[threadIdx.x & (kWave - 1)] : make_uint2(kNoKey, 0u);
#pragma unroll
  for (int d = kPartThreads / kWave / 2; d > 0; d >>= 1)
    v = vote_join(v, make_uint2((uint32_t)__shfl_xor((int)v.x, d, kWave), (uint32_t)__shfl_xor((int)v.y, d, kWave)));
  return v;  // every wave holds the result in every lane
}

// Packets per tile of a class: AES tiles stream from HBM (no LDS image), so always 8. ChaCha
// tiles take as many as fit the LDS image budget at the class's longest length and worst
// alignment (4b + 5 chunks), so the class's tiles stay on the staged path; classes that would
// need fewer than kMinPpt per tile (and the open-ended last one) keep 8 and take the direct path.
constexpr uint32_t kMinPpt = 5;
// cmax (r04): the largest image of the class's packets in this batch, in chunks (the count
// kernel's atomicMax; 0 = no packet), so aligned packets are not priced at the worst alignment —
// 1200-B packets at 16-B offsets take 75 chunks, 8 to a tile, where the class bound (77) gave 7
// and a receive batch of 1200-B packets ran 8/7 as many tiles.
__device__ __forceinline__ uint32_t class_ppt(uint32_t c, uint32_t cmax) {
  if (c < 2 * kLenClasses) return kPktsPerTile;  // groups 0 and 1: AES
  const uint32_t b = kLenClasses - 1 - (c % kLenClasses);
  if (b == kLenClasses - 1) return kPktsPerTile;
  const uint32_t worst = 4 * b + 5, need = cmax && cmax < worst ? cmax : worst;
  const uint32_t x = kBudgetChunks / need;
  return x >= kPktsPerTile ? kPktsPerTile : (x >= kMinPpt ? x : kPktsPerTile);
}
// Narrow tiles of list 1 (r05, mq_chacha.hip narrow_tile): a class whose largest image lets at least
// 3/4 of a narrow tile's Q = 64 / G packets fit the wave's image budget (kNarrowChunks, no pool
// scratch) runs G lanes per packet: G = 1, 2 or 4, the smallest that qualifies; else the octet
// layout (G = 8). cmax = 0: an empty class, G = 1 (it constrains no neighbour).
constexpr uint32_t kNarrowImageChunks = (kLdsBytes - 64) / 16;  // mq_chacha.hip kNarrowChunks
__device__ __forceinline__ uint32_t class_g(uint32_t b, uint32_t cmax) {
  if (cmax == 0) return 1;
  if (b == kLenClasses - 1) return kPktsPerTile;
#pragma unroll
  for (uint32_t g = 1; g <= 4; g <<= 1) {
    const uint32_t q = kWave / g, fit = kNarrowImageChunks / cmax;
    if (4 * min(fit, q) >= 3 * q) return g;
  }
  return kPktsPerTile;
}
}  // namespace

// Entries of one suite's list: every class segment is whole tiles of 8 entries, holes included.
// A class of c packets at p <= 8 per tile takes 8 * ceil(c / p) < 8c / kMinPpt + 8 entries, so a
// list of n packets spread over its classes needs at most 8n / kMinPpt + 8 per class. List 0 holds
// two class groups (hot AES key, other AES keys: 2 * kLenClasses classes), list 1 one; the cap
// covers the larger.
// Narrow ChaCha20 classes (tiles of Q = 16, 32 or 64 entries, at least 3Q/4 packets each) take at
// most 4c/3 + Q entries, and the regions' starts are aligned to their tile size: kNarrowSlack more
// per list covers both.
constexpr uint32_t kNarrowCapSlack = kWave * kLenClasses + 128;
uint32_t mq_partition_list_cap(uint32_t n) {
  const uint64_t c = ((uint64_t)n * kPktsPerTile + kMinPpt - 1) / kMinPpt + kPktsPerTile * 2 * kLenClasses +
                     kNarrowCapSlack;
  return (uint32_t)((c + kPktsPerTile - 1) & ~(uint64_t)(kPktsPerTile - 1));
}

// The batch's hot AES key: Boyer-Moore vote over a fixed sample of kVoteSample descriptors
// (evenly spaced), in kVoteSlices slices of 256 — init blocks 0 .. V-1 vote one slice each
// (votes[s]), and every count block folds the V slice votes the same way (lane 0's result),
// so no launch and no single workgroup carries it. The hot key only shapes tiles; any candidate
// gives the same results.
constexpr uint32_t kVoteSample = 4096, kVoteSlice = 256, kVoteSlices = kVoteSample / kVoteSlice;
__device__ __forceinline__ uint2 vote_slice(const KeyRow* __restrict__ kt, uint32_t n_rows,
                                            const mq_pkt_desc* __restrict__ desc, uint32_t n, uint32_t s) {
  const uint32_t S = min(n, kVoteSample), stride = n / S;
  const uint32_t k = s * kVoteSlice + threadIdx.x;
  uint2 v = make_uint2(kNoKey, 0u);
  if (threadIdx.x < kVoteSlice && k < S) {
    const uint32_t key = desc[k * stride].key_id;
    if (key < n_rows && kt[key].suite == MQ_SUITE_AES128GCM) v = make_uint2(key, 1u);
  }
  return block_vote(v);
}
// fold of the slice votes (every lane of a wave computes it; the result is lane 0's)
__device__ __forceinline__ uint32_t fold_votes(const uint2* __restrict__ votes, uint32_t nv) {
  const uint32_t lane = threadIdx.x & (kWave - 1);
  uint2 v = lane < nv ? votes[lane] : make_uint2(kNoKey, 0u);
#pragma unroll
  for (int d = kWave / 2; d > 0; d >>= 1)
    v = vote_join(v, make_uint2((uint32_t)__shfl_xor((int)v.x, d, kWave), (uint32_t)__shfl_xor((int)v.y, d, kWave)));
  const uint32_t x = __builtin_amdgcn_readfirstlane(v.x), y = __builtin_amdgcn_readfirstlane(v.y);
  return y ? x : kNoKey;
}
// meta: counts[0..1] | hot row | hot segment entries | seg[kClasses] | slice votes (kVoteSlices pairs) |
// cmax[kLenClasses] (list 1's largest image per class, chunks) | cls[kLenClasses] (list 1's classes:
// ppt | Q << 8) | reg[8] (list 1's regions: tiles of G = 8, 4, 2, 1, first entries of G = 4, 2, 1,
// all tiles; mq_chacha.hip chacha_list_tile) | ctot[kClasses] | ccur[kClasses] | done
constexpr uint32_t kMetaCmax = 4 + kClasses + 2 * kVoteSlices;
constexpr uint32_t kMetaCls = kMetaCmax + kLenClasses;
constexpr uint32_t kMetaReg = kMetaCls + kLenClasses;
constexpr uint32_t kMetaCtot = kMetaReg + 8;       // class totals (count kernel)
constexpr uint32_t kMetaCcur = kMetaCtot + kClasses;  // class cursors (scatter)
constexpr uint32_t kMetaDone = kMetaCcur + kClasses;  // count blocks finished
constexpr uint32_t kMetaWords = kMetaDone + 1;

// First launch: fills the lists with holes and zeroes the keyed bins (grid-stride, 16-B stores);
// blocks 0 .. nv-1 also vote a sample slice each.
extern "C" __global__ __launch_bounds__(kPartThreads) void mq_part_init_kernel(
    const KeyRow* __restrict__ kt, uint32_t n_rows, const mq_pkt_desc* __restrict__ desc, uint32_t n,
    uint2* __restrict__ votes, uint32_t nv, uint4* __restrict__ list, uint32_t list_q, uint4* __restrict__ bins,
    uint32_t bins_q, const uint32_t* __restrict__ live, uint32_t* __restrict__ cmax) {
  if (pass_empty(live)) return;
  if (blockIdx.x == 0 && threadIdx.x < kLenClasses) cmax[threadIdx.x] = 0;
  // ctot | ccur | done follow reg in the meta (kMetaCtot .. kMetaDone)
  if (blockIdx.x == 0 && threadIdx.x < 2 * kClasses + 1) cmax[kMetaCtot - kMetaCmax + threadIdx.x] = 0;
  if (blockIdx.x < nv) {  // block-uniform
    const uint2 v = vote_slice(kt, n_rows, desc, n, blockIdx.x);
    if (threadIdx.x == 0) votes[blockIdx.x] = v;
  }
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t q = blockIdx.x * blockDim.x + threadIdx.x; q < list_q; q += stride)
    list[q] = make_uint4(kListHole, kListHole, kListHole, kListHole);
  for (uint32_t q = blockIdx.x * blockDim.x + threadIdx.x; q < bins_q; q += stride) bins[q] = make_uint4(0, 0, 0, 0);
}

// Keyed-layout words (after the meta): bins[16 R] (per (row, class) packet counts; the count
// kernel's atomics hand each packet its rank inside its bin), rowseg[2 R] (per row: first list
// entry, entries including the tile padding), rowrel[R] (a row's first entry relative to its row
// block), btot[kRowBlocksMax] (row blocks' entries) and base (list 0's first keyed entry). Init
// zeroes the bins.
constexpr uint32_t kRowThreads = 256, kRowBlocksMax = 256;
struct KeyedWs { uint32_t *bins, *rowseg, *rowrel, *btot; };
__host__ __device__ __forceinline__ KeyedWs keyed_ws(uint32_t* base, uint32_t n_rows) {
  KeyedWs k;
  k.bins = base;
  k.rowseg = base ? base + 16ull * n_rows : nullptr;
  k.rowrel = base ? base + 18ull * n_rows : nullptr;
  k.btot = base ? base + 19ull * n_rows : nullptr;
  return k;
}
__host__ __device__ __forceinline__ size_t keyed_zero_quads(uint32_t n_rows) { return 4ull * n_rows; }
// row blocks of mq_part_rows_kernel: kRowThreads threads of R consecutive rows, at most
// kRowBlocksMax blocks
__host__ __device__ __forceinline__ uint32_t rows_per_thread(uint32_t n_rows) {
  const uint32_t per = kRowThreads * kRowBlocksMax;
  return n_rows > per ? (n_rows + per - 1) / per : 1u;
}

__device__ void part_layout(uint32_t cap, uint32_t* __restrict__ counts, uint32_t* __restrict__ seg,
                            const uint32_t* __restrict__ ctot, const KeyedWs& kw, uint32_t n_rows,
                            const uint32_t* __restrict__ cmax, uint32_t* __restrict__ cls, uint32_t* __restrict__ reg,
                            uint32_t narrow);
__device__ void part_empty(uint32_t* __restrict__ counts, uint32_t* __restrict__ reg, const KeyedWs& kw,
                           uint32_t n_rows);

// Per block: the class counts of its kPartBlock descriptors, added to the batch's class totals
// (ctot); keyed (bins != nullptr): non-majority AES packets are counted per (row, class) bin and
// per row instead, and each keyed packet's rank inside its bin comes back from the bin's atomic.
// Every packet's code (its class, or its bin and rank) goes to code[i] for the scatter, which then
// reads 8 B per packet instead of the descriptor and key row, and makes no keyed atomics (r05:
// the scatter's returning per-bin atomics took ~10 us of config E's and ~22 us of C/1024's scatter,
// tools/part_count_stamps.py). The block that finishes last lays the lists out (part_layout): no
// single-workgroup scan launch (r05: the r04 scan kernel took 32-35 us for config E, 19 of them
// scanning the 4098 rows' bins; the row totals are now counted directly).
constexpr uint32_t kCodeClass = 1u << 31;  // code.x: class item (| class), else keyed bin (< 2^26)
constexpr uint32_t kCodeNone = 0xFFFFFFFFu;  // in no list (skip_unkeyed)
extern "C" __global__ __launch_bounds__(kPartThreads) void mq_part_count_kernel(
    const KeyRow* __restrict__ kt, uint32_t n_rows, const mq_pkt_desc* __restrict__ desc, uint32_t n,
    const uint2* __restrict__ votes, uint32_t nv, uint32_t* __restrict__ hot_p, uint32_t* __restrict__ bins,
    uint32_t skip_unkeyed, const uint32_t* __restrict__ live, uint32_t* __restrict__ cmax,
    uint32_t* __restrict__ ctot, uint32_t* __restrict__ done, uint32_t cap, uint32_t* __restrict__ counts,
    uint32_t* __restrict__ seg, uint32_t* __restrict__ cls, uint32_t* __restrict__ reg, uint32_t narrow,
    uint2* __restrict__ code) {
  const KeyedWs kw = keyed_ws(bins, n_rows);
  if (pass_empty(live)) {  // empty lists: no hot key, no row segments, no regions
    if (blockIdx.x == 0) part_empty(counts, reg, kw, n_rows);
    return;
  }
  __shared__ uint32_t s_cnt[kClasses];
  __shared__ uint32_t s_max[kLenClasses];  // list 1's classes: the largest image, in chunks
  __shared__ uint32_t s_bcnt[kBinSlots];
  __shared__ uint32_t s_last;
  const bool lds_bins = bins_in_lds(bins, n_rows);  // kernel-uniform
  MQ_PSTAMP(blockIdx.x, 0);
  PartItem it[kPartItems];
  part_fetch(kt, n_rows, desc, n, it);
  if (threadIdx.x < kClasses) s_cnt[threadIdx.x] = 0;
  if (threadIdx.x < kLenClasses) s_max[threadIdx.x] = 0;
  if (lds_bins)
    for (uint32_t q = threadIdx.x; q < n_rows * kKeyClasses; q += blockDim.x) s_bcnt[q] = 0;
  const uint32_t hot = fold_votes(votes, nv);  // the same in every wave of every block
  if (blockIdx.x == 0 && threadIdx.x == 0) *hot_p = hot;
  __syncthreads();
  MQ_PSTAMP(blockIdx.x, 1);
  uint32_t kb[kPartItems], cl[kPartItems];
  bool kd[kPartItems], in[kPartItems];
#pragma unroll
  for (int k = 0; k < kPartItems; ++k) {
    const uint32_t i = blockIdx.x * kPartBlock + k * kPartThreads + threadIdx.x;
    in[k] = i < n && !(skip_unkeyed && it[k].key >= n_rows);
    const uint32_t c = in[k] ? part_class(hot, it[k]) : 0u;
    cl[k] = c;
    kd[k] = bins && in[k] && c / kLenClasses == 1;
    kb[k] = kd[k] ? key_bin(it[k]) : 0u;
    if (in[k] && !kd[k]) atomicAdd(&s_cnt[c], 1u);
    if (in[k] && c >= 2 * kLenClasses) atomicMax(&s_max[c - 2 * kLenClasses], it[k].nch);
  }
  // keyed bins: the thread's items of one bin claim their places with one atomic (a thread's items
  // are kPartThreads descriptors apart: with keys assigned round-robin over 1024 rows, as in config
  // C with 1024 keys, all four share a bin — 4x fewer atomics on the 1024 hot addresses); the
  // leader's returned count is the group's first rank, a follower's rank adds the items before it
  uint32_t kpos[kPartItems];
#pragma unroll
  for (int k = 0; k < kPartItems; ++k) {
    int lead = k;
    uint32_t cnt = 1, rank = 0;
#pragma unroll
    for (int j = 0; j < kPartItems; ++j) {
      const bool same = kd[j] && kb[j] == kb[k];
      if (j < k && same) { rank += 1; lead = lead == k ? j : lead; }
      if (j > k && same) ++cnt;
    }
    uint32_t base = 0;
    if (kd[k] && lead == k) base = atomicAdd(lds_bins ? &s_bcnt[kb[k]] : &kw.bins[kb[k]], cnt);
#pragma unroll
    for (int j = 0; j < kPartItems; ++j)
      if (j == lead && j < k) base = kpos[j];
    kpos[k] = kd[k] ? base + rank : 0u;  // lds_bins: the rank inside the block's count of the bin
  }
  MQ_PSTAMP(blockIdx.x, 2);
  __syncthreads();
  if (lds_bins) {  // kernel-uniform: the block's base in each bin, one global atomic per bin
    for (uint32_t q = threadIdx.x; q < n_rows * kKeyClasses; q += blockDim.x)
      if (s_bcnt[q]) s_bcnt[q] = atomicAdd(&kw.bins[q], s_bcnt[q]);
  }
  if (threadIdx.x < kClasses && s_cnt[threadIdx.x]) atomicAdd(&ctot[threadIdx.x], s_cnt[threadIdx.x]);
  if (threadIdx.x < kLenClasses && s_max[threadIdx.x]) atomicMax(&cmax[threadIdx.x], s_max[threadIdx.x]);
  if (lds_bins) __syncthreads();  // kernel-uniform
#pragma unroll
  for (int k = 0; k < kPartItems; ++k) {
    const uint32_t i = blockIdx.x * kPartBlock + k * kPartThreads + threadIdx.x;
    if (i < n)
      code[i] = kd[k] ? make_uint2(kb[k], kpos[k] + (lds_bins ? s_bcnt[kb[k]] : 0u))
                      : make_uint2(in[k] ? kCodeClass | cl[k] : kCodeNone, 0u);
  }
  // The last block to finish lays the lists out. Each thread waits until its atomics above are
  // performed (vmcnt counts them on gfx950) before the barrier that precedes the block's count, so
  // the block's totals are in when the count is. No __threadfence: on gfx950 a device-scope release
  // also writes back the XCD's L2 (measured: the count kernel 26 -> 108 us with one per block).
  // This is the hand-off the MI355X guide lists as measured-valid on gfx950 / ROCm 7.2 without a
  // release/acquire pair (MI355X_MICROARCH.md "Valid forms", first table row: every storing wave's
  // vmcnt(0), the barrier, ONE lane's agent-scope add to one counter, the block whose add came last
  // told by its returned value, every load of the handed-off words past L1 — ld_fresh — and the
  // handed-off words themselves written only by agent-scope atomics). It is outside the HIP memory
  // model, so tests/test_gpu_parity.py::test_partition_handoff_stress re-runs keyed partitions over
  // every XCD and checks each result byte for byte.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  MQ_PSTAMP(blockIdx.x, 3);
  if (threadIdx.x == 0) s_last = atomicAdd(done, 1u) == gridDim.x - 1;
  __syncthreads();
  MQ_PSTAMP(blockIdx.x, 4);
  if (!s_last) return;  // block-uniform
  part_layout(cap, counts, seg, ctot, kw, n_rows, cmax, cls, reg, narrow);
  MQ_PSTAMP(blockIdx.x, 6);
}

__device__ __forceinline__ uint32_t ld_fresh(const uint32_t* p) {  // past this CU's L1: other blocks' atomics
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ void part_empty(uint32_t* __restrict__ counts, uint32_t* __restrict__ reg, const KeyedWs& kw,
                           uint32_t n_rows) {
  if (threadIdx.x == 0) { counts[0] = 0; counts[1] = 0; counts[2] = kNoKey; counts[3] = 0; }
  if (threadIdx.x < 8) reg[threadIdx.x] = 0;
  if (kw.rowseg)
    for (uint32_t r = threadIdx.x; r < n_rows; r += blockDim.x) *(uint2*)(kw.rowseg + 2 * (size_t)r) = make_uint2(0, 0);
}

// The lists' layout (the count kernel's last block, 16 waves) from the class totals: the class
// segments (whole tiles) list by list (groups 0 and 1: list 0, group 2: list 1 at `cap`): seg[c] =
// first list entry of class c, counts[s] = entries of list s, holes included; counts[3] = entries of
// the hot key's classes (the front of list 0, whole tiles); keyed, the rows' segments after them.
__device__ void part_layout(uint32_t cap, uint32_t* __restrict__ counts, uint32_t* __restrict__ seg,
                            const uint32_t* __restrict__ ctot, const KeyedWs& kw, uint32_t n_rows,
                            const uint32_t* __restrict__ cmax, uint32_t* __restrict__ cls, uint32_t* __restrict__ reg,
                            uint32_t narrow) {
  __shared__ uint32_t s_tot[kClasses];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (threadIdx.x < kClasses) s_tot[threadIdx.x] = ld_fresh(ctot + threadIdx.x);
  __syncthreads();
  static_assert(2 * kLenClasses == kWave && kClasses - 2 * kLenClasses <= kWave, "one wave per list");
  if (wave == 0) {  // list 0 (AES): lane = class 0..63, tiles of 8 entries
    const uint32_t c = (uint32_t)lane;
    const uint32_t ppt = class_ppt(c, 0u);
    const uint32_t ent = kPktsPerTile * ((s_tot[c] + ppt - 1) / ppt);
    const uint32_t incl = wave_incl_scan(ent), e = lane_u32(incl, kWave - 1);
    seg[c] = incl - ent;
    const uint32_t hot_e = lane_u32(incl, kLenClasses - 1);  // list 0: the hot key's classes first
    if (lane == 0) {
      counts[3] = hot_e;
      // mq_partition_list_cap bounds e; the clamp only keeps a broken bound from running a suite
      // kernel over the other list (keyed: the scatter adds the rows' segments)
      counts[0] = min(e, cap);
      if (kw.btot) kw.btot[kRowBlocksMax] = e;  // keyed: the rows' segments follow
    }
  } else if (wave == 1) {
    // list 1 (ChaCha20 and the rest): lane l = class 2 kLenClasses + l, longest first. Each class
    // runs G lanes per packet (class_g; made non-increasing along the list by a suffix maximum, so
    // the list is four regions — G = 8, 4, 2, 1 — each a run of whole tiles of Q = 64 / G entries
    // starting at a multiple of Q); a class's tiles hold ppt <= Q packets, the rest holes.
    const bool in = lane < (int)kLenClasses;
    const uint32_t c = 2 * kLenClasses + (uint32_t)lane, b = kLenClasses - 1 - (uint32_t)lane;
    const uint32_t cm = in ? ld_fresh(cmax + lane) : 0u, tot = in ? s_tot[c] : 0u;
    // the receive composite's passes (skip_unkeyed) keep octet tiles only: their persistent list
    // kernels carry no narrow path (it spilled their registers)
    uint32_t g = in ? (narrow ? class_g(b, tot ? cm : 0u) : (tot ? kPktsPerTile : 1u)) : 0u;
#pragma unroll
    for (int d = 1; d < (int)kLenClasses; d <<= 1) {  // suffix maximum over the classes after this one
      const uint32_t v = (uint32_t)__shfl_down((int)g, d, kWave);
      if (lane + d < (int)kLenClasses) g = max(g, v);
    }
    const uint32_t Q = in ? kWave / g : 1u;
    const uint32_t ppt = !in ? 1u : (g == kPktsPerTile ? class_ppt(c, cm) : min(Q, kNarrowImageChunks / max(cm, 1u)));
    const uint32_t ent = in && tot ? Q * ((tot + ppt - 1) / ppt) : 0u;
    uint32_t E[4];  // entries of the regions G = 8, 4, 2, 1
#pragma unroll
    for (int r = 0; r < 4; ++r) E[r] = lane_u32(wave_incl_scan(in && g == (8u >> r) ? ent : 0u), kWave - 1);
    const uint32_t R4 = (E[0] + 15) & ~15u, R2 = (R4 + E[1] + 31) & ~31u, R1 = (R2 + E[2] + 63) & ~63u;
    // the list ends with its last non-empty region (no padding after it); every 8 entries of it also
    // form a valid octet tile (holes skipped), so a kernel that ignores the regions (the persistent
    // list kernels, MQ_CC_LIST=1) still processes every packet
    const uint32_t end = E[3] ? R1 + E[3] : E[2] ? R2 + E[2] : E[1] ? R4 + E[1] : E[0];
    const uint32_t incl = wave_incl_scan(ent), excl = incl - ent;
    const uint32_t start = g == 8 ? excl : g == 4 ? R4 + excl - E[0] : g == 2 ? R2 + excl - E[0] - E[1]
                                                                         : R1 + excl - E[0] - E[1] - E[2];
    if (in) {
      seg[c] = cap + start;
      cls[lane] = ppt | Q << 8;
    }
    if (lane == 0) {
      counts[1] = min(end, cap);
      // the regions (list-relative): tiles of each, then the narrow regions' first entries
      reg[0] = E[0] / 8; reg[1] = E[1] / 16; reg[2] = E[2] / 32; reg[3] = E[3] / 64;
      reg[4] = R4; reg[5] = R2; reg[6] = R1; reg[7] = reg[0] + reg[1] + reg[2] + reg[3];
    }
  }
  MQ_PSTAMP(blockIdx.x, 5);
}

// Keyed layout, after the count kernel: each row's segment (its packets, whole tiles) follows the
// majority key's classes in list 0, which end on a tile boundary at `base`. Row blocks of
// kRowThreads threads sum their rows' 16 bins each (64 B), scan the rows' entries (rounded up to
// whole tiles) inside the block: rowseg[2r + 1] = entries, rowrel[r] = first entry relative to the
// row block, btot[block] = the block's entries; the scatter adds the row blocks' prefix and writes
// rowseg[2r] = first entry. (r05: the count kernel's last block scanned all rows alone: 15 us for
// config E's 4098 rows, one CU's reads of lines the atomics had just updated, and before that a
// per-row counter cost one more global atomic per keyed packet, tools/part_count_stamps.py.)
extern "C" __global__ __launch_bounds__(kRowThreads) void mq_part_rows_kernel(uint32_t* __restrict__ bins,
                                                                           uint32_t n_rows,
                                                                           const uint32_t* __restrict__ live) {
  if (pass_empty(live)) return;
  __shared__ uint32_t s_w[kRowThreads / kWave];
  const KeyedWs kw = keyed_ws(bins, n_rows);
  const uint32_t R = rows_per_thread(n_rows);
  const uint32_t r0 = (blockIdx.x * kRowThreads + threadIdx.x) * R;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t sum = 0;
  for (uint32_t q = 0; q < R; ++q) {
    const uint32_t r = r0 + q;
    if (r >= n_rows) break;
    const uint4* b = (const uint4*)(kw.bins + (size_t)r * kKeyClasses);
    uint32_t tot = 0;
#pragma unroll
    for (int j = 0; j < (int)kKeyClasses / 4; ++j) {
      const uint4 v = b[j];
      tot += v.x + v.y + v.z + v.w;
    }
    const uint32_t ent = (tot + kPktsPerTile - 1) & ~(kPktsPerTile - 1);  // whole tiles
    kw.rowseg[2 * (size_t)r + 1] = ent;
    sum += ent;
  }
  const uint32_t incl = wave_incl_scan(sum);
  if (lane == 63) s_w[wave] = incl;
  __syncthreads();
  uint32_t at = incl - sum, blk = 0;
#pragma unroll
  for (int w = 0; w < (int)(kRowThreads / kWave); ++w) {
    at += w < wave ? s_w[w] : 0u;
    blk += s_w[w];
  }
  for (uint32_t q = 0; q < R; ++q) {
    const uint32_t r = r0 + q;
    if (r >= n_rows) break;
    kw.rowrel[r] = at;
    at += kw.rowseg[2 * (size_t)r + 1];
  }
  if (threadIdx.x == 0) kw.btot[blockIdx.x] = blk;
}

// first list entry of keyed bin kb: its row's start (the row block's prefix s_bpre, the row's
// offset inside its block) plus the row's packets in longer classes
__device__ __forceinline__ uint32_t bin_start(const KeyedWs& kw, uint32_t kb, const uint32_t* s_bpre, uint32_t rpb) {
  const uint32_t row = kb / kKeyClasses, c = kb % kKeyClasses;
  const uint4* b = (const uint4*)(kw.bins + (size_t)row * kKeyClasses);
  uint32_t p = s_bpre[row / rpb] + kw.rowrel[row];
#pragma unroll
  for (uint32_t k = 0; k < kKeyClasses / 4; ++k) {
    const uint4 v = b[k];
    p += (4 * k < c ? v.x : 0u) + (4 * k + 1 < c ? v.y : 0u) + (4 * k + 2 < c ? v.z : 0u) + (4 * k + 3 < c ? v.w : 0u);
  }
  return p;
}

// Each block counts its packets per class again (from the count kernel's codes) and reserves
// their ranks inside each class with one global atomic per class (ccur): the block's packets of a
// class take consecutive ranks (the order of blocks inside a class is whichever reserved first —
// packets are independent, so only the tile composition can change between runs, never a result).
// Keyed packets sit at bin_start + the rank their count-kernel atomic returned.
extern "C" __global__ __launch_bounds__(kPartThreads) void mq_part_scatter_kernel(
    const uint2* __restrict__ code, uint32_t n, uint32_t n_rows, uint32_t* __restrict__ ccur,
    const uint32_t* __restrict__ seg, uint32_t* __restrict__ list, uint32_t* __restrict__ bins,
    const uint32_t* __restrict__ live, const uint32_t* __restrict__ cls, uint32_t* __restrict__ counts,
    uint32_t cap) {
  if (pass_empty(live)) return;
  MQ_PSTAMP(gridDim.x + blockIdx.x, 0);
  const KeyedWs kw = keyed_ws(bins, n_rows);
  __shared__ uint32_t s_rank[kClasses];
  __shared__ uint32_t s_cls[kLenClasses];  // list 1's classes: ppt | Q << 8 (the layout's)
  __shared__ uint32_t s_bpre[kRowBlocksMax];  // keyed: first list entry of each row block
  __shared__ uint32_t s_bw[kRowBlocksMax / kWave];
  if (threadIdx.x < kLenClasses) s_cls[threadIdx.x] = cls[threadIdx.x];
  if (threadIdx.x < kClasses) s_rank[threadIdx.x] = 0;
  const uint32_t rpb = kRowThreads * rows_per_thread(n_rows);  // rows per row block
  if (bins) {  // kernel-uniform: the row blocks' exclusive prefix, from list 0's keyed base
    const uint32_t nrb = (n_rows + rpb - 1) / rpb;
    const uint32_t t = threadIdx.x;
    const uint32_t v = t < nrb ? kw.btot[t] : 0u;
    const uint32_t incl = wave_incl_scan(v);
    if (t < kRowBlocksMax && (t & 63) == 63) s_bw[t >> 6] = incl;
    __syncthreads();
    if (t < kRowBlocksMax) {
      uint32_t x = kw.btot[kRowBlocksMax] + incl - v, all = kw.btot[kRowBlocksMax];
#pragma unroll
      for (int w = 0; w < (int)(kRowBlocksMax / kWave); ++w) {
        x += w < (int)(t >> 6) ? s_bw[w] : 0u;
        all += s_bw[w];
      }
      s_bpre[t] = x;
      if (blockIdx.x == 0 && t == 0) counts[0] = min(all, cap);  // list 0: hot classes + rows
    }
  }
  uint2 x[kPartItems];
#pragma unroll
  for (int k = 0; k < kPartItems; ++k) {
    const uint32_t i = blockIdx.x * kPartBlock + k * kPartThreads + threadIdx.x;
    x[k] = i < n ? code[i] : make_uint2(kCodeNone, 0u);
  }
  const int lane = threadIdx.x & 63;
  uint32_t cl[kPartItems];
  bool in[kPartItems];
#pragma unroll
  for (int k = 0; k < kPartItems; ++k) {
    in[k] = (x[k].x & kCodeClass) && x[k].x != kCodeNone;
    cl[k] = in[k] ? x[k].x & ~kCodeClass : 0u;
  }
  __syncthreads();  // s_rank zeroed, s_bpre
  MQ_PSTAMP(gridDim.x + blockIdx.x, 1);
  if (bins) {  // kernel-uniform: this block's share of the rows' absolute first entries
    const uint32_t share = (n_rows + gridDim.x - 1) / gridDim.x;
    const uint32_t lo = blockIdx.x * share, hi = min(n_rows, lo + share);
    for (uint32_t r = lo + threadIdx.x; r < hi; r += blockDim.x) kw.rowseg[2 * (size_t)r] = s_bpre[r / rpb] + kw.rowrel[r];
  }
  // the block's counts per class (as the count kernel made them), then one global reservation each
#pragma unroll
  for (int k = 0; k < kPartItems; ++k)
    if (in[k]) atomicAdd(&s_rank[cl[k]], 1u);
#pragma unroll
  for (int k = 0; k < kPartItems; ++k)
    if (!(x[k].x & kCodeClass))  // keyed
      list[bin_start(kw, x[k].x, s_bpre, rpb) + x[k].y] = blockIdx.x * kPartBlock + k * kPartThreads + threadIdx.x;
  MQ_PSTAMP(gridDim.x + blockIdx.x, 2);
  __syncthreads();
  if (threadIdx.x < kClasses && s_rank[threadIdx.x]) s_rank[threadIdx.x] = atomicAdd(&ccur[threadIdx.x], s_rank[threadIdx.x]);
  __syncthreads();
  MQ_PSTAMP(gridDim.x + blockIdx.x, 3);
  const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
#pragma unroll
  for (int k = 0; k < kPartItems; ++k) {
    const uint32_t i = blockIdx.x * kPartBlock + k * kPartThreads + threadIdx.x;
    const uint32_t c = cl[k];
    // lanes of this wave with the same class (7 ballots), rank among them = peers below
    uint64_t peers = __ballot(in[k]);
#pragma unroll
    for (int bit = 0; bit < 7; ++bit) {
      const uint64_t b = __ballot((c >> bit) & 1u);
      peers &= ((c >> bit) & 1u) ? b : ~b;
    }
    const uint32_t rank = (uint32_t)__popcll(peers & below);
    uint32_t base = 0;
    if (in[k] && rank == 0) base = atomicAdd(&s_rank[c], (uint32_t)__popcll(peers));
    // the leader (lowest lane of the peer group) hands its base to the group
    const int leader = in[k] ? __ffsll((unsigned long long)peers) - 1 : lane;
    base = (uint32_t)__shfl((int)base, leader, kWave);
    if (in[k]) {
      const uint32_t r = base + rank;
      const uint32_t y = c >= 2 * kLenClasses ? s_cls[c - 2 * kLenClasses] : (class_ppt(c, 0u) | kPktsPerTile << 8);
      const uint32_t ppt = y & 0xffu, Q = y >> 8;
      list[seg[c] + Q * (r / ppt) + r % ppt] = i;
    }
  }
  MQ_PSTAMP(gridDim.x + blockIdx.x, 4);
}

// keyed layout bins: one counter per (row, class), within a budget of 2 per packet (at least
// 64 Ki) and below 2^26, and only when the keyed list (at most 7 holes per row) fits the list
// capacity
static size_t key_bins(uint32_t n) { return 2 * (size_t)n > 65536 ? 2 * (size_t)n : 65536; }
static bool keyed_layout(uint32_t n, uint32_t n_rows) {
  return (size_t)n_rows * kKeyClasses <= key_bins(n) && (size_t)n_rows * kKeyClasses < (1u << 26) &&
         (uint64_t)n + kPktsPerTile * kLenClasses + (uint64_t)(kPktsPerTile - 1) * n_rows <= mq_partition_list_cap(n);
}


// list (2 x cap entries) | codes (8 B per packet, the count kernel's) |
// meta (2 totals, hot row, hot segment entries, kClasses segment starts) | keyed bins, 256-B aligned pieces
static size_t part_align(size_t b) { return (b + 255) & ~(size_t)255; }

// The per-row segments of a keyed partition (rowseg, 2 words per row, keyed_ws), or null when
// mq_launch_partition(n, n_rows) does not lay the list out keyed. counts: the partition's meta (as
// passed to mq_launch_partition).
const uint32_t* mq_partition_rowseg(uint32_t n, uint32_t n_rows, const uint32_t* counts) {
  if (!keyed_layout(n, n_rows)) return nullptr;
  return keyed_ws((uint32_t*)((uint8_t*)counts + part_align(sizeof(uint32_t) * kMetaWords)), n_rows).rowseg;
}

hipError_t mq_launch_partition(const KeyRow* kt, uint32_t n_rows, const mq_pkt_desc* desc, uint32_t n,
                               uint32_t* list, uint32_t* codes, uint32_t* counts, hipStream_t s, bool skip_unkeyed,
                               const uint32_t* live) {
  const uint32_t nblocks = (n + kPartBlock - 1) / kPartBlock;
  // narrow ChaCha20 regions: not for the receive passes (skip_unkeyed); MQ_CC_NARROW=0 (diagnostic /
  // A-B, mq_opts.h) turns them off as it turns off the flat narrow kernels
  const bool narrow = !skip_unkeyed && mq::opt(mq::Opt::CcNarrow) != 0;
  if (nblocks == 0) {  // no lists, no regions
    const hipError_t e = hipMemsetAsync(counts, 0, 4 * sizeof(uint32_t), s);
    return e != hipSuccess ? e : hipMemsetAsync(counts + kMetaReg, 0, 8 * sizeof(uint32_t), s);
  }
  const uint32_t cap = mq_partition_list_cap(n);
  uint32_t* hot = counts + 2;  // meta (kMetaWords): counts[0..1] | hot row | hot entries | seg | votes
  uint32_t* seg = counts + 4;
  uint2* votes = (uint2*)(counts + 4 + kClasses);
  uint32_t* cmax = counts + kMetaCmax;
  uint32_t* cls = counts + kMetaCls;
  uint32_t* reg = counts + kMetaReg;
  uint32_t* bins = keyed_layout(n, n_rows) ? (uint32_t*)((uint8_t*)counts + part_align(sizeof(uint32_t) * kMetaWords))
                                           : nullptr;
  const uint32_t list_q = cap / 2, bins_q = bins ? (uint32_t)keyed_zero_quads(n_rows) : 0u;  // 16-B words
  const uint32_t init_blocks = max(1u, min(256u, (list_q + bins_q + kPartThreads - 1) / kPartThreads));
  const uint32_t nv = min(kVoteSlices, init_blocks);
  const uint32_t S = min(n, kVoteSample), used = (S + kVoteSlice - 1) / kVoteSlice;  // slices with samples
  const uint32_t grid = max(init_blocks, used);
  hipLaunchKernelGGL(mq_part_init_kernel, dim3(grid), dim3(kPartThreads), 0, s, kt, n_rows, desc, n, votes,
                     max(nv, used), (uint4*)list, list_q, (uint4*)bins, bins_q, live, cmax);
  hipLaunchKernelGGL(mq_part_count_kernel, dim3(nblocks), dim3(kPartThreads), 0, s, kt, n_rows, desc, n, votes,
                     max(nv, used), hot, bins, (uint32_t)skip_unkeyed, live, cmax, counts + kMetaCtot,
                     counts + kMetaDone, cap, counts, seg, cls, reg, (uint32_t)narrow, (uint2*)codes);
  if (bins && n_rows) {
    const uint32_t rpb = kRowThreads * rows_per_thread(n_rows);
    hipLaunchKernelGGL(mq_part_rows_kernel, dim3((n_rows + rpb - 1) / rpb), dim3(kRowThreads), 0, s, bins, n_rows, live);
  }
  hipLaunchKernelGGL(mq_part_scatter_kernel, dim3(nblocks), dim3(kPartThreads), 0, s, (const uint2*)codes, n, n_rows,
                     counts + kMetaCcur, seg, list, bins, live, cls, counts, cap);
  return hipGetLastError();
}

// list 1's region words (reg[8], see kMetaWords) of a partition whose meta is `counts`
const uint32_t* mq_partition_regions(const uint32_t* counts) { return counts + kMetaReg; }

size_t mq_partition_workspace(uint32_t n) {
  // keyed words (keyed_ws): 19 per row, rows <= key_bins(n) / 16, then btot and base
  return part_align(sizeof(uint32_t) * 2 * (size_t)mq_partition_list_cap(n)) +
         part_align(sizeof(uint2) * (size_t)n) + part_align(sizeof(uint32_t) * kMetaWords) +
         part_align(sizeof(uint32_t) * (key_bins(n) / 16 * 19 + kRowBlocksMax + 8));
}

// offsets of the pieces inside the partition workspace
void mq_partition_layout(uint32_t n, size_t* codes_off, size_t* counts_off) {
  *codes_off = part_align(sizeof(uint32_t) * 2 * (size_t)mq_partition_list_cap(n));
  *counts_off = *codes_off + part_align(sizeof(uint2) * (size_t)n);
}

#ifdef MQ_STAMPS
void mq_stamps_set_part(uint64_t* p) { (void)hipMemcpyToSymbol(HIP_SYMBOL(mq_part_stamp_buf), &p, sizeof p); }
#endif
