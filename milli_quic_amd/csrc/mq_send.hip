// mq_send.hip — the send composite from plaintext frames on gfx950.
//
// The reference builds each packet in build_and_encrypt_initial_packet (src/connection/
// transmit.rs:499-622) and build_and_encrypt_packet (:625-755): PN length from largest_acked
// (src/packet/number.rs:9-26), the Initial / Handshake long header with its Length varint
// (src/packet/long_header.rs:214-314) or the 1-RTT short header (short_header.rs:33-47, first
// byte 0x40 | key_phase << 2 | pn_len - 1), encode_pn (number.rs:32-43), the frames, PADDING
// (Initial up to 1200 bytes when pad_to_min; otherwise pn_len + payload + tag >= 20), then seal
// and header protection. Here mq_build_kernel does everything up to the seal for a whole batch —
// eight packets per wave, one octet of lanes each (build_octet) — and emits an mq_pkt_desc per
// packet; the ChaCha20-Poly1305 / AES-128-GCM tile kernels then seal and header-protect those
// descriptors, and mq_send_status_kernel folds the build statuses in.
#include "mq_build.h"

using namespace mq;


// Eight packets per wave (r04), one octet of lanes per packet as in the tile kernels: the octet
// reads its request and connection row, computes the layout, writes header and PN bytes (8 bytes
// per lane) and moves the frames in 16-B chunks at any alignment (unaligned dwordx4 loads and
// stores, every chunk's load issued before the stores), then PADDING and the tag room as zero
// chunks; a packet's last partial chunk goes byte-wise, so no byte outside [out_offset,
// out_offset + len) is touched. r03 built one packet per wave at a time, 16 B per lane with
// per-packet dependent loads: 1.35 ms for 2^20 x 1200 B (profiles/r04g_kernel_stats_protect.csv)
// against ~0.5 ms for its 2.5 GB of traffic.
constexpr uint32_t kBuildWaves = 4;   // waves per workgroup
#ifndef MQ_BUILD_BATCH
#define MQ_BUILD_BATCH 10
#endif
constexpr uint32_t kBuildBatch = MQ_BUILD_BATCH;  // chunks per lane whose loads are in flight together
                                                  // (10: all of a 1200-B packet's)

__device__ __forceinline__ void build_octet(
    uint32_t i, bool valid, int j, const KeyRow* __restrict__ kt, uint32_t n_rows,
    const mq_conn_send* __restrict__ conns, uint32_t n_conns, const uint8_t* __restrict__ frames, uint64_t frames_len,
    uint8_t* __restrict__ out, uint64_t out_len, const mq_send_req* __restrict__ req, mq_pkt_desc* __restrict__ desc,
    uint8_t* __restrict__ bstatus, uint32_t* __restrict__ pkt_len, uint32_t suite_hint) {
  const BuildLayout b = build_layout(i, valid, kt, n_rows, conns, n_conns, frames_len, out_len, req, suite_hint);
  build_store<kBuildBatch>(b, j, frames, out);
  if (valid && j == 0) {
    desc[i] = b.d;
    bstatus[i] = (uint8_t)b.st;
    pkt_len[i] = b.len_out;
  }
}

extern "C" __global__ __launch_bounds__(64 * kBuildWaves) void mq_build_kernel(
    const KeyRow* __restrict__ kt, uint32_t n_rows, const mq_conn_send* __restrict__ conns, uint32_t n_conns,
    const uint8_t* __restrict__ frames, uint64_t frames_len, uint8_t* __restrict__ out, uint64_t out_len,
    const mq_send_req* __restrict__ req, uint32_t n, mq_pkt_desc* __restrict__ desc, uint8_t* __restrict__ bstatus,
    uint32_t* __restrict__ pkt_len, uint32_t suite_hint) {
  const int lane = threadIdx.x & (kWave - 1), p = lane / kLanesPerPkt, j = lane % kLanesPerPkt;
  const uint32_t i = (blockIdx.x * kBuildWaves + (threadIdx.x >> 6)) * kPktsPerTile + (uint32_t)p;
  build_octet(i, i < n, j, kt, n_rows, conns, n_conns, frames, frames_len, out, out_len, req, desc, bstatus, pkt_len, suite_hint);
}

// build failures keep their status (the seal kernel saw an invalid key id for them)
extern "C" __global__ __launch_bounds__(256) void mq_send_status_kernel(const uint8_t* __restrict__ bstatus,
                                                                        uint8_t* __restrict__ status, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && bstatus[i] != MQ_OK) status[i] = bstatus[i];
}

hipError_t mq_launch_build(const KeyRow* kt, uint32_t n_rows, const mq_conn_send* conns, uint32_t n_conns,
                           const uint8_t* frames, uint64_t frames_len, uint8_t* out, uint64_t out_len,
                           const mq_send_req* req, uint32_t n, mq_pkt_desc* desc, uint8_t* bstatus,
                           uint32_t* pkt_len, uint32_t suite_hint, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint32_t per_wg = kBuildWaves * kPktsPerTile, wgs = (n + per_wg - 1) / per_wg;
  hipLaunchKernelGGL(mq_build_kernel, dim3(wgs), dim3(64 * kBuildWaves), 0, s, kt, n_rows, conns, n_conns, frames,
                     frames_len, out, out_len, req, n, desc, bstatus, pkt_len, suite_hint);
  return hipGetLastError();
}

hipError_t mq_launch_send_status(const uint8_t* bstatus, uint8_t* status, uint32_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(mq_send_status_kernel, dim3((n + 255) / 256), dim3(256), 0, s, bstatus, status, n);
  return hipGetLastError();
}
