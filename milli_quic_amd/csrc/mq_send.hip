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
#include "mq_device.h"

using namespace mq;

namespace {

__device__ __forceinline__ uint32_t varint_len(uint64_t v) {
  return v < 64 ? 1u : v < 16384 ? 2u : v < (1u << 30) ? 4u : 8u;
}

// encode_initial_header / encode_handshake_header length (long_header.rs:222-225, 279-280)
__device__ __forceinline__ uint32_t long_header_len(const mq_conn_send& c, bool initial, uint64_t payload_length) {
  return 1 + 4 + 1 + c.dcid_len + 1 + c.scid_len + (initial ? 1u : 0u) + varint_len(payload_length);
}

// byte b of the header (b < hdr_len); wave-uniform inputs
__device__ __forceinline__ uint8_t header_byte(const mq_conn_send& c, uint32_t level, uint32_t pn_len,
                                              uint64_t payload_length, uint32_t b) {
  if (level == MQ_LEVEL_APPLICATION) {
    if (b == 0) return (uint8_t)(0x40 | ((c.key_phase & 1) << 2) | (pn_len - 1));
    return c.dcid[b - 1];
  }
  const bool initial = level == MQ_LEVEL_INITIAL;
  if (b == 0) return (uint8_t)((initial ? 0xC0 : 0xE0) | ((pn_len - 1) & 3));
  if (b < 5) return b == 4 ? 1 : 0;  // QUIC_VERSION_1
  uint32_t p = 5;
  if (b == p) return c.dcid_len;
  if (b < p + 1 + c.dcid_len) return c.dcid[b - p - 1];
  p += 1 + c.dcid_len;
  if (b == p) return c.scid_len;
  if (b < p + 1 + c.scid_len) return c.scid[b - p - 1];
  p += 1 + c.scid_len;
  if (initial) {
    if (b == p) return 0;  // token length (the reference sends no token, transmit.rs:519)
    ++p;
  }
  const uint32_t n = varint_len(payload_length), k = b - p;  // varint.rs:72-110
  uint8_t v = (uint8_t)(payload_length >> (8 * (n - 1 - k)));
  if (k == 0) v |= n == 1 ? 0 : n == 2 ? 0x40 : n == 4 ? 0x80 : 0xc0;
  return v;
}

}  // namespace

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
    uint8_t* __restrict__ bstatus, uint32_t* __restrict__ pkt_len) {
  mq_send_req r{};
  if (valid) r = req[i];
  mq_pkt_desc d;
  d.offset = r.out_offset; d.len = 0; d.key_id = 0xFFFFFFFFu; d.pn = r.pn; d.pn_offset = 0; d.pn_len = 0;
  d.flags = 0; d.reserved = 0;
  int st = MQ_OK;
  uint32_t len = 0;
  const mq_conn_send* cp = valid && r.conn < n_conns ? conns + r.conn : nullptr;
  mq_conn_send c{};
  if (cp) c = *cp;
  if (!cp || r.level > MQ_LEVEL_APPLICATION || r.frames_offset + (uint64_t)r.frame_len > frames_len ||
      r.out_offset + (uint64_t)r.out_cap > out_len || c.key_row[r.level] >= n_rows || c.dcid_len > 20 ||
      c.scid_len > 20) {
    st = MQ_ERR_INVALID_ARG;
  } else if (r.level == MQ_LEVEL_INITIAL && kt[c.key_row[0]].suite != MQ_SUITE_AES128GCM) {
    st = MQ_ERR_SUITE;  // Initial packets are AES-128-GCM (keys.rs:131-136)
  }
  // pn_length (number.rs:9-26)
  const uint64_t unacked = r.pn > r.largest_acked ? r.pn - r.largest_acked : 1;
  const uint32_t pn_len = unacked < (1u << 7) ? 1u : unacked < (1u << 15) ? 2u : unacked < (1u << 23) ? 3u : 4u;
  uint32_t pad = 0, hdr = 0;
  uint64_t payload_length = 0, total = 0;
  if (st == MQ_OK) {
    if (r.level == MQ_LEVEL_INITIAL) {  // transmit.rs:521-558
      const uint64_t pl = pn_len + (uint64_t)r.frame_len + 16;
      const uint64_t t0 = long_header_len(c, true, pl) + pl;
      if ((r.flags & MQ_SEND_PAD_TO_MIN) && t0 < 1200) pad = (uint32_t)(1200 - t0);
      payload_length = pl + pad;
      hdr = long_header_len(c, true, payload_length);
    } else {  // :641-686
      const uint32_t min_enc = pn_len >= 20 ? 0u : 20u - pn_len;
      if (r.frame_len + 16u < min_enc) pad = min_enc - r.frame_len - 16u;
      payload_length = pn_len + (uint64_t)r.frame_len + pad + 16;
      hdr = r.level == MQ_LEVEL_HANDSHAKE ? long_header_len(c, false, payload_length) : 1u + c.dcid_len;
    }
    total = (uint64_t)hdr + pn_len + r.frame_len + pad + 16;
    if (r.out_cap < hdr) { st = MQ_ERR_BUFFER_TOO_SMALL; len = hdr; }
    else if (r.out_cap < hdr + pn_len) { st = MQ_ERR_BUFFER_TOO_SMALL; len = pn_len; }
    else if (total > r.out_cap) { st = MQ_ERR_BUFFER_TOO_SMALL; len = (uint32_t)total; }
  }
  const bool ok = valid && st == MQ_OK;
  uint8_t* dst = out + r.out_offset;
  // header and PN bytes: bytes 8j .. 8j + 7 of the octet's packet
  const uint32_t hp = ok ? hdr + pn_len : 0u;
  for (uint32_t b = 8u * (uint32_t)j; b < hp && b < 8u * (uint32_t)j + 8u; ++b)
    dst[b] = b < hdr ? header_byte(*cp, r.level, pn_len, payload_length, b)
                     : (uint8_t)(r.pn >> (8 * (pn_len - 1 - (b - hdr))));
  // frames, PADDING and the tag room: chunk q = payload bytes [16q, 16q + 16), lane j takes q = j,
  // j + 8, ...; chunks wholly inside the frames are copied with 16-B accesses
  uint8_t* pd = dst + hp;
  const uint8_t* ps = frames + r.frames_offset;
  const uint32_t m = ok ? r.frame_len : 0u, body = ok ? m + pad + 16u : 0u;
  const uint32_t nq = (body + 15u) / 16u;
  for (uint32_t q0 = (uint32_t)j; q0 < nq; q0 += 8u * kBuildBatch) {
    uint4 v[kBuildBatch];
#pragma unroll
    for (uint32_t t = 0; t < kBuildBatch; ++t) {
      const uint32_t q = q0 + 8u * t;
      v[t] = (q < nq && 16u * q + 16u <= m) ? ld16(ps + 16u * q) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (uint32_t t = 0; t < kBuildBatch; ++t) {
      const uint32_t q = q0 + 8u * t;
      if (q >= nq) continue;
      if (16u * q + 16u <= m) {
        uint32_t w[4];
        u4w(v[t], w);
        st16(pd + 16u * q, w);
      } else {  // the frames' last bytes, zeros after them; the packet's last chunk may be partial
        const uint32_t end = min(16u, body - 16u * q);
        for (uint32_t b = 0; b < end; ++b) {
          const uint32_t y = 16u * q + b;
          pd[y] = y < m ? ps[y] : 0;
        }
      }
    }
  }
  if (valid && j == 0) {
    if (ok) {
      d.len = (uint32_t)total;
      d.key_id = c.key_row[r.level];
      d.pn_offset = (uint16_t)hdr;
      d.pn_len = (uint8_t)pn_len;
      d.flags = r.level != MQ_LEVEL_APPLICATION ? MQ_PKT_LONG_HEADER : 0;
      len = (uint32_t)total;
    }
    desc[i] = d;
    bstatus[i] = (uint8_t)st;
    pkt_len[i] = len;
  }
}

extern "C" __global__ __launch_bounds__(64 * kBuildWaves) void mq_build_kernel(
    const KeyRow* __restrict__ kt, uint32_t n_rows, const mq_conn_send* __restrict__ conns, uint32_t n_conns,
    const uint8_t* __restrict__ frames, uint64_t frames_len, uint8_t* __restrict__ out, uint64_t out_len,
    const mq_send_req* __restrict__ req, uint32_t n, mq_pkt_desc* __restrict__ desc, uint8_t* __restrict__ bstatus,
    uint32_t* __restrict__ pkt_len) {
  const int lane = threadIdx.x & (kWave - 1), p = lane / kLanesPerPkt, j = lane % kLanesPerPkt;
  const uint32_t i = (blockIdx.x * kBuildWaves + (threadIdx.x >> 6)) * kPktsPerTile + (uint32_t)p;
  build_octet(i, i < n, j, kt, n_rows, conns, n_conns, frames, frames_len, out, out_len, req, desc, bstatus, pkt_len);
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
                           uint32_t* pkt_len, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint32_t per_wg = kBuildWaves * kPktsPerTile, wgs = (n + per_wg - 1) / per_wg;
  hipLaunchKernelGGL(mq_build_kernel, dim3(wgs), dim3(64 * kBuildWaves), 0, s, kt, n_rows, conns, n_conns, frames,
                     frames_len, out, out_len, req, n, desc, bstatus, pkt_len);
  return hipGetLastError();
}

hipError_t mq_launch_send_status(const uint8_t* bstatus, uint8_t* status, uint32_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(mq_send_status_kernel, dim3((n + 255) / 256), dim3(256), 0, s, bstatus, status, n);
  return hipGetLastError();
}
