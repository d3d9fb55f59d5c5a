// mq_build.h — packet layout of the send composite from frames, shared by the
// build kernel (mq_send.hip) and the fused ChaCha20-Poly1305 protect kernel (mq_chacha.hip).
//
// The reference builds each packet in build_and_encrypt_initial_packet (src/connection/
// transmit.rs:499-622) and build_and_encrypt_packet (:625-755): PN length from largest_acked
// (src/packet/number.rs:9-26), the Initial / Handshake long header with its Length varint
// (src/packet/long_header.rs:214-314) or the 1-RTT short header (short_header.rs:33-47, first
// byte 0x40 | key_phase << 2 | pn_len - 1), encode_pn (number.rs:32-43), the frames, PADDING
// (Initial up to 1200 bytes when pad_to_min; otherwise pn_len + payload + tag >= 20).
#pragma once
#include "mq_device.h"

namespace mq {

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


// One packet's layout from its request (octet-uniform values). st: the build status (MQ_OK, or
// the error the build reports for the request, as mq_batch_protect's status); d: its descriptor
// (key_id 0xFFFFFFFF unless built); len_out: pkt_len (the packet length, or `needed` on
// MQ_ERR_BUFFER_TOO_SMALL, else 0); hp = header + PN bytes; body = frames + PADDING + tag room.
struct BuildLayout {
  int st;
  uint32_t len_out, hdr, pn_len, hp, m, body;
  uint8_t level;
  uint64_t pn, payload_length, frames_offset;
  const mq_conn_send* cp;
  mq_pkt_desc d;
  // byte x < hp of the packet (header, then the truncated PN)
  __device__ __forceinline__ uint8_t header(uint32_t x) const {
    return x < hdr ? header_byte(*cp, level, pn_len, payload_length, x) : (uint8_t)(pn >> (8 * (pn_len - 1 - (x - hdr))));
  }
};

__device__ __forceinline__ BuildLayout build_layout(uint32_t i, bool valid, const KeyRow* __restrict__ kt, uint32_t n_rows,
                                                    const mq_conn_send* __restrict__ conns, uint32_t n_conns,
                                                    uint64_t frames_len, uint64_t out_len,
                                                    const mq_send_req* __restrict__ req, uint32_t suite_hint) {
  mq_send_req r{};
  if (valid) r = req[i];
  BuildLayout b;
  b.d.offset = r.out_offset; b.d.len = 0; b.d.key_id = 0xFFFFFFFFu; b.d.pn = r.pn; b.d.pn_offset = 0;
  b.d.pn_len = 0; b.d.flags = 0; b.d.reserved = 0;
  b.st = MQ_OK;
  b.len_out = 0;
  b.level = r.level;
  b.pn = r.pn;
  b.frames_offset = r.frames_offset;
  const mq_conn_send* cp = valid && r.conn < n_conns ? conns + r.conn : nullptr;
  b.cp = cp;
  // the row's fields read from global memory where used (a private copy would put key_row[level]
  // in scratch)
  const bool lv_ok = r.level <= MQ_LEVEL_APPLICATION;
  const uint32_t key_row = cp && lv_ok ? cp->key_row[r.level] : 0xFFFFFFFFu;
  // checks in the oracle's order (orc_batch_protect, then orc_protect_frames): request ranges, the
  // row's suite against the caller's hint and Initial = AES-128-GCM (keys.rs:131-136), then the
  // connection IDs
  uint32_t row_suite = 0;
  if (!cp || r.level > MQ_LEVEL_APPLICATION || r.frames_offset + (uint64_t)r.frame_len > frames_len ||
      r.out_offset + (uint64_t)r.out_cap > out_len || key_row >= n_rows) {
    b.st = MQ_ERR_INVALID_ARG;
  } else {
    row_suite = kt[key_row].suite;
    if ((suite_hint != MQ_SUITE_MIXED && row_suite != suite_hint) ||
        (r.level == MQ_LEVEL_INITIAL && row_suite != MQ_SUITE_AES128GCM))
      b.st = MQ_ERR_SUITE;
    else if (cp->dcid_len > 20 || cp->scid_len > 20)
      b.st = MQ_ERR_INVALID_ARG;
  }
  // pn_length (number.rs:9-26)
  const uint64_t unacked = r.pn > r.largest_acked ? r.pn - r.largest_acked : 1;
  b.pn_len = unacked < (1u << 7) ? 1u : unacked < (1u << 15) ? 2u : unacked < (1u << 23) ? 3u : 4u;
  uint32_t pad = 0, hdr = 0;
  uint64_t payload_length = 0, total = 0;
  if (b.st == MQ_OK) {
    if (r.level == MQ_LEVEL_INITIAL) {  // transmit.rs:521-558
      const uint64_t pl = b.pn_len + (uint64_t)r.frame_len + 16;
      const uint64_t t0 = long_header_len(*cp, true, pl) + pl;
      if ((r.flags & MQ_SEND_PAD_TO_MIN) && t0 < 1200) pad = (uint32_t)(1200 - t0);
      payload_length = pl + pad;
      hdr = long_header_len(*cp, true, payload_length);
    } else {  // :641-686
      const uint32_t min_enc = b.pn_len >= 20 ? 0u : 20u - b.pn_len;
      if (r.frame_len + 16u < min_enc) pad = min_enc - r.frame_len - 16u;
      payload_length = b.pn_len + (uint64_t)r.frame_len + pad + 16;
      hdr = r.level == MQ_LEVEL_HANDSHAKE ? long_header_len(*cp, false, payload_length) : 1u + cp->dcid_len;
    }
    total = (uint64_t)hdr + b.pn_len + r.frame_len + pad + 16;
    if (r.out_cap < hdr) { b.st = MQ_ERR_BUFFER_TOO_SMALL; b.len_out = hdr; }
    else if (r.out_cap < hdr + b.pn_len) { b.st = MQ_ERR_BUFFER_TOO_SMALL; b.len_out = b.pn_len; }
    else if (total > r.out_cap) { b.st = MQ_ERR_BUFFER_TOO_SMALL; b.len_out = (uint32_t)total; }
    // a row of neither suite (MQ_SUITE_MIXED hint) fails the seal itself: nothing written, length 0
    else if (row_suite != MQ_SUITE_AES128GCM && row_suite != MQ_SUITE_CHACHA20) b.st = MQ_ERR_SUITE;
  }
  const bool ok = valid && b.st == MQ_OK;
  b.hdr = hdr;
  b.payload_length = payload_length;
  b.hp = ok ? hdr + b.pn_len : 0u;
  b.m = ok ? r.frame_len : 0u;
  b.body = ok ? r.frame_len + pad + 16u : 0u;
  if (ok) {
    b.d.len = (uint32_t)total;
    b.d.key_id = key_row;
    b.d.pn_offset = (uint16_t)hdr;
    b.d.pn_len = (uint8_t)b.pn_len;
    b.d.flags = r.level != MQ_LEVEL_APPLICATION ? MQ_PKT_LONG_HEADER : 0;
    b.len_out = (uint32_t)total;
  }
  return b;
}


// The packet's bytes written to out (global stores) by octet lane j: header and PN bytes 8j ..
// 8j + 7, then payload chunk q = bytes [16q, 16q + 16) after them for q = j, j + 8, ...; chunks
// wholly inside the frames are copied with 16-B accesses at any alignment (B loads in flight per
// lane before their stores); the frames' last bytes, PADDING and the tag room byte-wise / as zero
// chunks, so no byte outside [out_offset, out_offset + len) is touched. Nothing for a failed build.
template <uint32_t B>
__device__ __forceinline__ void build_store(const BuildLayout& b, int j, const uint8_t* __restrict__ frames,
                                            uint8_t* __restrict__ out) {
  uint8_t* dst = out + b.d.offset;
  // header and PN bytes: bytes 8j .. 8j + 7 of the octet's packet
  for (uint32_t x = 8u * (uint32_t)j; x < b.hp && x < 8u * (uint32_t)j + 8u; ++x) dst[x] = b.header(x);
  // frames, PADDING and the tag room: chunk q = payload bytes [16q, 16q + 16), lane j takes q = j,
  // j + 8, ...; chunks wholly inside the frames are copied with 16-B accesses
  uint8_t* pd = dst + b.hp;
  const uint8_t* ps = frames + b.frames_offset;
  const uint32_t m = b.m, body = b.body;
  const uint32_t nq = (body + 15u) / 16u;
  for (uint32_t q0 = (uint32_t)j; q0 < nq; q0 += 8u * B) {
    uint4 v[B];
#pragma unroll
    for (uint32_t t = 0; t < B; ++t) {
      const uint32_t q = q0 + 8u * t;
      v[t] = (q < nq && 16u * q + 16u <= m) ? ld16(ps + 16u * q) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (uint32_t t = 0; t < B; ++t) {
      const uint32_t q = q0 + 8u * t;
      if (q >= nq) continue;
      if (16u * q + 16u <= m) {
        uint32_t w[4];
        u4w(v[t], w);
        st16(pd + 16u * q, w);
      } else {  // the frames' last bytes, zeros after them; the packet's last chunk may be partial
        const uint32_t end = min(16u, body - 16u * q);
        for (uint32_t y0 = 0; y0 < end; ++y0) {
          const uint32_t y = 16u * q + y0;
          pd[y] = y < m ? ps[y] : 0;
        }
      }
    }
  }
}


// Header bytes 8j .. 8j + 7 of a packet for octet lane j, from two 8-byte windows of its connection
// row (mq_conn_send: dcid_len @0, scid_len @1, key_phase @2, dcid @4, scid @24) — the DCID bytes
// and the SCID bytes those header positions would hold — so a lane waits on two loads rather than
// one dependent load per byte, and no byte is picked from a run-time-indexed private array (which
// the compiler would keep in scratch).
__device__ __forceinline__ uint64_t conn_window(const mq_conn_send* cp, int off) {  // row bytes [off, off + 8)
  const int c = min(max(off, 0), (int)sizeof(mq_conn_send) - 8);
  const uint8_t* p = reinterpret_cast<const uint8_t*>(cp) + c;
  uint64_t v = (uint64_t)*(const u32_u*)p | (uint64_t)*(const u32_u*)(p + 4) << 32;
  if (off > c) v = off - c >= 8 ? 0ull : v >> (8 * (off - c));
  if (off < c) v = c - off >= 8 ? 0ull : v << (8 * (c - off));
  return v;
}

struct HeaderLane {
  uint64_t wd, ws;      // row bytes under this lane's DCID / SCID positions
  uint32_t dl, sl, kp;  // CID lengths, key phase
  __device__ __forceinline__ void load(const mq_conn_send* cp, uint32_t level, int j) {
    const uint32_t w0 = *(const u32_u*)cp;
    dl = w0 & 0xffu; sl = (w0 >> 8) & 0xffu; kp = (w0 >> 16) & 0xffu;
    // 1-RTT: dcid[x - 1] = row byte x + 3; long: dcid[x - 6] = row byte x - 2, scid[x - 7 - dl] =
    // row byte x + 17 - dl
    wd = conn_window(cp, 8 * j + (level == MQ_LEVEL_APPLICATION ? 3 : -2));
    ws = conn_window(cp, 8 * j + 17 - (int)dl);
  }
  // header byte x = 8j + u (x < hdr_len); header_byte's layout
  __device__ __forceinline__ uint8_t byte(uint32_t level, uint32_t pn_len, uint64_t payload_length, uint32_t x,
                                          uint32_t u) const {
    const uint8_t d = (uint8_t)(wd >> (8 * u)), sc = (uint8_t)(ws >> (8 * u));
    if (level == MQ_LEVEL_APPLICATION) return x == 0 ? (uint8_t)(0x40 | ((kp & 1) << 2) | (pn_len - 1)) : d;
    const bool initial = level == MQ_LEVEL_INITIAL;
    if (x == 0) return (uint8_t)((initial ? 0xC0 : 0xE0) | ((pn_len - 1) & 3));
    if (x < 5) return x == 4 ? 1 : 0;  // QUIC_VERSION_1
    if (x == 5) return (uint8_t)dl;
    if (x < 6 + dl) return d;
    if (x == 6 + dl) return (uint8_t)sl;
    if (x < 7 + dl + sl) return sc;
    uint32_t p = 7 + dl + sl;
    if (initial) {
      if (x == p) return 0;  // token length (the reference sends no token, transmit.rs:519)
      ++p;
    }
    const uint32_t n = varint_len(payload_length), k = x - p;  // varint.rs:72-110
    uint8_t v = (uint8_t)(payload_length >> (8 * (n - 1 - k)));
    if (k == 0) v |= n == 1 ? 0 : n == 2 ? 0x40 : n == 4 ? 0x80 : 0xc0;
    return v;
  }
};

// The frames part of an image chunk whose first byte is packet byte x0 (header positions and
// bytes past the frames zero): one 16-B load when the chunk's frames window lies inside the frames
// buffer (fo: the packet's frames offset, flen: the buffer's length), byte-wise at its ends.
__device__ __forceinline__ uint4 edge_frames(const BuildLayout& b, const uint8_t* __restrict__ fr, int x0,
                                             uint64_t fo, uint64_t flen) {
  const int64_t src = (int64_t)x0 - (int64_t)b.hp;  // frames offset of the chunk's first byte
  uint32_t w[4];
  if (src + (int64_t)fo >= 0 && (uint64_t)((int64_t)fo + src) + 16 <= flen) {
    u4w(ld16(fr + src), w);
  } else {
    uint64_t lo = 0, hi = 0;
    for (int y = 0; y < 16; ++y) {
      const int64_t f = src + y;
      if (f < 0 || f >= (int64_t)b.m) continue;
      const uint64_t v = fr[f];
      if (y < 8) lo |= v << (8 * y);
      else hi |= v << (8 * (y - 8));
    }
    w[0] = (uint32_t)lo; w[1] = (uint32_t)(lo >> 32); w[2] = (uint32_t)hi; w[3] = (uint32_t)(hi >> 32);
  }
  // keep packet bytes [hp, hp + m) of the chunk
  const int lo = min(max((int)b.hp - x0, 0), 16), hi = min(max((int)(b.hp + b.m) - x0, 0), 16);
#pragma unroll
  for (int q = 0; q < 4; ++q) w[q] &= byte_mask(hi, q) & ~byte_mask(lo, q);
  return make_uint4(w[0], w[1], w[2], w[3]);
}

}  // namespace mq
