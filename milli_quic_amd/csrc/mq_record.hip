// mq_record.hip — TLS 1.3 record layer epilogue.
//
// The record seal/open itself runs in the ChaCha20-Poly1305 / AES-128-GCM tile kernels
// (descriptors flagged MQ_PKT_TLS_RECORD: AAD = the 5-byte record header, nonce = iv ^ seq,
// reference src/tcp_tls/record.rs:70-143). What remains after a successful open is
// find_inner_content_type (src/tcp_tls/connection.rs:546-556): strip the zero padding, take the
// last non-zero byte as the content type. One lane per record; the scan is normally one byte.
#include "mq_device.h"

using namespace mq;

extern "C" __global__ __launch_bounds__(256) void mq_record_inner_kernel(
    const uint8_t* __restrict__ arena, uint64_t arena_len, const mq_pkt_desc* __restrict__ desc, uint32_t n,
    uint8_t* __restrict__ status, uint64_t* __restrict__ info) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || status[i] != MQ_OK) return;
  const mq_pkt_desc d = desc[i];
  if (!(d.flags & 0x04)) return;  // not a TLS record
  // validated by the tile kernel: d.len >= 21, offset + len <= arena_len; plaintext is
  // [offset + 5, offset + len - 16)
  const uint64_t lo = d.offset + 5;
  uint64_t pos = d.offset + d.len - 16;
  while (pos > lo && arena[pos - 1] == 0) --pos;
  const uint8_t ct = pos > lo ? arena[pos - 1] : 0;
  if (ct < 20 || ct > 23) {  // no content type, or ContentType::from_byte fails (record.rs:16-24)
    status[i] = MQ_ERR_TLS;
    return;
  }
  if (info) info[i] = (pos - 1 - lo) | ((uint64_t)ct << 32);
}

hipError_t mq_launch_record_inner(const uint8_t* arena, uint64_t arena_len, const mq_pkt_desc* desc, uint32_t n,
                                  uint8_t* status, uint64_t* info, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(mq_record_inner_kernel, dim3((n + 255) / 256), dim3(256), 0, s, arena, arena_len, desc, n,
                     status, info);
  return hipGetLastError();
}
