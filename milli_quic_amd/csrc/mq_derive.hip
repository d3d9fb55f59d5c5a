// mq_derive.hip — batched QUIC v1 Initial key derivation on gfx950.
//
// A server under an Initial flood runs derive_initial (reference src/connection/keys.rs:181-212)
// once per new client DCID: HKDF-Extract(v1 salt, DCID) -> "client in" / "server in" secrets
// (src/crypto/key_schedule.rs:60-72), then per secret "quic key" / "quic iv" / "quic hp"
// (derive_directional_keys, key_schedule.rs:123-151, hp length max(16, 16) = 16), then what
// Aes128GcmProvider::aead / ::header_protection precompute (src/crypto/rustcrypto.rs:232-252):
// the AES-128 key schedules and the GHASH subkey H = E_K(0^128). Initial packets are always
// AES-128-GCM (keys.rs:187-188).
//
// One lane per connection, 24 SHA-256 compressions (FIPS 180-4) per lane: the HMAC pads of the
// fixed salt and the padded HKDF-Expand-Label message blocks are constants computed once on the
// host (MQDeriveConsts); per lane: extract (2), PRK pads (2), client/server secrets (2 x 2), and
// per secret its pads (2) + key/iv/hp (3 x 2). The results go straight into device key-table
// rows in the layout mq_keytable_create builds on the host (client keys at row 2i, server keys at
// 2i + 1): AES round keys from the LDS T-table S-box, H^1..H^8 by the reflected GF(2^128)
// multiply of mq_aes.h.
#include "mq_aes.h"

namespace mq {

__device__ __forceinline__ uint32_t rotr32(uint32_t x, int r) { return (x >> r) | (x << (32 - r)); }

// FIPS 180-4 §6.2.2: one compression of the 16 big-endian words w (clobbered: schedule in place).
__device__ __attribute__((noinline)) void sha256_compress(uint32_t (&st)[8], uint32_t (&w)[16]) {
  constexpr uint32_t K[64] = {
      0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
      0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
      0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
      0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
      0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
      0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
      0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
      0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
  for (int i = 0; i < 64; ++i) {
    uint32_t wi;
    if (i < 16) {
      wi = w[i];
    } else {
      const uint32_t w15 = w[(i + 1) & 15], w2 = w[(i + 14) & 15];
      wi = w[i & 15] + (rotr32(w15, 7) ^ rotr32(w15, 18) ^ (w15 >> 3)) + w[(i + 9) & 15] +
           (rotr32(w2, 17) ^ rotr32(w2, 19) ^ (w2 >> 10));
      w[i & 15] = wi;
    }
    const uint32_t t1 = h + (rotr32(e, 6) ^ rotr32(e, 11) ^ rotr32(e, 25)) + ((e & f) ^ (~e & g)) + K[i] + wi;
    const uint32_t t2 = (rotr32(a, 2) ^ rotr32(a, 13) ^ rotr32(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
    h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

__device__ __forceinline__ void sha256_iv(uint32_t (&st)[8]) {
  st[0] = 0x6a09e667; st[1] = 0xbb67ae85; st[2] = 0x3c6ef372; st[3] = 0xa54ff53a;
  st[4] = 0x510e527f; st[5] = 0x9b05688c; st[6] = 0x1f83d9ab; st[7] = 0x5be0cd19;
}

struct HmacPads { uint32_t ist[8], ost[8]; };

// RFC 2104 with a 32-byte key (a PRK or a traffic secret): the compressed ipad / opad blocks.
__device__ __forceinline__ HmacPads hmac_pads(const uint32_t (&key)[8]) {
  HmacPads p;
  uint32_t w[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) w[q] = (q < 8 ? key[q] : 0u) ^ 0x36363636u;
  sha256_iv(p.ist);
  sha256_compress(p.ist, w);
#pragma unroll
  for (int q = 0; q < 16; ++q) w[q] = (q < 8 ? key[q] : 0u) ^ 0x5c5c5c5cu;
  sha256_iv(p.ost);
  sha256_compress(p.ost, w);
  return p;
}

// HMAC(key, m) for a message m that fits one padded block after the key block: `blk` is that
// block (message || 0x80 || 0.. || bit length of 64 + |m| bytes).
__device__ __forceinline__ void hmac_block(const uint32_t (&ist)[8], const uint32_t (&ost)[8],
                                           const uint32_t (&blk)[16], uint32_t (&out)[8]) {
  uint32_t s[8], w[16];
#pragma unroll
  for (int q = 0; q < 8; ++q) s[q] = ist[q];
#pragma unroll
  for (int q = 0; q < 16; ++q) w[q] = blk[q];
  sha256_compress(s, w);
#pragma unroll
  for (int q = 0; q < 8; ++q) { out[q] = ost[q]; w[q] = s[q]; }
  w[8] = 0x80000000u;
#pragma unroll
  for (int q = 9; q < 15; ++q) w[q] = 0;
  w[15] = (64 + 32) * 8;
  sha256_compress(out, w);
}

__device__ __forceinline__ uint32_t sub_word(uint32_t t, uint32_t rb) {  // FIPS-197 SubWord via T0
  return ((tlook(t, 3, rb) << 8) & 0xff000000u) | (tlook(t, 2, rb) & 0x00ff0000u) |
         ((tlook(t, 1, rb) >> 8) & 0x0000ff00u) | ((tlook(t, 0, rb) >> 16) & 0x000000ffu);
}

// FIPS-197 §5.2 key expansion of a 16-byte key given as 4 big-endian words.
__device__ __forceinline__ void aes_expand(const uint32_t (&key)[4], uint32_t rb, AesRk& rk) {
#pragma unroll
  for (int q = 0; q < 4; ++q) rk.w[q] = key[q];
  uint32_t rcon = 1;
#pragma unroll
  for (int i = 4; i < 44; ++i) {
    uint32_t t = rk.w[i - 1];
    if (i % 4 == 0) {
      t = sub_word((t << 8) | (t >> 24), rb) ^ (rcon << 24);
      rcon = ((rcon << 1) ^ ((rcon & 0x80) ? 0x11bu : 0u)) & 0xffu;
    }
    rk.w[i] = rk.w[i - 4] ^ t;
  }
}

// derive_directional_keys for one AES-128-GCM Initial secret -> a key-table row (+ material).
__device__ __attribute__((noinline)) void derive_row(const MQDeriveConsts& k, const uint32_t (&secret)[8], uint32_t rb,
                                           KeyRow* row, mq_key_material* km) {
  const HmacPads p = hmac_pads(secret);
  uint32_t key[8], iv[8], hp[8];
  hmac_block(p.ist, p.ost, k.lbl[2], key);  // "quic key", 16 bytes
  hmac_block(p.ist, p.ost, k.lbl[3], iv);   // "quic iv", 12 bytes
  hmac_block(p.ist, p.ost, k.lbl[4], hp);   // "quic hp", 16 bytes
  uint32_t* r = reinterpret_cast<uint32_t*>(row);
  r[0] = MQ_SUITE_AES128GCM; r[1] = 0; r[2] = 0; r[3] = 0;
#pragma unroll
  for (int q = 0; q < 3; ++q) row->iv[q] = bswap32(iv[q]);
  row->pad1 = 0;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    row->key[q] = q < 4 ? bswap32(key[q]) : 0u;
    row->hp[q] = q < 4 ? bswap32(hp[q]) : 0u;
  }
  AesRk rk;
  {
    const uint32_t hk[4] = {hp[0], hp[1], hp[2], hp[3]};
    aes_expand(hk, rb, rk);
#pragma unroll
    for (int q = 0; q < 44; ++q) row->hp_rk[q] = rk.w[q];
  }
  const uint32_t kk[4] = {key[0], key[1], key[2], key[3]};
  aes_expand(kk, rb, rk);
#pragma unroll
  for (int q = 0; q < 44; ++q) row->aes_rk[q] = rk.w[q];
  // H = E_K(0^128), then H^2..H^8 (reflected basis; stored as GCM-order big-endian words)
  uint32_t s0 = 0, s1 = 0, s2 = 0, s3 = 0;
  aes128_block(rk, rb, s0, s1, s2, s3);
  const uint32_t h[4] = {s0, s1, s2, s3};
  uint32_t hr[4] = {brev(s0), brev(s1), brev(s2), brev(s3)}, acc[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) { row->H[0][q] = h[q]; acc[q] = hr[q]; }
  const GfOp mh = gf_prepare(hr);
  for (int e = 1; e < 8; ++e) {
    gf_mul(acc, mh);
#pragma unroll
    for (int q = 0; q < 4; ++q) row->H[e][q] = brev(acc[q]);
  }
  if (km) {  // mq_key_material: suite, reserved, key[32], iv[12], pad[4], hp[32] (little-endian words)
    uint32_t* m = reinterpret_cast<uint32_t*>(km);
    m[0] = MQ_SUITE_AES128GCM; m[1] = 0;
#pragma unroll
    for (int q = 0; q < 8; ++q) { m[2 + q] = row->key[q]; m[14 + q] = row->hp[q]; }
#pragma unroll
    for (int q = 0; q < 3; ++q) m[10 + q] = row->iv[q];
    m[13] = 0;
  }
}

}  // namespace mq

using namespace mq;

extern "C" __global__ __launch_bounds__(256) void mq_derive_initial_kernel(
    MQDeriveConsts k, const uint8_t* __restrict__ dcids, const uint8_t* __restrict__ dcid_lens, uint32_t n,
    KeyRow* __restrict__ rows, mq_key_material* __restrict__ km_out, uint8_t* __restrict__ status) {
  build_t0(threadIdx.x, blockDim.x);
  __syncthreads();
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t rb = (threadIdx.x & (kTReplicas - 1)) * 4;
  const uint32_t len = dcid_lens[i];
  if (len > kMaxCidLen) {  // RFC 9000 §17.2: connection IDs are at most 20 bytes
    reinterpret_cast<uint32_t*>(rows + 2 * (size_t)i)[0] = 0;  // suite 0: rejected per packet
    reinterpret_cast<uint32_t*>(rows + 2 * (size_t)i + 1)[0] = 0;
    status[i] = MQ_ERR_INVALID_ARG;
    return;
  }
  // HKDF-Extract(salt, dcid) = HMAC(salt, dcid): one block dcid || 0x80 || .. || (64 + len) * 8
  uint32_t w[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) w[q] = 0;
  const uint8_t* c = dcids + (size_t)kMaxCidLen * i;
#pragma unroll
  for (uint32_t b = 0; b <= kMaxCidLen; ++b) {
    const uint32_t v = b < len ? c[b] : (b == len ? 0x80u : 0u);
    w[b >> 2] |= v << (24 - 8 * (b & 3));
  }
  w[15] = (64 + len) * 8;
  uint32_t prk[8], client[8], server[8];
  hmac_block(k.salt_ist, k.salt_ost, w, prk);
  {
    const HmacPads p = hmac_pads(prk);
    hmac_block(p.ist, p.ost, k.lbl[0], client);  // "client in"
    hmac_block(p.ist, p.ost, k.lbl[1], server);  // "server in"
  }
  derive_row(k, client, rb, rows + 2 * (size_t)i, km_out ? km_out + 2 * (size_t)i : nullptr);
  derive_row(k, server, rb, rows + 2 * (size_t)i + 1, km_out ? km_out + 2 * (size_t)i + 1 : nullptr);
  status[i] = MQ_OK;
}

hipError_t mq_launch_derive_initial(const MQDeriveConsts& k, const uint8_t* dcids, const uint8_t* dcid_lens,
                                    uint32_t n, KeyRow* rows, mq_key_material* km_out, uint8_t* status,
                                    hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(mq_derive_initial_kernel, dim3((n + 255) / 256), dim3(256), 0, s, k, dcids, dcid_lens, n,
                     rows, km_out, status);
  return hipGetLastError();
}
