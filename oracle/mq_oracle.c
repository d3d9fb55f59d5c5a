/*
 * mq_oracle.c — CPU restatement of milli-quic's QUIC packet-protection path.
 *
 * TEST INFRASTRUCTURE ONLY (see mq_oracle.h): the parity checker for the HIP kernels and the
 * "port" CPU baseline of bench.py. Never linked into libmq_aead.so.
 *
 * Written for clarity, not speed: byte-oriented AES, bitwise GHASH (SP 800-38D Alg. 1),
 * 26-bit-limb Poly1305. Citations "ref:" are paths in computer-whisperer/milli-quic.
 */
#include "mq_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------------------------------- */
/* byte helpers                                                                             */
static uint32_t ld32le(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
static void st32le(uint8_t* p, uint32_t v) {
  p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); p[2] = (uint8_t)(v >> 16); p[3] = (uint8_t)(v >> 24);
}
static uint32_t ld32be(const uint8_t* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3];
}
static void st32be(uint8_t* p, uint32_t v) {
  p[0] = (uint8_t)(v >> 24); p[1] = (uint8_t)(v >> 16); p[2] = (uint8_t)(v >> 8); p[3] = (uint8_t)v;
}
static void st64be(uint8_t* p, uint64_t v) { st32be(p, (uint32_t)(v >> 32)); st32be(p + 4, (uint32_t)v); }
static void st64le(uint8_t* p, uint64_t v) { st32le(p, (uint32_t)v); st32le(p + 4, (uint32_t)(v >> 32)); }

/* ---------------------------------------------------------------------------------------- */
/* ChaCha20 block function, RFC 8439 §2.3 (crate chacha20 0.9.1; used by ref
 * src/crypto/rustcrypto.rs:128-132,156-163 via chacha20poly1305 and :210-217 for HP).        */
static uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
#define QR(a, b, c, d)                    \
  a += b; d ^= a; d = rotl32(d, 16);      \
  c += d; b ^= c; b = rotl32(b, 12);      \
  a += b; d ^= a; d = rotl32(d, 8);       \
  c += d; b ^= c; b = rotl32(b, 7);

void orc_chacha20_block(const uint8_t key[32], uint32_t counter, const uint8_t nonce[12],
                        uint8_t out[64]) {
  uint32_t s[16], x[16];
  s[0] = 0x61707865u; s[1] = 0x3320646eu; s[2] = 0x79622d32u; s[3] = 0x6b206574u;
  for (int i = 0; i < 8; ++i) s[4 + i] = ld32le(key + 4 * i);
  s[12] = counter;
  for (int i = 0; i < 3; ++i) s[13 + i] = ld32le(nonce + 4 * i);
  memcpy(x, s, sizeof x);
  for (int i = 0; i < 10; ++i) {
    QR(x[0], x[4], x[8], x[12]); QR(x[1], x[5], x[9], x[13]);
    QR(x[2], x[6], x[10], x[14]); QR(x[3], x[7], x[11], x[15]);
    QR(x[0], x[5], x[10], x[15]); QR(x[1], x[6], x[11], x[12]);
    QR(x[2], x[7], x[8], x[13]); QR(x[3], x[4], x[9], x[14]);
  }
  for (int i = 0; i < 16; ++i) st32le(out + 4 * i, x[i] + s[i]);
}

/* ---------------------------------------------------------------------------------------- */
/* Poly1305, RFC 8439 §2.5 (crate poly1305 0.8.0). 26-bit limbs, h = (h + m) * r mod 2^130-5. */
typedef struct { uint32_t r[5], h[5]; uint8_t s[16]; } orc_poly;

static void poly_init(orc_poly* p, const uint8_t key[32]) {
  /* r is clamped: r &= 0x0ffffffc0ffffffc0ffffffc0fffffff */
  uint32_t t0 = ld32le(key), t1 = ld32le(key + 4), t2 = ld32le(key + 8), t3 = ld32le(key + 12);
  p->r[0] = t0 & 0x3ffffff;
  p->r[1] = ((t0 >> 26) | (t1 << 6)) & 0x3ffff03;
  p->r[2] = ((t1 >> 20) | (t2 << 12)) & 0x3ffc0ff;
  p->r[3] = ((t2 >> 14) | (t3 << 18)) & 0x3f03fff;
  p->r[4] = (t3 >> 8) & 0x00fffff;
  memset(p->h, 0, sizeof p->h);
  memcpy(p->s, key + 16, 16);
}

static void poly_block(orc_poly* p, const uint8_t m[16], uint32_t hibit) {
  uint32_t* h = p->h;
  const uint32_t* r = p->r;
  uint32_t t0 = ld32le(m), t1 = ld32le(m + 4), t2 = ld32le(m + 8), t3 = ld32le(m + 12);
  h[0] += t0 & 0x3ffffff;
  h[1] += ((t0 >> 26) | (t1 << 6)) & 0x3ffffff;
  h[2] += ((t1 >> 20) | (t2 << 12)) & 0x3ffffff;
  h[3] += ((t2 >> 14) | (t3 << 18)) & 0x3ffffff;
  h[4] += (t3 >> 8) | (hibit << 24);
  uint32_t s1 = r[1] * 5, s2 = r[2] * 5, s3 = r[3] * 5, s4 = r[4] * 5;
  uint64_t d0 = (uint64_t)h[0] * r[0] + (uint64_t)h[1] * s4 + (uint64_t)h[2] * s3 + (uint64_t)h[3] * s2 + (uint64_t)h[4] * s1;
  uint64_t d1 = (uint64_t)h[0] * r[1] + (uint64_t)h[1] * r[0] + (uint64_t)h[2] * s4 + (uint64_t)h[3] * s3 + (uint64_t)h[4] * s2;
  uint64_t d2 = (uint64_t)h[0] * r[2] + (uint64_t)h[1] * r[1] + (uint64_t)h[2] * r[0] + (uint64_t)h[3] * s4 + (uint64_t)h[4] * s3;
  uint64_t d3 = (uint64_t)h[0] * r[3] + (uint64_t)h[1] * r[2] + (uint64_t)h[2] * r[1] + (uint64_t)h[3] * r[0] + (uint64_t)h[4] * s4;
  uint64_t d4 = (uint64_t)h[0] * r[4] + (uint64_t)h[1] * r[3] + (uint64_t)h[2] * r[2] + (uint64_t)h[3] * r[1] + (uint64_t)h[4] * r[0];
  uint32_t c;
  c = (uint32_t)(d0 >> 26); h[0] = (uint32_t)d0 & 0x3ffffff; d1 += c;
  c = (uint32_t)(d1 >> 26); h[1] = (uint32_t)d1 & 0x3ffffff; d2 += c;
  c = (uint32_t)(d2 >> 26); h[2] = (uint32_t)d2 & 0x3ffffff; d3 += c;
  c = (uint32_t)(d3 >> 26); h[3] = (uint32_t)d3 & 0x3ffffff; d4 += c;
  c = (uint32_t)(d4 >> 26); h[4] = (uint32_t)d4 & 0x3ffffff;
  h[0] += c * 5; c = h[0] >> 26; h[0] &= 0x3ffffff; h[1] += c;
}

static void poly_finish(orc_poly* p, uint8_t tag[16]) {
  uint32_t* h = p->h;
  uint32_t c, g[5];
  c = h[1] >> 26; h[1] &= 0x3ffffff; h[2] += c;
  c = h[2] >> 26; h[2] &= 0x3ffffff; h[3] += c;
  c = h[3] >> 26; h[3] &= 0x3ffffff; h[4] += c;
  c = h[4] >> 26; h[4] &= 0x3ffffff; h[0] += c * 5;
  c = h[0] >> 26; h[0] &= 0x3ffffff; h[1] += c;
  /* g = h + 5 - 2^130; take g if it did not go negative */
  g[0] = h[0] + 5; c = g[0] >> 26; g[0] &= 0x3ffffff;
  g[1] = h[1] + c; c = g[1] >> 26; g[1] &= 0x3ffffff;
  g[2] = h[2] + c; c = g[2] >> 26; g[2] &= 0x3ffffff;
  g[3] = h[3] + c; c = g[3] >> 26; g[3] &= 0x3ffffff;
  g[4] = h[4] + c - (1u << 26);
  uint32_t use_g = (g[4] >> 31) ? 0 : 0xffffffffu; /* all-ones if g[4] did not underflow */
  for (int i = 0; i < 5; ++i) h[i] = (h[i] & ~use_g) | (g[i] & use_g);
  uint32_t w0 = h[0] | (h[1] << 26);
  uint32_t w1 = (h[1] >> 6) | (h[2] << 20);
  uint32_t w2 = (h[2] >> 12) | (h[3] << 14);
  uint32_t w3 = (h[3] >> 18) | (h[4] << 8);
  uint64_t f;
  f = (uint64_t)w0 + ld32le(p->s); st32le(tag, (uint32_t)f);
  f = (uint64_t)w1 + ld32le(p->s + 4) + (f >> 32); st32le(tag + 4, (uint32_t)f);
  f = (uint64_t)w2 + ld32le(p->s + 8) + (f >> 32); st32le(tag + 8, (uint32_t)f);
  f = (uint64_t)w3 + ld32le(p->s + 12) + (f >> 32); st32le(tag + 12, (uint32_t)f);
}

/* feed `len` bytes as zero-padded 16-byte blocks (the AEAD construction's pad16) */
static void poly_padded(orc_poly* p, const uint8_t* m, size_t len) {
  uint8_t blk[16];
  while (len >= 16) { poly_block(p, m, 1); m += 16; len -= 16; }
  if (len) { memset(blk, 0, 16); memcpy(blk, m, len); poly_block(p, blk, 1); }
}

void orc_poly1305(const uint8_t key[32], const uint8_t* msg, size_t len, uint8_t tag[16]) {
  orc_poly p;
  uint8_t blk[16];
  poly_init(&p, key);
  while (len >= 16) { poly_block(&p, msg, 1); msg += 16; len -= 16; }
  if (len) {  /* RFC 8439 §2.5.1: a final short block gets a 0x01 byte appended, no 2^128 */
    memset(blk, 0, 16); memcpy(blk, msg, len); blk[len] = 1; poly_block(&p, blk, 0);
  }
  poly_finish(&p, tag);
}

/* AEAD_CHACHA20_POLY1305, RFC 8439 §2.8 */
static void chacha_aead_tag(const uint8_t key[32], const uint8_t nonce[12], const uint8_t* aad,
                            size_t aad_len, const uint8_t* ct, size_t ct_len, uint8_t tag[16]) {
  uint8_t otk[64], lens[16];
  orc_poly p;
  orc_chacha20_block(key, 0, nonce, otk);
  poly_init(&p, otk);
  poly_padded(&p, aad, aad_len);
  poly_padded(&p, ct, ct_len);
  st64le(lens, aad_len); st64le(lens + 8, ct_len);
  poly_block(&p, lens, 1);
  poly_finish(&p, tag);
}

static void chacha_xor(const uint8_t key[32], const uint8_t nonce[12], uint8_t* buf, size_t len) {
  uint8_t ks[64];
  for (uint32_t ctr = 1; len; ++ctr) {
    orc_chacha20_block(key, ctr, nonce, ks);
    size_t n = len < 64 ? len : 64;
    for (size_t i = 0; i < n; ++i) buf[i] ^= ks[i];
    buf += n; len -= n;
  }
}

/* ---------------------------------------------------------------------------------------- */
/* AES-128, FIPS-197 (crate aes 0.8.4), byte-oriented; S-box built from GF(2^8) inverse.     */
static uint8_t g_sbox[256];
static pthread_once_t g_sbox_once = PTHREAD_ONCE_INIT;

static uint8_t gf8_mul(uint8_t a, uint8_t b) {
  uint8_t r = 0;
  while (b) { if (b & 1) r ^= a; a = (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0)); b >>= 1; }
  return r;
}
static void build_sbox(void) {
  for (int x = 0; x < 256; ++x) {
    uint8_t inv = 0;
    if (x) for (int y = 1; y < 256; ++y) if (gf8_mul((uint8_t)x, (uint8_t)y) == 1) { inv = (uint8_t)y; break; }
    uint8_t s = inv, r = inv;
    for (int i = 0; i < 4; ++i) { r = (uint8_t)((r << 1) | (r >> 7)); s ^= r; }
    g_sbox[x] = s ^ 0x63;
  }
}
static const uint8_t* sbox(void) { pthread_once(&g_sbox_once, build_sbox); return g_sbox; }

void orc_aes128_expand(const uint8_t key[16], uint32_t rk[44]) {
  const uint8_t* S = sbox();
  uint8_t rcon = 1;
  for (int i = 0; i < 4; ++i) rk[i] = ld32be(key + 4 * i);
  for (int i = 4; i < 44; ++i) {
    uint32_t t = rk[i - 1];
    if (i % 4 == 0) {
      t = (t << 8) | (t >> 24);
      t = ((uint32_t)S[t >> 24] << 24) | ((uint32_t)S[(t >> 16) & 0xff] << 16) |
          ((uint32_t)S[(t >> 8) & 0xff] << 8) | S[t & 0xff];
      t ^= (uint32_t)rcon << 24;
      rcon = gf8_mul(rcon, 2);
    }
    rk[i] = rk[i - 4] ^ t;
  }
}

void orc_aes128_encrypt(const uint32_t rk[44], const uint8_t in[16], uint8_t out[16]) {
  const uint8_t* S = sbox();
  uint8_t st[16], t[16];
  for (int c = 0; c < 4; ++c) st32be(st + 4 * c, ld32be(in + 4 * c) ^ rk[c]);
  for (int round = 1; round <= 10; ++round) {
    for (int i = 0; i < 16; ++i) t[i] = S[st[i]];                       /* SubBytes */
    for (int c = 0; c < 4; ++c)                                         /* ShiftRows */
      for (int r = 0; r < 4; ++r) st[4 * c + r] = t[4 * ((c + r) % 4) + r];
    if (round != 10)                                                    /* MixColumns */
      for (int c = 0; c < 4; ++c) {
        uint8_t a0 = st[4 * c], a1 = st[4 * c + 1], a2 = st[4 * c + 2], a3 = st[4 * c + 3];
        st[4 * c + 0] = gf8_mul(a0, 2) ^ gf8_mul(a1, 3) ^ a2 ^ a3;
        st[4 * c + 1] = a0 ^ gf8_mul(a1, 2) ^ gf8_mul(a2, 3) ^ a3;
        st[4 * c + 2] = a0 ^ a1 ^ gf8_mul(a2, 2) ^ gf8_mul(a3, 3);
        st[4 * c + 3] = gf8_mul(a0, 3) ^ a1 ^ a2 ^ gf8_mul(a3, 2);
      }
    for (int c = 0; c < 4; ++c) st32be(st + 4 * c, ld32be(st + 4 * c) ^ rk[4 * round + c]);
  }
  memcpy(out, st, 16);
}

/* GF(2^128) multiply, SP 800-38D §6.3 Algorithm 1 (bit-reflected, R = 0xE1 || 0^120). */
void orc_gf128_mul(const uint8_t x[16], const uint8_t y[16], uint8_t out[16]) {
  uint8_t z[16] = {0}, v[16];
  memcpy(v, y, 16);
  for (int i = 0; i < 128; ++i) {
    if ((x[i / 8] >> (7 - i % 8)) & 1) for (int k = 0; k < 16; ++k) z[k] ^= v[k];
    int lsb = v[15] & 1;
    for (int k = 15; k > 0; --k) v[k] = (uint8_t)((v[k] >> 1) | (v[k - 1] << 7));
    v[0] >>= 1;
    if (lsb) v[0] ^= 0xe1;
  }
  memcpy(out, z, 16);
}

static void ghash_padded(const uint8_t h[16], uint8_t y[16], const uint8_t* m, size_t len) {
  uint8_t blk[16];
  while (len) {
    size_t n = len < 16 ? len : 16;
    memset(blk, 0, 16); memcpy(blk, m, n);
    for (int k = 0; k < 16; ++k) y[k] ^= blk[k];
    orc_gf128_mul(y, h, y);
    m += n; len -= n;
  }
}

void orc_ghash(const uint8_t h[16], const uint8_t* aad, size_t aad_len, const uint8_t* ct,
               size_t ct_len, uint8_t out[16]) {
  uint8_t y[16] = {0}, lens[16];
  ghash_padded(h, y, aad, aad_len);
  ghash_padded(h, y, ct, ct_len);
  st64be(lens, (uint64_t)aad_len * 8); st64be(lens + 8, (uint64_t)ct_len * 8);
  ghash_padded(h, y, lens, 16);
  memcpy(out, y, 16);
}

/* AES-128-GCM with a 96-bit IV, SP 800-38D §7 (crate aes-gcm 0.10.3): J0 = IV || 0^31 || 1,
 * keystream from inc32(J0), tag = E_K(J0) xor GHASH_H(A, C), H = E_K(0^128). */
static void gcm_ctr(const uint32_t rk[44], const uint8_t nonce[12], uint8_t* buf, size_t len) {
  uint8_t cb[16], ks[16];
  memcpy(cb, nonce, 12);
  for (uint32_t ctr = 2; len; ++ctr) {
    st32be(cb + 12, ctr);
    orc_aes128_encrypt(rk, cb, ks);
    size_t n = len < 16 ? len : 16;
    for (size_t i = 0; i < n; ++i) buf[i] ^= ks[i];
    buf += n; len -= n;
  }
}
static void gcm_tag(const uint32_t rk[44], const uint8_t nonce[12], const uint8_t* aad,
                    size_t aad_len, const uint8_t* ct, size_t ct_len, uint8_t tag[16]) {
  uint8_t h[16] = {0}, j0[16], ej0[16], s[16];
  orc_aes128_encrypt(rk, h, h);
  memcpy(j0, nonce, 12); st32be(j0 + 12, 1);
  orc_aes128_encrypt(rk, j0, ej0);
  orc_ghash(h, aad, aad_len, ct, ct_len, s);
  for (int i = 0; i < 16; ++i) tag[i] = s[i] ^ ej0[i];
}

/* ---------------------------------------------------------------------------------------- */
/* Aead::seal_in_place / open_in_place adapters: ref src/crypto/rustcrypto.rs:38-94 (AES)
 * and :111-165 (ChaCha): nonce.len() != 12 -> Crypto; buf.len() < payload+16 ->
 * BufferTooSmall{needed}; ct < 16 -> Crypto; tag mismatch -> Crypto (buffer unchanged:
 * both 0.10 crates verify before decrypting). ct_len > buf.len() panics in the reference
 * (rustcrypto.rs:83,154): reported here as MQ_ERR_INVALID_ARG. */
static size_t suite_key_len(uint32_t suite) {
  return suite == MQ_SUITE_AES128GCM ? 16 : suite == MQ_SUITE_CHACHA20 ? 32 : 0;
}

int orc_aead_seal(uint32_t suite, const uint8_t* key, size_t key_len, const uint8_t* nonce,
                  size_t nonce_len, const uint8_t* aad, size_t aad_len, uint8_t* buf,
                  size_t buf_len, size_t payload_len, size_t* out_len, size_t* needed) {
  if (!suite_key_len(suite) || key_len != suite_key_len(suite)) return MQ_ERR_CRYPTO;
  if (nonce_len != 12) return MQ_ERR_CRYPTO;
  size_t total = payload_len + 16;
  if (buf_len < total) { if (needed) *needed = total; return MQ_ERR_BUFFER_TOO_SMALL; }
  if (suite == MQ_SUITE_CHACHA20) {
    chacha_xor(key, nonce, buf, payload_len);
    chacha_aead_tag(key, nonce, aad, aad_len, buf, payload_len, buf + payload_len);
  } else {
    uint32_t rk[44];
    orc_aes128_expand(key, rk);
    gcm_ctr(rk, nonce, buf, payload_len);
    gcm_tag(rk, nonce, aad, aad_len, buf, payload_len, buf + payload_len);
  }
  if (out_len) *out_len = total;
  return MQ_OK;
}

int orc_aead_open(uint32_t suite, const uint8_t* key, size_t key_len, const uint8_t* nonce,
                  size_t nonce_len, const uint8_t* aad, size_t aad_len, uint8_t* buf,
                  size_t buf_len, size_t ct_len, size_t* out_len) {
  if (!suite_key_len(suite) || key_len != suite_key_len(suite)) return MQ_ERR_CRYPTO;
  if (nonce_len != 12) return MQ_ERR_CRYPTO;
  if (ct_len < 16) return MQ_ERR_CRYPTO;
  if (ct_len > buf_len) return MQ_ERR_INVALID_ARG;
  size_t pt_len = ct_len - 16;
  uint8_t tag[16];
  uint32_t rk[44];
  if (suite == MQ_SUITE_CHACHA20) {
    chacha_aead_tag(key, nonce, aad, aad_len, buf, pt_len, tag);
  } else {
    orc_aes128_expand(key, rk);
    gcm_tag(rk, nonce, aad, aad_len, buf, pt_len, tag);
  }
  uint8_t diff = 0;
  for (int i = 0; i < 16; ++i) diff |= (uint8_t)(tag[i] ^ buf[pt_len + i]);
  if (diff) return MQ_ERR_CRYPTO;
  if (suite == MQ_SUITE_CHACHA20) chacha_xor(key, nonce, buf, pt_len);
  else gcm_ctr(rk, nonce, buf, pt_len);
  if (out_len) *out_len = pt_len;
  return MQ_OK;
}

/* HeaderProtection::mask: AES: ref rustcrypto.rs:175-186 (AES-ECB(hp, sample)[0..5]);
 * ChaCha: :197-220 (counter = LE32(sample[0..4]), nonce = sample[4..16], 5 keystream bytes).
 * sample.len() < 16 panics in the reference -> MQ_ERR_INVALID_ARG here. */
int orc_hp_mask(uint32_t suite, const uint8_t* hp_key, size_t key_len, const uint8_t* sample,
                size_t sample_len, uint8_t mask[5]) {
  if (sample_len < 16) return MQ_ERR_INVALID_ARG;
  if (suite == MQ_SUITE_AES128GCM) {
    if (key_len != 16) return MQ_ERR_CRYPTO;
    uint32_t rk[44];
    uint8_t blk[16];
    orc_aes128_expand(hp_key, rk);
    orc_aes128_encrypt(rk, sample, blk);
    memcpy(mask, blk, 5);
  } else if (suite == MQ_SUITE_CHACHA20) {
    if (key_len != 32) return MQ_ERR_CRYPTO;
    uint8_t blk[64];
    orc_chacha20_block(hp_key, ld32le(sample), sample + 4, blk);
    memcpy(mask, blk, 5);
  } else {
    return MQ_ERR_CRYPTO;
  }
  return MQ_OK;
}

/* DirectionalKeys::nonce, ref src/crypto/mod.rs:66-74 */
void orc_nonce(const uint8_t iv[12], uint64_t pn, uint8_t nonce[12]) {
  memcpy(nonce, iv, 12);
  for (int i = 0; i < 8; ++i) nonce[4 + i] ^= (uint8_t)(pn >> (56 - 8 * i));
}

/* ---------------------------------------------------------------------------------------- */
/* SHA-256 (FIPS 180-4), HMAC (RFC 2104), HKDF (RFC 5869): ref rustcrypto.rs:9-24           */
static const uint32_t K256[64] = {
  0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
  0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
  0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
  0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
  0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
  0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
  0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
  0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

static uint32_t rotr32(uint32_t x, int r) { return (x >> r) | (x << (32 - r)); }

static void sha256_compress(uint32_t st[8], const uint8_t blk[64]) {
  uint32_t w[64], a, b, c, d, e, f, g, h;
  for (int i = 0; i < 16; ++i) w[i] = ld32be(blk + 4 * i);
  for (int i = 16; i < 64; ++i) {
    uint32_t s0 = rotr32(w[i - 15], 7) ^ rotr32(w[i - 15], 18) ^ (w[i - 15] >> 3);
    uint32_t s1 = rotr32(w[i - 2], 17) ^ rotr32(w[i - 2], 19) ^ (w[i - 2] >> 10);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  a = st[0]; b = st[1]; c = st[2]; d = st[3]; e = st[4]; f = st[5]; g = st[6]; h = st[7];
  for (int i = 0; i < 64; ++i) {
    uint32_t S1 = rotr32(e, 6) ^ rotr32(e, 11) ^ rotr32(e, 25);
    uint32_t ch = (e & f) ^ (~e & g);
    uint32_t t1 = h + S1 + ch + K256[i] + w[i];
    uint32_t S0 = rotr32(a, 2) ^ rotr32(a, 13) ^ rotr32(a, 22);
    uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
    uint32_t t2 = S0 + mj;
    h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

void orc_sha256(const uint8_t* msg, size_t len, uint8_t out[32]) {
  uint32_t st[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                    0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  uint8_t blk[64];
  size_t total = len;
  while (len >= 64) { sha256_compress(st, msg); msg += 64; len -= 64; }
  memset(blk, 0, 64); memcpy(blk, msg, len); blk[len] = 0x80;
  if (len >= 56) { sha256_compress(st, blk); memset(blk, 0, 64); }
  st64be(blk + 56, (uint64_t)total * 8);
  sha256_compress(st, blk);
  for (int i = 0; i < 8; ++i) st32be(out + 4 * i, st[i]);
}

void orc_hmac_sha256(const uint8_t* key, size_t key_len, const uint8_t* msg, size_t len,
                     uint8_t out[32]) {
  uint8_t k[64] = {0}, ipad[64], opad[64], inner[32];
  if (key_len > 64) orc_sha256(key, key_len, k); else memcpy(k, key, key_len);
  for (int i = 0; i < 64; ++i) { ipad[i] = k[i] ^ 0x36; opad[i] = k[i] ^ 0x5c; }
  uint8_t* buf = (uint8_t*)malloc(64 + len + 32);
  memcpy(buf, ipad, 64); memcpy(buf + 64, msg, len);
  orc_sha256(buf, 64 + len, inner);
  memcpy(buf, opad, 64); memcpy(buf + 64, inner, 32);
  orc_sha256(buf, 96, out);
  free(buf);
}

void orc_hkdf_extract(const uint8_t* salt, size_t salt_len, const uint8_t* ikm, size_t ikm_len,
                      uint8_t prk[32]) {
  orc_hmac_sha256(salt, salt_len, ikm, ikm_len, prk);
}

int orc_hkdf_expand(const uint8_t* prk, size_t prk_len, const uint8_t* info, size_t info_len,
                    uint8_t* okm, size_t okm_len) {
  if (prk_len < 32 || okm_len > 255 * 32) return MQ_ERR_CRYPTO;
  uint8_t t[32], *buf = (uint8_t*)malloc(32 + info_len + 1);
  size_t tlen = 0, done = 0;
  for (uint8_t i = 1; done < okm_len; ++i) {
    memcpy(buf, t, tlen); memcpy(buf + tlen, info, info_len); buf[tlen + info_len] = i;
    orc_hmac_sha256(prk, prk_len, buf, tlen + info_len + 1, t);
    tlen = 32;
    size_t n = okm_len - done < 32 ? okm_len - done : 32;
    memcpy(okm + done, t, n); done += n;
  }
  free(buf);
  return MQ_OK;
}

/* hkdf_expand_label, ref src/crypto/key_schedule.rs:23-55 (80-byte info limit -> Crypto) */
int orc_hkdf_expand_label(const uint8_t* secret, size_t secret_len, const uint8_t* label,
                          size_t label_len, const uint8_t* ctx, size_t ctx_len, uint8_t* out,
                          size_t out_len) {
  uint8_t info[80];
  size_t full = 6 + label_len, info_len = 2 + 1 + full + 1 + ctx_len;
  if (info_len > 80) return MQ_ERR_CRYPTO;
  info[0] = (uint8_t)(out_len >> 8); info[1] = (uint8_t)out_len; info[2] = (uint8_t)full;
  memcpy(info + 3, "tls13 ", 6); memcpy(info + 9, label, label_len);
  info[3 + full] = (uint8_t)ctx_len;
  if (ctx_len) memcpy(info + 4 + full, ctx, ctx_len);
  return orc_hkdf_expand(secret, secret_len, info, info_len, out, out_len);
}

/* derive_initial_secrets, ref key_schedule.rs:60-72 (salt :10-13) */
int orc_derive_initial_secrets(const uint8_t* dcid, size_t dcid_len, uint8_t client[32],
                               uint8_t server[32]) {
  static const uint8_t salt[20] = {0x38, 0x76, 0x2c, 0xf7, 0xf5, 0x59, 0x34, 0xb3, 0x4d, 0x17,
                                   0x9a, 0xe6, 0xa4, 0xc8, 0x0c, 0xad, 0xcc, 0xbb, 0x7f, 0x0a};
  uint8_t initial[32];
  orc_hkdf_extract(salt, 20, dcid, dcid_len, initial);
  int rc = orc_hkdf_expand_label(initial, 32, (const uint8_t*)"client in", 9, NULL, 0, client, 32);
  if (rc) return rc;
  return orc_hkdf_expand_label(initial, 32, (const uint8_t*)"server in", 9, NULL, 0, server, 32);
}

/* derive_packet_keys + derive_directional_keys, ref key_schedule.rs:79-90,123-151 */
int orc_derive_key_material(uint32_t suite, const uint8_t* secret, size_t secret_len,
                            mq_key_material* out) {
  size_t klen = suite_key_len(suite), hplen = klen > 16 ? klen : 16;
  if (!klen) return MQ_ERR_CRYPTO;
  memset(out, 0, sizeof *out);
  out->suite = suite;
  int rc = orc_hkdf_expand_label(secret, secret_len, (const uint8_t*)"quic key", 8, NULL, 0, out->key, klen);
  if (!rc) rc = orc_hkdf_expand_label(secret, secret_len, (const uint8_t*)"quic iv", 7, NULL, 0, out->iv, 12);
  if (!rc) rc = orc_hkdf_expand_label(secret, secret_len, (const uint8_t*)"quic hp", 7, NULL, 0, out->hp, hplen);
  return rc;
}

/* ---------------------------------------------------------------------------------------- */
/* packet numbers, ref src/packet/number.rs:9-26 (pn_length) and :52-70 (decode_pn)          */
size_t orc_pn_length(uint64_t full_pn, uint64_t largest_acked) {
  uint64_t num_unacked = full_pn > largest_acked ? full_pn - largest_acked : 1;
  if (num_unacked < (1u << 7)) return 1;
  if (num_unacked < (1u << 15)) return 2;
  if (num_unacked < (1u << 23)) return 3;
  return 4;
}

uint64_t orc_decode_pn(uint32_t truncated, size_t pn_len, uint64_t largest_pn) {
  uint64_t pn_nbits = (uint64_t)pn_len * 8;
  uint64_t pn_win = 1ull << pn_nbits, pn_hwin = pn_win / 2, pn_mask = pn_win - 1;
  uint64_t expected = largest_pn + 1;
  uint64_t candidate = (expected & ~pn_mask) | truncated;
  if (candidate + pn_hwin <= expected && candidate + pn_win <= (1ull << 62)) return candidate + pn_win;
  if (candidate > expected + pn_hwin && candidate >= pn_win) return candidate - pn_win;
  return candidate;
}

/* ---------------------------------------------------------------------------------------- */
/* Composites. Descriptor semantics are those of include/mq_aead.h; status != MQ_OK leaves the
 * packet bytes unchanged (the batch contract).                                              */
static const size_t MAX_VARINT = (1ull << 62) - 1;

/* TLS 1.3 records over the same Aead (descriptor flag MQ_PKT_TLS_RECORD): a record is
 * [5-byte header][data][inner content type][tag]. seal: ref src/tcp_tls/connection.rs:561-600
 * (encrypt_into: header 23, 0x0303, u16 length; plaintext || inner type sealed with AAD = header)
 * and record.rs:88-113 (seal_record); nonce = iv ^ (0^4 || BE64(seq)) = record.rs:70-78. */
static int orc_record_checks(const mq_pkt_desc* d) {
  if ((d->flags & MQ_PKT_TLS_RECORD) != MQ_PKT_TLS_RECORD || d->pn_offset != 5 || d->pn_len != 0 ||
      d->len > 5u + 0xFFFFu)
    return MQ_ERR_INVALID_ARG;
  return MQ_OK;
}

static int orc_seal_record(const mq_key_material* km, uint8_t* rec, const mq_pkt_desc* d) {
  size_t klen = suite_key_len(km->suite);
  int rc = orc_record_checks(d);
  if (rc) return rc;
  if (d->len < 5 + 1 + 16) return MQ_ERR_BUFFER_TOO_SMALL; /* record.rs:97-99 */
  size_t inner_len = d->len - 5 - 16, out_len;
  uint8_t* tmp = (uint8_t*)malloc(d->len);
  memcpy(tmp, rec, d->len);
  uint16_t outer = (uint16_t)(d->len - 5);
  tmp[0] = 23; tmp[1] = 3; tmp[2] = 3; tmp[3] = (uint8_t)(outer >> 8); tmp[4] = (uint8_t)outer;
  tmp[5 + inner_len - 1] = (uint8_t)d->reserved;
  uint8_t nonce[12];
  orc_nonce(km->iv, d->pn, nonce);
  rc = orc_aead_seal(km->suite, km->key, klen, nonce, 12, tmp, 5, tmp + 5, d->len - 5, inner_len, &out_len, NULL);
  if (rc == MQ_OK) memcpy(rec, tmp, d->len);
  free(tmp);
  return rc;
}

/* open: ref record.rs:122-143 (open_record) and connection.rs:546-556 (find_inner_content_type:
 * last non-zero byte, ContentType::from_byte accepts 20..23, else Error::Tls with the plaintext
 * already decrypted in place). *info = data_len | inner_type << 32. */
static int orc_open_record(const mq_key_material* km, uint8_t* rec, const mq_pkt_desc* d, uint64_t* info) {
  size_t klen = suite_key_len(km->suite), pt_len;
  int rc = orc_record_checks(d);
  if (rc) return rc;
  if (d->len < 5 + 16) return MQ_ERR_CRYPTO; /* open_in_place: ciphertext shorter than the tag */
  uint8_t* tmp = (uint8_t*)malloc(d->len);
  memcpy(tmp, rec, d->len);
  uint8_t nonce[12];
  orc_nonce(km->iv, d->pn, nonce);
  rc = orc_aead_open(km->suite, km->key, klen, nonce, 12, tmp, 5, tmp + 5, d->len - 5, d->len - 5, &pt_len);
  if (rc == MQ_OK) {
    size_t pos = pt_len;
    while (pos > 0 && tmp[5 + pos - 1] == 0) --pos;
    uint8_t ct = pos ? tmp[5 + pos - 1] : 0;
    if (ct < 20 || ct > 23) rc = MQ_ERR_TLS;
    else if (info) *info = (uint64_t)(pos - 1) | ((uint64_t)ct << 32);
    memcpy(rec, tmp, d->len); /* decrypted in place even when the content type is bad */
  }
  free(tmp);
  return rc;
}

/* send: ref src/connection/transmit.rs:625-755 (build_and_encrypt_packet) and :499-622 */
int orc_protect_packet(const mq_key_material* km, uint8_t* pkt, const mq_pkt_desc* d) {
  int no_hp = (d->flags & MQ_PKT_NO_HP) != 0;
  size_t klen = suite_key_len(km->suite);
  if (!klen) return MQ_ERR_SUITE;
  if (d->flags & 0x04) return orc_seal_record(km, pkt, d);
  if (!no_hp && (d->pn_len < 1 || d->pn_len > 4)) return MQ_ERR_INVALID_ARG;
  size_t hdr = (size_t)d->pn_offset + d->pn_len;
  if ((size_t)d->len < hdr + 16) return MQ_ERR_BUFFER_TOO_SMALL;
  /* transmit.rs:593-597 / :721-725: sample_offset + 16 > total_pkt_len -> Err(Crypto) */
  if (!no_hp && (size_t)d->pn_offset + 4 + 16 > (size_t)d->len) return MQ_ERR_CRYPTO;
  size_t payload_len = d->len - hdr - 16;
  uint8_t* tmp = (uint8_t*)malloc(d->len);
  memcpy(tmp, pkt, d->len);
  uint8_t nonce[12];
  orc_nonce(km->iv, d->pn, nonce);
  size_t out_len;
  int rc = orc_aead_seal(km->suite, km->key, klen, nonce, 12, tmp, hdr, tmp + hdr,
                         d->len - hdr, payload_len, &out_len, NULL);
  if (rc == MQ_OK && !no_hp) {
    uint8_t mask[5];
    rc = orc_hp_mask(km->suite, km->hp, klen > 16 ? klen : 16, tmp + d->pn_offset + 4, 16, mask);
    if (rc == MQ_OK) {
      tmp[0] ^= mask[0] & ((d->flags & MQ_PKT_LONG_HEADER) ? 0x0f : 0x1f);
      for (int i = 0; i < d->pn_len; ++i) tmp[d->pn_offset + i] ^= mask[1 + i];
    }
  }
  if (rc == MQ_OK) memcpy(pkt, tmp, d->len);
  free(tmp);
  return rc;
}

/* receive: ref src/connection/recv.rs:340-421 (recv_short) and :953-1025 (decrypt_long_packet) */
int orc_unprotect_packet(const mq_key_material* km, uint8_t* pkt, const mq_pkt_desc* d,
                         uint64_t* pn_out) {
  int no_hp = (d->flags & MQ_PKT_NO_HP) != 0;
  size_t klen = suite_key_len(km->suite);
  if (!klen) return MQ_ERR_SUITE;
  if (d->flags & 0x04) return orc_open_record(km, pkt, d, pn_out);
  /* recv.rs:356-360 (recv_short) / :962-965 (decrypt_long_packet): copy into a 2048-B stack buffer,
   * Err(BufferTooSmall { needed: len }) above that — before the sample check (:364-366) */
  if (!no_hp && !(d->flags & MQ_PKT_NO_RECV_LIMIT) && d->len > MQ_RECV_MAX_PACKET) return MQ_ERR_BUFFER_TOO_SMALL;
  uint8_t* tmp = (uint8_t*)malloc(d->len ? d->len : 1);
  memcpy(tmp, pkt, d->len);
  size_t pn_len;
  uint64_t pn;
  int rc = MQ_OK;
  if (no_hp) {
    pn_len = d->pn_len;
    pn = d->pn;
    if ((size_t)d->len < (size_t)d->pn_offset + pn_len) rc = MQ_ERR_CRYPTO;
  } else {
    /* recv.rs:364-366 / :970-973 */
    if ((size_t)d->pn_offset + 4 + 16 > (size_t)d->len) { free(tmp); return MQ_ERR_CRYPTO; }
    uint8_t mask[5];
    rc = orc_hp_mask(km->suite, km->hp, klen > 16 ? klen : 16, tmp + d->pn_offset + 4, 16, mask);
    if (rc) { free(tmp); return rc; }
    tmp[0] ^= mask[0] & ((d->flags & MQ_PKT_LONG_HEADER) ? 0x0f : 0x1f);
    pn_len = (size_t)(tmp[0] & 3) + 1;
    uint32_t trunc = 0;
    for (size_t i = 0; i < pn_len; ++i) {
      tmp[d->pn_offset + i] ^= mask[1 + i];
      trunc = (trunc << 8) | tmp[d->pn_offset + i];
    }
    pn = orc_decode_pn(trunc, pn_len, d->pn);
    if (pn > MAX_VARINT) { free(tmp); return MQ_ERR_PROTOCOL; } /* recv.rs:393-395 */
  }
  if (rc == MQ_OK) {
    size_t hdr = (size_t)d->pn_offset + pn_len, ct_len = d->len - hdr;
    uint8_t nonce[12];
    orc_nonce(km->iv, pn, nonce);
    size_t pt_len;
    rc = orc_aead_open(km->suite, km->key, klen, nonce, 12, tmp, hdr, tmp + hdr, ct_len, ct_len,
                       &pt_len);
  }
  if (rc == MQ_OK) {
    memcpy(pkt, tmp, d->len);
    if (pn_out) *pn_out = pn;
  }
  free(tmp);
  return rc;
}

/* ---------------------------------------------------------------------------------------- */
/* Send composite from frames: ref src/connection/transmit.rs:499-622 (Initial, pad_to_min) and
 * :625-755 (Handshake / 1-RTT), with the header codecs of src/packet/long_header.rs:214-314,
 * short_header.rs:33-47, number.rs:32-43 and varint.rs:72-110. Writes the protected packet to
 * out[0..] only on success; *len = its length, or `needed` of a BufferTooSmall.             */
static size_t orc_varint_len(uint64_t v) { return v < 64 ? 1 : v < 16384 ? 2 : v < (1u << 30) ? 4 : 8; }
static size_t orc_put_varint(uint8_t* p, uint64_t v) {
  size_t n = orc_varint_len(v);
  for (size_t i = 0; i < n; ++i) p[i] = (uint8_t)(v >> (8 * (n - 1 - i)));
  p[0] |= (uint8_t)(n == 1 ? 0 : n == 2 ? 0x40 : n == 4 ? 0x80 : 0xc0);
  return n;
}
/* encode_initial_header (long_header.rs:214-265; token always empty, transmit.rs:519) /
 * encode_handshake_header (:272-314) */
static size_t orc_long_header(uint8_t* h, const mq_conn_send* c, int initial, size_t pn_len,
                              uint64_t payload_length) {
  size_t p = 0;
  h[p++] = (uint8_t)((initial ? 0xC0 : 0xE0) | ((pn_len - 1) & 3));
  h[p++] = 0; h[p++] = 0; h[p++] = 0; h[p++] = 1; /* QUIC_VERSION_1 */
  h[p++] = c->dcid_len; memcpy(h + p, c->dcid, c->dcid_len); p += c->dcid_len;
  h[p++] = c->scid_len; memcpy(h + p, c->scid, c->scid_len); p += c->scid_len;
  if (initial) h[p++] = 0; /* token length 0 */
  p += orc_put_varint(h + p, payload_length);
  return p;
}

int orc_protect_frames(const mq_key_material* km, const mq_conn_send* c, const mq_send_req* r,
                       const uint8_t* frames, uint8_t* out, uint64_t out_cap, uint32_t* len) {
  size_t pn_len = orc_pn_length(r->pn, r->largest_acked), frame_len = r->frame_len, pad = 0, hdr;
  uint8_t h[128];
  int is_long = r->level != MQ_LEVEL_APPLICATION;
  if (r->level > MQ_LEVEL_APPLICATION || c->dcid_len > 20 || c->scid_len > 20) return MQ_ERR_INVALID_ARG;
  if (r->level == MQ_LEVEL_INITIAL) {
    uint64_t payload_length = pn_len + frame_len + 16;
    hdr = orc_long_header(h, c, 1, pn_len, payload_length);
    if ((r->flags & MQ_SEND_PAD_TO_MIN) && hdr + payload_length < 1200) pad = 1200 - (hdr + payload_length);
    hdr = orc_long_header(h, c, 1, pn_len, pn_len + frame_len + pad + 16); /* :551-558 */
  } else {
    size_t min_enc = pn_len >= 20 ? 0 : 20 - pn_len; /* :644-649 */
    if (frame_len + 16 < min_enc) pad = min_enc - frame_len - 16;
    if (r->level == MQ_LEVEL_HANDSHAKE) {
      hdr = orc_long_header(h, c, 0, pn_len, pn_len + frame_len + pad + 16);
    } else {
      h[0] = (uint8_t)(0x40 | ((c->key_phase & 1) << 2) | (pn_len - 1)); /* :677-679 */
      memcpy(h + 1, c->dcid, c->dcid_len);
      hdr = 1 + (size_t)c->dcid_len;
    }
  }
  if (out_cap < hdr) { *len = (uint32_t)hdr; return MQ_ERR_BUFFER_TOO_SMALL; }             /* encode_*_header */
  if (out_cap < hdr + pn_len) { *len = (uint32_t)pn_len; return MQ_ERR_BUFFER_TOO_SMALL; } /* encode_pn */
  size_t total = hdr + pn_len + frame_len + pad + 16;
  if (total > out_cap) { *len = (uint32_t)total; return MQ_ERR_BUFFER_TOO_SMALL; }         /* :566-570, :693-697 */
  uint8_t* pkt = (uint8_t*)calloc(total, 1);
  memcpy(pkt, h, hdr);
  for (size_t i = 0; i < pn_len; ++i) pkt[hdr + i] = (uint8_t)(r->pn >> (8 * (pn_len - 1 - i)));
  memcpy(pkt + hdr + pn_len, frames, frame_len); /* then PADDING frames (0x00) and the tag room */
  mq_pkt_desc d;
  memset(&d, 0, sizeof d);
  d.len = (uint32_t)total; d.pn = r->pn; d.pn_offset = (uint16_t)hdr; d.pn_len = (uint8_t)pn_len;
  d.flags = is_long ? MQ_PKT_LONG_HEADER : 0;
  int rc = orc_protect_packet(km, pkt, &d);
  if (rc == MQ_OK) { memcpy(out, pkt, total); *len = (uint32_t)total; }
  free(pkt);
  return rc;
}

void orc_batch_protect(const mq_key_material* rows, uint32_t n_rows, const mq_conn_send* conns,
                       uint32_t n_conns, const uint8_t* frames, uint64_t frames_len, uint8_t* out,
                       uint64_t out_len, const mq_send_req* req, uint32_t n, uint8_t* status,
                       uint32_t* pkt_len, uint32_t suite_hint) {
  for (uint32_t i = 0; i < n; ++i) {
    const mq_send_req* r = &req[i];
    int st;
    uint32_t len = 0;
    if (r->conn >= n_conns || r->level > MQ_LEVEL_APPLICATION ||
        r->frames_offset + (uint64_t)r->frame_len > frames_len ||
        r->out_offset + (uint64_t)r->out_cap > out_len || conns[r->conn].key_row[r->level] >= n_rows) {
      st = MQ_ERR_INVALID_ARG;
    } else {
      const mq_key_material* km = &rows[conns[r->conn].key_row[r->level]];
      if ((suite_hint != MQ_SUITE_MIXED && km->suite != suite_hint) ||
          (r->level == MQ_LEVEL_INITIAL && km->suite != MQ_SUITE_AES128GCM))
        st = MQ_ERR_SUITE;
      else
        st = orc_protect_frames(km, &conns[r->conn], r, frames + r->frames_offset, out + r->out_offset,
                                r->out_cap, &len);
    }
    status[i] = (uint8_t)st;
    pkt_len[i] = len;
  }
}

/* ---------------------------------------------------------------------------------------- */
/* Receive composite over raw datagrams: ref src/connection/recv.rs:189-265 (datagram loop,
 * errors drop the packet), :268-337 + :953-1025 (Initial / Handshake), :340-510 (1-RTT with key
 * phase), src/packet/coalesce.rs:26-133 and long_header.rs:92-206 (parsing), varint.rs (decode).
 * Frame dispatch is out of scope: a packet that opens counts as processed (largest_recv_pn).   */
static int orc_get_varint(const uint8_t* p, size_t avail, uint64_t* v, size_t* used) {
  if (avail < 1) return MQ_ERR_BUFFER_TOO_SMALL;
  size_t n = (size_t)1 << (p[0] >> 6);
  if (avail < n) return MQ_ERR_BUFFER_TOO_SMALL;
  uint64_t x = p[0] & 0x3f;
  for (size_t i = 1; i < n; ++i) x = (x << 8) | p[i];
  *v = x; *used = n;
  return MQ_OK;
}

/* CoalescedPackets::next (coalesce.rs:29-132): *plen = packet length; *kind = 0 Initial,
 * 1 0-RTT, 2 Handshake, 3 Retry, 4 short, 5 version negotiation; *pn_off / *length for Initial /
 * Handshake (parse_*_header). Returns non-zero when the datagram's iteration stops (error). */
static int orc_next_packet(const uint8_t* rem, size_t avail, size_t* plen, int* kind, size_t* pn_off,
                           uint64_t* length) {
  if (!(rem[0] & 0x80)) { *plen = avail; *kind = 4; return 0; }
  if (avail < 6) return 1;
  uint32_t version = ((uint32_t)rem[1] << 24) | ((uint32_t)rem[2] << 16) | ((uint32_t)rem[3] << 8) | rem[4];
  if (version == 0) { *plen = avail; *kind = 5; return 0; }
  size_t pos = 6 + rem[5];
  if (pos >= avail) return 1; /* pos + dcid_len >= len (:62) */
  size_t scid = rem[pos++];
  if (pos + scid > avail) return 1;
  pos += scid;
  int type = (rem[0] & 0x30) >> 4;
  uint64_t v;
  size_t used;
  if (type == 0) {
    if (orc_get_varint(rem + pos, avail - pos, &v, &used)) return 1;
    pos += used;
    if (v > avail - pos) return 1;
    pos += (size_t)v;
  }
  if (type == 3) { *plen = avail; *kind = 3; return 0; }
  if (orc_get_varint(rem + pos, avail - pos, &v, &used)) return 1;
  pos += used;
  if (v > avail - pos) return 1;
  *plen = pos + (size_t)v; *kind = type; *pn_off = pos; *length = v;
  return 0;
}

/* HP removal + decode_pn + open of one packet at pkt[0..len) with keys `km` (recv.rs:363-421 /
 * 968-1018); the packet is only written on success. *pn_out / *poff on success. */
static int orc_recv_open(const mq_key_material* km, uint8_t* pkt, size_t len, size_t pn_off, int long_hdr,
                         uint64_t largest, uint64_t* pn_out, size_t* poff, int* phase_out) {
  if (pn_off + 4 + 16 > len) return MQ_ERR_CRYPTO;
  uint8_t mask[5], b0;
  size_t klen = suite_key_len(km->suite);
  if (!klen) return MQ_ERR_CRYPTO;
  orc_hp_mask(km->suite, km->hp, klen > 16 ? klen : 16, pkt + pn_off + 4, 16, mask);
  b0 = pkt[0] ^ (mask[0] & (long_hdr ? 0x0f : 0x1f));
  size_t pn_len = (size_t)(b0 & 3) + 1;
  uint32_t trunc = 0;
  for (size_t i = 0; i < pn_len; ++i) trunc = (trunc << 8) | (uint8_t)(pkt[pn_off + i] ^ mask[1 + i]);
  uint64_t pn = orc_decode_pn(trunc, pn_len, largest);
  if (pn > (1ull << 62) - 1) return MQ_ERR_PROTOCOL;
  if (phase_out) *phase_out = (b0 >> 2) & 1;
  *pn_out = pn;
  *poff = pn_off + pn_len;
  return MQ_OK;
}

static int orc_recv_aead(const mq_key_material* km, uint8_t* pkt, size_t len, size_t pn_off, int long_hdr,
                         uint64_t pn) {
  mq_pkt_desc d;
  memset(&d, 0, sizeof d);
  d.len = (uint32_t)len; d.pn = pn - 1; d.pn_offset = (uint16_t)pn_off;
  d.flags = long_hdr ? MQ_PKT_LONG_HEADER : 0;
  /* largest = pn - 1 decodes back to pn for any encoding; the composite redoes HP removal */
  uint64_t got;
  if (pn == 0) { d.pn = 0; }
  int rc = orc_unprotect_packet(km, pkt, &d, &got);
  return rc;
}

/* One datagram of the receive loop (recv.rs:189-265): its packets in order, records out[np..) (those
 * below max_pkts). upd0: the connection's key_updates at batch start. Returns the packets seen. */
static uint32_t orc_recv_dgram(const mq_key_material* rows, uint32_t n_rows, mq_conn_recv* c, uint8_t upd0,
                               uint8_t* arena, const mq_dgram* d, uint32_t g, mq_recv_pkt* out, uint32_t max_pkts,
                               uint32_t np) {
  const uint32_t np0 = np;
  uint8_t* base = arena + d->offset;
  size_t off = 0;
  while (off < d->len) {
    size_t plen = 0, pn_off = 0;
    uint64_t length = 0;
    int kind;
    if (orc_next_packet(base + off, d->len - off, &plen, &kind, &pn_off, &length)) break;
    uint8_t* pkt = base + off;
    off += plen;
    if (kind == 1 || kind == 3 || kind == 5) continue; /* 0-RTT, Retry, VN skipped (:221-226) */
    mq_recv_pkt r;
    memset(&r, 0, sizeof r);
    r.offset = (uint64_t)(pkt - arena); r.len = (uint32_t)plen; r.dgram = g;
    int st = MQ_OK, lvl = kind == 0 ? MQ_LEVEL_INITIAL : kind == 2 ? MQ_LEVEL_HANDSHAKE : MQ_LEVEL_APPLICATION;
    r.level = (uint8_t)lvl;
    uint64_t pn = 0;
    size_t poff = 0;
    if (lvl != MQ_LEVEL_APPLICATION) { /* recv_initial / recv_handshake -> decrypt_long_packet */
      uint32_t row = lvl == MQ_LEVEL_INITIAL ? c->initial_row : c->handshake_row;
      int has = c->flags & (lvl == MQ_LEVEL_INITIAL ? MQ_RECV_HAS_INITIAL : MQ_RECV_HAS_HANDSHAKE);
      size_t total = pn_off + (size_t)length;
      if (!has || row >= n_rows) st = MQ_ERR_CRYPTO;
      else if (total > 2048) st = MQ_ERR_BUFFER_TOO_SMALL; /* :963-965 */
      else st = orc_recv_open(&rows[row], pkt, total, pn_off, 1, c->largest_pn[lvl], &pn, &poff, NULL);
      if (st == MQ_OK) st = orc_recv_aead(&rows[row], pkt, total, pn_off, 1, pn);
      r.len = (uint32_t)total;
    } else { /* recv_short (:340-510) */
      size_t dl = c->dcid_len;
      int phase = 0;
      if (plen < 1 + dl) st = MQ_ERR_BUFFER_TOO_SMALL;                       /* parse_short_header */
      else if (!(c->flags & MQ_RECV_HAS_APP) || c->app_row[1] >= n_rows) st = MQ_ERR_CRYPTO;
      else if (plen > 2048) st = MQ_ERR_BUFFER_TOO_SMALL;                    /* :356-360 */
      else st = orc_recv_open(&rows[c->app_row[1]], pkt, plen, 1 + dl, 0, c->largest_pn[2], &pn, &poff, &phase);
      if (st == MQ_OK) {
        if (phase == c->key_phase) {
          st = orc_recv_aead(&rows[c->app_row[1]], pkt, plen, 1 + dl, 0, pn);
          r.key_gen = 1;
          if (st != MQ_OK) { /* :441-474: previous keys, else Error::Crypto */
            st = MQ_ERR_CRYPTO;
            if ((c->flags & MQ_RECV_HAS_PREV) && c->app_row[0] < n_rows) {
              st = orc_recv_aead(&rows[c->app_row[0]], pkt, plen, 1 + dl, 0, pn);
              r.key_gen = 0;
            }
          }
        } else { /* :476-509: next generation, rotate on success */
          /* no next-generation keys installed: Crypto (derive_next_recv_keys without a secret);
           * after a rotation inside this batch the next-next keys need the host: Deferred */
          st = c->key_updates != upd0 ? MQ_ERR_DEFERRED : MQ_ERR_CRYPTO;
          if ((c->flags & MQ_RECV_HAS_NEXT) && c->app_row[2] < n_rows) {
            st = orc_recv_aead(&rows[c->app_row[2]], pkt, plen, 1 + dl, 0, pn);
            r.key_gen = 2;
            if (st == MQ_OK) {
              c->app_row[0] = c->app_row[1]; c->app_row[1] = c->app_row[2];
              c->flags = (uint8_t)((c->flags | MQ_RECV_HAS_PREV) & ~MQ_RECV_HAS_NEXT);
              c->key_phase ^= 1; c->key_updates++;
            }
          }
        }
      }
    }
    if (st != MQ_OK) r.key_gen = 0; /* only meaningful for opened 1-RTT packets */
    if (st == MQ_OK) {
      r.pn = pn; r.payload_offset = (uint16_t)poff;
      if (pn > c->largest_pn[lvl]) c->largest_pn[lvl] = pn; /* :239-247 */
    }
    r.status = (uint8_t)st;
    if (np < max_pkts) out[np] = r;
    ++np;
  }
  return np - np0;
}

static int orc_dgram_ok(const mq_dgram* d, uint32_t n_conns, uint64_t arena_len) {
  return d->conn < n_conns && d->offset + (uint64_t)d->len <= arena_len;
}

void orc_batch_recv(const mq_key_material* rows, uint32_t n_rows, mq_conn_recv* conns, uint32_t n_conns,
                    uint8_t* arena, uint64_t arena_len, const mq_dgram* dg, uint32_t n_dgrams,
                    mq_recv_pkt* out, uint32_t max_pkts, uint32_t* n_pkts) {
  uint32_t np = 0;
  uint8_t* upd0 = (uint8_t*)malloc(n_conns ? n_conns : 1);
  for (uint32_t k = 0; k < n_conns; ++k) upd0[k] = conns[k].key_updates;
  for (uint32_t g = 0; g < n_dgrams; ++g) {
    if (!orc_dgram_ok(&dg[g], n_conns, arena_len)) continue;
    np += orc_recv_dgram(rows, n_rows, &conns[dg[g].conn], upd0[dg[g].conn], arena, &dg[g], g, out, max_pkts, np);
  }
  free(upd0);
  *n_pkts = np;
}

/* The same loop on `threads` threads: connections are independent (each one's state and packets
 * are its own; its datagrams keep their arrival order), so thread t takes the datagrams of the
 * connections c with c % threads == t. Each datagram's first record index comes from a sequential
 * pass that only parses (CoalescedPackets does not depend on decryption). Identical records,
 * connection table and arena as orc_batch_recv. */
typedef struct {
  const mq_key_material* rows; uint32_t n_rows; mq_conn_recv* conns; uint32_t n_conns; uint8_t* arena;
  uint64_t arena_len; const mq_dgram* dg; uint32_t n_dgrams; mq_recv_pkt* out; uint32_t max_pkts;
  const uint32_t* base; const uint8_t* upd0; int t, threads;
} orc_recv_job;

static void* orc_recv_run(void* arg) {
  orc_recv_job* j = (orc_recv_job*)arg;
  for (uint32_t g = 0; g < j->n_dgrams; ++g) {
    const mq_dgram* d = &j->dg[g];
    if (!orc_dgram_ok(d, j->n_conns, j->arena_len) || (int)(d->conn % (uint32_t)j->threads) != j->t) continue;
    (void)orc_recv_dgram(j->rows, j->n_rows, &j->conns[d->conn], j->upd0[d->conn], j->arena, d, g, j->out,
                         j->max_pkts, j->base[g]);
  }
  return NULL;
}

void orc_batch_recv_mt(const mq_key_material* rows, uint32_t n_rows, mq_conn_recv* conns, uint32_t n_conns,
                       uint8_t* arena, uint64_t arena_len, const mq_dgram* dg, uint32_t n_dgrams,
                       mq_recv_pkt* out, uint32_t max_pkts, uint32_t* n_pkts, int threads) {
  if (threads < 1) threads = 1;
  uint32_t* base = (uint32_t*)malloc(sizeof(uint32_t) * (n_dgrams ? n_dgrams : 1));
  uint8_t* upd0 = (uint8_t*)malloc(n_conns ? n_conns : 1);
  for (uint32_t k = 0; k < n_conns; ++k) upd0[k] = conns[k].key_updates;
  uint32_t np = 0;
  for (uint32_t g = 0; g < n_dgrams; ++g) {  /* parse-only pass: packets per datagram */
    base[g] = np;
    if (!orc_dgram_ok(&dg[g], n_conns, arena_len)) continue;
    const uint8_t* b = arena + dg[g].offset;
    size_t off = 0;
    while (off < dg[g].len) {
      size_t plen = 0, pn_off = 0;
      uint64_t length = 0;
      int kind;
      if (orc_next_packet(b + off, dg[g].len - off, &plen, &kind, &pn_off, &length)) break;
      off += plen;
      if (kind == 1 || kind == 3 || kind == 5) continue;
      ++np;
    }
  }
  orc_recv_job* jobs = (orc_recv_job*)calloc((size_t)threads, sizeof(orc_recv_job));
  pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
  for (int t = 0; t < threads; ++t) {
    orc_recv_job jb = {rows, n_rows, conns, n_conns, arena, arena_len, dg, n_dgrams, out, max_pkts, base, upd0, t,
                       threads};
    jobs[t] = jb;
  }
  if (threads == 1) orc_recv_run(&jobs[0]);
  else {
    for (int t = 0; t < threads; ++t) pthread_create(&th[t], NULL, orc_recv_run, &jobs[t]);
    for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
  }
  free(jobs); free(th); free(base); free(upd0);
  *n_pkts = np;
}

/* ---------------------------------------------------------------------------------------- */
typedef struct {
  const mq_key_material* rows; uint32_t n_rows; uint8_t* arena; uint64_t arena_len;
  const mq_pkt_desc* desc; uint8_t* status; uint64_t* pn_out; uint32_t suite_hint;
  uint32_t lo, hi; int open;
} orc_job;

static void* orc_run(void* arg) {
  orc_job* j = (orc_job*)arg;
  for (uint32_t i = j->lo; i < j->hi; ++i) {
    const mq_pkt_desc* d = &j->desc[i];
    int st;
    if (d->key_id >= j->n_rows || d->offset + (uint64_t)d->len > j->arena_len) {
      st = MQ_ERR_INVALID_ARG;
    } else {
      const mq_key_material* km = &j->rows[d->key_id];
      if (j->suite_hint != MQ_SUITE_MIXED && km->suite != j->suite_hint) st = MQ_ERR_SUITE;
      else if (j->open) st = orc_unprotect_packet(km, j->arena + d->offset, d, j->pn_out ? &j->pn_out[i] : NULL);
      else st = orc_protect_packet(km, j->arena + d->offset, d);
    }
    j->status[i] = (uint8_t)st;
  }
  return NULL;
}

static void orc_batch(const mq_key_material* rows, uint32_t n_rows, uint8_t* arena,
                      uint64_t arena_len, const mq_pkt_desc* desc, uint32_t n, uint8_t* status,
                      uint64_t* pn_out, uint32_t suite_hint, int threads, int open) {
  if (threads < 1) threads = 1;
  if ((uint32_t)threads > n) threads = n ? (int)n : 1;
  orc_job* jobs = (orc_job*)calloc((size_t)threads, sizeof(orc_job));
  pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
  for (int t = 0; t < threads; ++t) {
    orc_job j = {rows, n_rows, arena, arena_len, desc, status, pn_out, suite_hint,
                 (uint32_t)((uint64_t)n * t / threads), (uint32_t)((uint64_t)n * (t + 1) / threads), open};
    jobs[t] = j;
  }
  if (threads == 1) orc_run(&jobs[0]);
  else {
    for (int t = 0; t < threads; ++t) pthread_create(&th[t], NULL, orc_run, &jobs[t]);
    for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
  }
  free(jobs); free(th);
}

void orc_batch_seal(const mq_key_material* rows, uint32_t n_rows, uint8_t* arena,
                    uint64_t arena_len, const mq_pkt_desc* desc, uint32_t n, uint8_t* status,
                    uint32_t suite_hint, int threads) {
  orc_batch(rows, n_rows, arena, arena_len, desc, n, status, NULL, suite_hint, threads, 0);
}

void orc_batch_open(const mq_key_material* rows, uint32_t n_rows, uint8_t* arena,
                    uint64_t arena_len, const mq_pkt_desc* desc, uint32_t n, uint8_t* status,
                    uint64_t* pn_out, uint32_t suite_hint, int threads) {
  orc_batch(rows, n_rows, arena, arena_len, desc, n, status, pn_out, suite_hint, threads, 1);
}
