/* ossl_baseline.c — OpenSSL EVP leg of the CPU baseline (TEST / MEASUREMENT INFRASTRUCTURE ONLY).
 *
 * SURVEY §8d asks for the reference's own CPU path timed on the GPU box's host cores. The Rust
 * reference cannot be built there (no toolchain, crates not vendored), so bench.py times two
 * stand-ins on the same batch: the C restatement (mq_oracle.c, scalar, "port") and this file —
 * OpenSSL 3 EVP (ChaCha20-Poly1305 / AES-128-GCM with its AVX2/AVX-512/AES-NI/CLMUL code paths),
 * the like-for-like stand-in for the cpufeatures-selected backends of chacha20poly1305 0.10.1 /
 * aes-gcm 0.10.3. libcrypto.so.3 is dlopen'ed at run time, so nothing links against it and a box
 * without it reports "skipped". Only bench.py's cpu_baseline leg calls this; the product never does.
 *
 * Per packet it runs the same composites as the product's batch API:
 *   seal (transmit.rs:584-599 / 714-729): nonce = iv ^ BE64(pn) (crypto/mod.rs:66-74), AEAD seal
 *        of the payload with AAD = header || PN, tag appended, then the header-protection mask
 *        from the sample at pn_offset + 4 (rustcrypto.rs:175-220) applied to byte 0 and the PN;
 *   open (recv.rs:363-421): mask, unmask byte 0 and the PN, decode_pn (number.rs:52-70), AEAD open.
 * Every packet's status is MQ_OK or MQ_ERR_CRYPTO; bench.py checks the results against the GPU's.
 */
#include <dlfcn.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/mq_aead.h"

typedef struct evp_cipher_ctx_st EVP_CIPHER_CTX;
typedef struct evp_cipher_st EVP_CIPHER;

static struct {
  int ok;
  EVP_CIPHER_CTX* (*ctx_new)(void);
  void (*ctx_free)(EVP_CIPHER_CTX*);
  EVP_CIPHER* (*fetch)(void*, const char*, const char*);
  void* (*libctx_new)(void);
  void (*libctx_free)(void*);
  int (*enc_init)(EVP_CIPHER_CTX*, const EVP_CIPHER*, void*, const uint8_t*, const uint8_t*);
  int (*enc_update)(EVP_CIPHER_CTX*, uint8_t*, int*, const uint8_t*, int);
  int (*enc_final)(EVP_CIPHER_CTX*, uint8_t*, int*);
  int (*dec_init)(EVP_CIPHER_CTX*, const EVP_CIPHER*, void*, const uint8_t*, const uint8_t*);
  int (*dec_update)(EVP_CIPHER_CTX*, uint8_t*, int*, const uint8_t*, int);
  int (*dec_final)(EVP_CIPHER_CTX*, uint8_t*, int*);
  int (*ctrl)(EVP_CIPHER_CTX*, int, int, void*);
  void (*cipher_free)(EVP_CIPHER*);
} E;

enum { CTRL_SET_IVLEN = 0x9, CTRL_GET_TAG = 0x10, CTRL_SET_TAG = 0x11 };

static pthread_once_t g_once = PTHREAD_ONCE_INIT;

static void load_libcrypto(void) {
  void* h = dlopen("libcrypto.so.3", RTLD_NOW | RTLD_LOCAL);
  if (!h) return;
#define SYM(f, n) *(void**)(&E.f) = dlsym(h, n); if (!E.f) return;
  SYM(ctx_new, "EVP_CIPHER_CTX_new") SYM(ctx_free, "EVP_CIPHER_CTX_free")
  SYM(fetch, "EVP_CIPHER_fetch") SYM(libctx_new, "OSSL_LIB_CTX_new") SYM(libctx_free, "OSSL_LIB_CTX_free")
  SYM(enc_init, "EVP_EncryptInit_ex") SYM(enc_update, "EVP_EncryptUpdate") SYM(enc_final, "EVP_EncryptFinal_ex")
  SYM(dec_init, "EVP_DecryptInit_ex") SYM(dec_update, "EVP_DecryptUpdate") SYM(dec_final, "EVP_DecryptFinal_ex")
  SYM(ctrl, "EVP_CIPHER_CTX_ctrl")
  SYM(cipher_free, "EVP_CIPHER_free")
#undef SYM
  EVP_CIPHER* c = E.fetch(NULL, "ChaCha20-Poly1305", NULL);
  if (!c) return;
  E.cipher_free(c);
  E.ok = 1;
}

/* Explicitly fetched ciphers, one set per thread, each from the thread's own library context
 * (OSSL_LIB_CTX_new): the legacy EVP_chacha20_poly1305() objects re-fetch from the provider
 * (under a global lock) on every init, and in OpenSSL 3.0 every EVP_*Init_ex — including the
 * per-packet re-IV — serialises on state of the library context its cipher came from. Measured on
 * the GPU box's host (tools/ossl_scaling.c, profiles/r02_ossl_scaling.txt): re-IV calls 21.3 M/s
 * on 1 thread, 21.7 M/s on 16 with the default context; 21.0 M/s PER THREAD on 16 and 19.4 M/s
 * per thread on 64 with one context per thread. */
static const char* const kCipherNames[4] = {"ChaCha20-Poly1305", "ChaCha20", "AES-128-GCM", "AES-128-ECB"};

int ossl_available(void) {
  pthread_once(&g_once, load_libcrypto);
  return E.ok;
}

/* decode_pn, reference src/packet/number.rs:52-70 */
static uint64_t decode_pn(uint32_t truncated, uint32_t pn_len, uint64_t largest) {
  const uint64_t win = 1ull << (8 * pn_len), hwin = win >> 1, mask = win - 1, expected = largest + 1;
  const uint64_t cand = (expected & ~mask) | truncated;
  if (cand + hwin <= expected && cand + win <= (1ull << 62)) return cand + win;
  if (cand > expected + hwin && cand >= win) return cand - win;
  return cand;
}

typedef struct {
  EVP_CIPHER_CTX *aead_e, *aead_d, *hp;  /* keyed once per key row, then re-IV'ed per packet */
  uint32_t suite, row;
} Ctx;

static void set_row(Ctx* c, const mq_key_material* rows, uint32_t row) {
  if (c->row == row) return;
  const mq_key_material* k = rows + row;
  E.enc_init(c->aead_e, NULL, NULL, k->key, NULL);
  E.dec_init(c->aead_d, NULL, NULL, k->key, NULL);
  E.enc_init(c->hp, NULL, NULL, k->hp, NULL);
  c->row = row;
}

static void hp_mask(Ctx* c, const uint8_t* sample, uint8_t mask[5]) {
  uint8_t out[32];
  int l = 0;
  if (c->suite == MQ_SUITE_CHACHA20) {  /* EVP ChaCha20 IV = counter (LE32) || nonce: the sample */
    static const uint8_t zero[5];
    E.enc_init(c->hp, NULL, NULL, NULL, sample);
    E.enc_update(c->hp, mask, &l, zero, 5);
  } else {
    E.enc_update(c->hp, out, &l, sample, 16);
    memcpy(mask, out, 5);
  }
}

static int one(Ctx* c, const mq_key_material* rows, uint8_t* arena, const mq_pkt_desc* d, int open) {
  const mq_key_material* k = rows + d->key_id;
  set_row(c, rows, d->key_id);
  uint8_t* pkt = arena + d->offset;
  const uint8_t fb = (d->flags & MQ_PKT_LONG_HEADER) ? 0x0f : 0x1f;
  uint8_t mask[5], nonce[12];
  uint32_t pn_len = d->pn_len;
  uint64_t pn = d->pn;
  int l = 0;
  if (open) {
    hp_mask(c, pkt + d->pn_offset + 4, mask);
    pkt[0] ^= mask[0] & fb;
    pn_len = (pkt[0] & 3u) + 1;
    uint32_t t = 0;
    for (uint32_t b = 0; b < pn_len; ++b) {
      pkt[d->pn_offset + b] ^= mask[1 + b];
      t = (t << 8) | pkt[d->pn_offset + b];
    }
    pn = decode_pn(t, pn_len, d->pn);
  }
  memcpy(nonce, k->iv, 12);
  for (int b = 0; b < 8; ++b) nonce[4 + b] ^= (uint8_t)(pn >> (56 - 8 * b));
  const int aad = (int)(d->pn_offset + pn_len), P = (int)d->len - aad - 16;
  uint8_t* pay = pkt + aad;
  if (!open) {
    E.enc_init(c->aead_e, NULL, NULL, NULL, nonce);
    E.enc_update(c->aead_e, NULL, &l, pkt, aad);
    E.enc_update(c->aead_e, pay, &l, pay, P);
    E.enc_final(c->aead_e, pay + P, &l);
    E.ctrl(c->aead_e, CTRL_GET_TAG, 16, pay + P);
    hp_mask(c, pkt + d->pn_offset + 4, mask);
    pkt[0] ^= mask[0] & fb;
    for (uint32_t b = 0; b < pn_len; ++b) pkt[d->pn_offset + b] ^= mask[1 + b];
    return MQ_OK;
  }
  E.dec_init(c->aead_d, NULL, NULL, NULL, nonce);
  E.dec_update(c->aead_d, NULL, &l, pkt, aad);
  E.dec_update(c->aead_d, pay, &l, pay, P);
  E.ctrl(c->aead_d, CTRL_SET_TAG, 16, pay + P);
  return E.dec_final(c->aead_d, pay + P, &l) > 0 ? MQ_OK : MQ_ERR_CRYPTO;
}

typedef struct {
  const mq_key_material* rows;
  uint8_t* arena;
  const mq_pkt_desc* desc;
  uint8_t* status;
  uint32_t lo, hi;
  int open;
} Job;

static void* worker(void* p) {
  Job* j = (Job*)p;
  Ctx c[2];
  const uint32_t suites[2] = {MQ_SUITE_CHACHA20, MQ_SUITE_AES128GCM};
  EVP_CIPHER* ciph[4];
  void* lc = E.libctx_new();  /* NULL on failure: the default context (still correct, slower) */
  for (int i = 0; i < 4; ++i) ciph[i] = E.fetch(lc, kCipherNames[i], NULL);
  for (int s = 0; s < 2; ++s) {
    c[s].suite = suites[s];
    c[s].row = 0xffffffffu;
    c[s].aead_e = E.ctx_new();
    c[s].aead_d = E.ctx_new();
    c[s].hp = E.ctx_new();
    E.enc_init(c[s].aead_e, ciph[2 * s], NULL, NULL, NULL);
    E.dec_init(c[s].aead_d, ciph[2 * s], NULL, NULL, NULL);
    E.enc_init(c[s].hp, ciph[2 * s + 1], NULL, NULL, NULL);
  }
  for (uint32_t i = j->lo; i < j->hi; ++i) {
    const mq_pkt_desc* d = j->desc + i;
    Ctx* cx = j->rows[d->key_id].suite == MQ_SUITE_CHACHA20 ? &c[0] : &c[1];
    j->status[i] = (uint8_t)one(cx, j->rows, j->arena, d, j->open);
  }
  for (int s = 0; s < 2; ++s) { E.ctx_free(c[s].aead_e); E.ctx_free(c[s].aead_d); E.ctx_free(c[s].hp); }
  for (int i = 0; i < 4; ++i) E.cipher_free(ciph[i]);
  if (lc) E.libctx_free(lc);
  return NULL;
}

/* Seal (open = 0) or open (open = 1) n packets in place with `threads` threads over contiguous
 * ranges. Descriptors must be valid (the bench's own workload). Returns 0, or -1 when
 * libcrypto.so.3 cannot be loaded. */
int ossl_batch(const mq_key_material* rows, uint32_t n_rows, uint8_t* arena, uint64_t arena_len,
               const mq_pkt_desc* desc, uint32_t n, uint8_t* status, int threads, int open) {
  (void)n_rows; (void)arena_len;
  if (!ossl_available()) return -1;
  if (threads < 1) threads = 1;
  Job* jobs = (Job*)calloc((size_t)threads, sizeof(Job));
  pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
  for (int t = 0; t < threads; ++t) {
    jobs[t] = (Job){rows, arena, desc, status, (uint32_t)((uint64_t)n * t / threads),
                    (uint32_t)((uint64_t)n * (t + 1) / threads), open};
    pthread_create(&th[t], NULL, worker, &jobs[t]);
  }
  for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
  free(jobs);
  free(th);
  return 0;
}
