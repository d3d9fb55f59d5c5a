/*
 * gen_golden.c — generates the committed golden vectors under tests/golden/ with OpenSSL
 * (libcrypto 3.x EVP), an implementation independent of both the product kernels and the
 * CPU oracle. Run here only (the GPU box receives the JSON files, not this program):
 *
 *   gcc -O2 -o /tmp/gen_golden tests/golden/gen_golden.c -lcrypto && /tmp/gen_golden tests/golden
 *
 * Outputs:
 *   aead_vectors.json    Aead::seal_in_place results (ciphertext||tag) for both suites over
 *                        edge-case lengths (0,1,15,16,17,63,64,65,...,1171,1350) and AAD lengths
 *   hp_vectors.json      HeaderProtection::mask results, incl. all-zero / all-0xff samples and
 *                        the ChaCha counter 0xffffffff case (SURVEY §8c divergence note)
 *   packet_vectors.json  full QUIC packets before/after protection (RFC 9001 §5: seal, sample,
 *                        mask byte 0 with 0x0f/0x1f, mask PN) for short and long headers,
 *                        pn_len 1..4, both suites, plus the decoded PN for the receive side
 * Deterministic: SplitMix64 seeded with 0x6D696C6C69717569 ("milliqui").
 */
#include <openssl/evp.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t g_rng = 0x6D696C6C69717569ull;
static uint64_t splitmix(void) {
  uint64_t z = (g_rng += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static void rnd(uint8_t* p, size_t n) { for (size_t i = 0; i < n; ++i) p[i] = (uint8_t)splitmix(); }
static uint32_t rndu(uint32_t lo, uint32_t hi) { return lo + (uint32_t)(splitmix() % (hi - lo + 1)); }

static void die(const char* m) { fprintf(stderr, "gen_golden: %s\n", m); exit(1); }

static void hex(FILE* f, const uint8_t* p, size_t n) {
  fputc('"', f);
  for (size_t i = 0; i < n; ++i) fprintf(f, "%02x", p[i]);
  fputc('"', f);
}

/* ---- OpenSSL primitives ---------------------------------------------------------------- */
static void aead_seal(int suite, const uint8_t* key, const uint8_t* nonce, const uint8_t* aad,
                      size_t aad_len, const uint8_t* pt, size_t pt_len, uint8_t* out) {
  EVP_CIPHER_CTX* c = EVP_CIPHER_CTX_new();
  const EVP_CIPHER* ci = suite == 1 ? EVP_aes_128_gcm() : EVP_chacha20_poly1305();
  int n;
  if (!EVP_EncryptInit_ex(c, ci, NULL, NULL, NULL)) die("init");
  if (!EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_AEAD_SET_IVLEN, 12, NULL)) die("ivlen");
  if (!EVP_EncryptInit_ex(c, NULL, NULL, key, nonce)) die("key");
  if (aad_len && !EVP_EncryptUpdate(c, NULL, &n, aad, (int)aad_len)) die("aad");
  if (pt_len && !EVP_EncryptUpdate(c, out, &n, pt, (int)pt_len)) die("pt");
  if (!EVP_EncryptFinal_ex(c, out + pt_len, &n)) die("final");
  if (!EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_AEAD_GET_TAG, 16, out + pt_len)) die("tag");
  EVP_CIPHER_CTX_free(c);
}

static int aead_open(int suite, const uint8_t* key, const uint8_t* nonce, const uint8_t* aad,
                     size_t aad_len, const uint8_t* ct, size_t ct_len, uint8_t* out) {
  EVP_CIPHER_CTX* c = EVP_CIPHER_CTX_new();
  const EVP_CIPHER* ci = suite == 1 ? EVP_aes_128_gcm() : EVP_chacha20_poly1305();
  int n, ok;
  size_t pt_len = ct_len - 16;
  EVP_DecryptInit_ex(c, ci, NULL, NULL, NULL);
  EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_AEAD_SET_IVLEN, 12, NULL);
  EVP_DecryptInit_ex(c, NULL, NULL, key, nonce);
  if (aad_len) EVP_DecryptUpdate(c, NULL, &n, aad, (int)aad_len);
  if (pt_len) EVP_DecryptUpdate(c, out, &n, ct, (int)pt_len);
  EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_AEAD_SET_TAG, 16, (void*)(ct + pt_len));
  ok = EVP_DecryptFinal_ex(c, out + pt_len, &n);
  EVP_CIPHER_CTX_free(c);
  return ok == 1;
}

static void hp_mask(int suite, const uint8_t* hp, const uint8_t* sample, uint8_t mask[5]) {
  EVP_CIPHER_CTX* c = EVP_CIPHER_CTX_new();
  int n;
  uint8_t out[16] = {0}, zero[16] = {0};
  if (suite == 1) {
    EVP_EncryptInit_ex(c, EVP_aes_128_ecb(), NULL, hp, NULL);
    EVP_CIPHER_CTX_set_padding(c, 0);
    EVP_EncryptUpdate(c, out, &n, sample, 16);
  } else {
    /* OpenSSL's EVP_chacha20 IV = 32-bit LE counter || 96-bit nonce = the 16-byte sample */
    EVP_EncryptInit_ex(c, EVP_chacha20(), NULL, hp, sample);
    EVP_EncryptUpdate(c, out, &n, zero, 5);
  }
  memcpy(mask, out, 5);
  EVP_CIPHER_CTX_free(c);
}

static void nonce_of(const uint8_t iv[12], uint64_t pn, uint8_t nonce[12]) {
  memcpy(nonce, iv, 12);
  for (int i = 0; i < 8; ++i) nonce[4 + i] ^= (uint8_t)(pn >> (56 - 8 * i));
}

/* ---- aead_vectors.json --------------------------------------------------------------------- */
static void gen_aead(const char* dir) {
  char path[512];
  snprintf(path, sizeof path, "%s/aead_vectors.json", dir);
  FILE* f = fopen(path, "w");
  if (!f) die("open aead");
  static const size_t lens[] = {0, 1, 2, 3, 4, 5, 7, 11, 12, 13, 15, 16, 17, 31, 32, 33, 47, 48,
                                49, 63, 64, 65, 100, 127, 128, 129, 191, 192, 193, 255, 256,
                                257, 300, 511, 512, 513, 1000, 1024, 1171, 1200, 1350};
  static const size_t aads[] = {0, 1, 13, 15, 16, 17, 21, 30, 52, 63};
  fprintf(f, "{\"generator\": \"tests/golden/gen_golden.c (OpenSSL %s)\",\n \"cases\": [\n",
          OPENSSL_VERSION_TEXT);
  int first = 1;
  for (int suite = 1; suite <= 2; ++suite) {
    for (size_t li = 0; li < sizeof lens / sizeof *lens; ++li) {
      uint8_t key[32], nonce[12], aad[64], pt[1400], out[1416];
      size_t pl = lens[li], al = aads[(li + suite) % (sizeof aads / sizeof *aads)];
      rnd(key, 32); rnd(nonce, 12); rnd(aad, al); rnd(pt, pl);
      if (li == 0) memset(pt, 0, pl);
      if (li == 1) memset(pt, 0xff, pl);
      aead_seal(suite, key, nonce, aad, al, pt, pl, out);
      fprintf(f, "%s  {\"suite\": %d, \"key\": ", first ? "" : ",\n", suite);
      hex(f, key, suite == 1 ? 16 : 32);
      fprintf(f, ", \"nonce\": "); hex(f, nonce, 12);
      fprintf(f, ", \"aad\": "); hex(f, aad, al);
      fprintf(f, ", \"pt\": "); hex(f, pt, pl);
      fprintf(f, ", \"ct_tag\": "); hex(f, out, pl + 16);
      fprintf(f, "}");
      first = 0;
    }
  }
  /* RFC 8439 §2.8.2 test vector (AEAD_CHACHA20_POLY1305) re-derived through OpenSSL */
  {
    const char* pts = "Ladies and Gentlemen of the class of '99: If I could offer you only one "
                      "tip for the future, sunscreen would be it.";
    uint8_t key[32], nonce[12] = {0x07, 0, 0, 0, 0x40, 0x41, 0x42, 0x43, 0x44, 0x45, 0x46, 0x47};
    uint8_t aad[12] = {0x50, 0x51, 0x52, 0x53, 0xc0, 0xc1, 0xc2, 0xc3, 0xc4, 0xc5, 0xc6, 0xc7};
    uint8_t out[200];
    for (int i = 0; i < 32; ++i) key[i] = (uint8_t)(0x80 + i);
    size_t pl = strlen(pts);
    aead_seal(2, key, nonce, aad, 12, (const uint8_t*)pts, pl, out);
    fprintf(f, ",\n  {\"suite\": 2, \"name\": \"rfc8439-2.8.2\", \"key\": "); hex(f, key, 32);
    fprintf(f, ", \"nonce\": "); hex(f, nonce, 12);
    fprintf(f, ", \"aad\": "); hex(f, aad, 12);
    fprintf(f, ", \"pt\": "); hex(f, (const uint8_t*)pts, pl);
    fprintf(f, ", \"ct_tag\": "); hex(f, out, pl + 16);
    fprintf(f, "}");
  }
  fprintf(f, "\n]}\n");
  fclose(f);
}

/* ---- hp_vectors.json ----------------------------------------------------------------------- */
static void gen_hp(const char* dir) {
  char path[512];
  snprintf(path, sizeof path, "%s/hp_vectors.json", dir);
  FILE* f = fopen(path, "w");
  if (!f) die("open hp");
  fprintf(f, "{\"generator\": \"tests/golden/gen_golden.c (OpenSSL %s)\",\n \"cases\": [\n",
          OPENSSL_VERSION_TEXT);
  int first = 1;
  for (int suite = 1; suite <= 2; ++suite) {
    for (int i = 0; i < 24; ++i) {
      uint8_t hp[32], sample[16], mask[5];
      rnd(hp, 32); rnd(sample, 16);
      if (i == 0) memset(sample, 0, 16);
      if (i == 1) memset(sample, 0xff, 16);
      if (i == 2) memset(sample, 0xff, 4);               /* ChaCha counter = 0xffffffff */
      if (i == 3) { memset(sample, 0, 4); }              /* counter = 0 */
      hp_mask(suite, hp, sample, mask);
      fprintf(f, "%s  {\"suite\": %d, \"hp\": ", first ? "" : ",\n", suite);
      hex(f, hp, suite == 1 ? 16 : 32);
      fprintf(f, ", \"sample\": "); hex(f, sample, 16);
      fprintf(f, ", \"mask\": "); hex(f, mask, 5);
      fprintf(f, "}");
      first = 0;
    }
  }
  fprintf(f, "\n]}\n");
  fclose(f);
}

/* ---- packet_vectors.json ------------------------------------------------------------------- */
/* RFC 9001 §5.3-5.4 protection of one packet: AAD = header||PN, seal payload, sample at
 * pn_offset+4, byte0 ^= mask[0] & (long ? 0x0f : 0x1f), PN ^= mask[1..]. */
static void protect(int suite, const uint8_t* key, const uint8_t* iv, const uint8_t* hp,
                    uint8_t* pkt, size_t pn_offset, size_t pn_len, uint64_t pn, int long_hdr,
                    size_t payload_len) {
  uint8_t nonce[12], mask[5], *tmp = malloc(payload_len + 16);
  size_t hdr = pn_offset + pn_len;
  nonce_of(iv, pn, nonce);
  aead_seal(suite, key, nonce, pkt, hdr, pkt + hdr, payload_len, tmp);
  memcpy(pkt + hdr, tmp, payload_len + 16);
  hp_mask(suite, hp, pkt + pn_offset + 4, mask);
  pkt[0] ^= mask[0] & (long_hdr ? 0x0f : 0x1f);
  for (size_t i = 0; i < pn_len; ++i) pkt[pn_offset + i] ^= mask[1 + i];
  free(tmp);
}

static void emit_packet(FILE* f, int* first, const char* name, int suite, const uint8_t* key,
                        const uint8_t* iv, const uint8_t* hp, const uint8_t* plain, size_t len,
                        size_t pn_offset, size_t pn_len, uint64_t pn, uint64_t largest_pn,
                        int long_hdr, const uint8_t* prot) {
  fprintf(f, "%s  {\"name\": \"%s\", \"suite\": %d, \"key\": ", *first ? "" : ",\n", name, suite);
  hex(f, key, suite == 1 ? 16 : 32);
  fprintf(f, ", \"iv\": "); hex(f, iv, 12);
  fprintf(f, ", \"hp\": "); hex(f, hp, suite == 1 ? 16 : 32);
  fprintf(f, ", \"pn_offset\": %zu, \"pn_len\": %zu, \"pn\": %llu, \"largest_pn\": %llu, "
             "\"long_header\": %s, \"len\": %zu,\n   \"unprotected\": ",
          pn_offset, pn_len, (unsigned long long)pn, (unsigned long long)largest_pn,
          long_hdr ? "true" : "false", len);
  hex(f, plain, len);
  fprintf(f, ",\n   \"protected\": "); hex(f, prot, len);
  fprintf(f, "}");
  *first = 0;
}

static size_t unhex(const char* s, uint8_t* out) {
  size_t n = 0;
  for (; s[0] && s[1]; s += 2) { unsigned v; sscanf(s, "%2x", &v); out[n++] = (uint8_t)v; }
  return n;
}

static void gen_packets(const char* dir) {
  char path[512];
  snprintf(path, sizeof path, "%s/packet_vectors.json", dir);
  FILE* f = fopen(path, "w");
  if (!f) die("open packets");
  fprintf(f, "{\"generator\": \"tests/golden/gen_golden.c (OpenSSL %s)\",\n \"packets\": [\n",
          OPENSSL_VERSION_TEXT);
  int first = 1;
  uint8_t plain[2048], prot[2048];
  /* random short-header (1-RTT) and long-header (Initial-shaped) packets */
  for (int i = 0; i < 96; ++i) {
    int suite = (i % 3 == 0) ? 2 : 1;
    if (i % 2) suite = 2;
    int long_hdr = (i % 4 == 3);
    uint8_t key[32], iv[12], hp[32];
    rnd(key, 32); rnd(iv, 12); rnd(hp, 32);
    size_t pn_len = 1 + (i % 4);
    uint64_t largest = splitmix() & ((1ull << 40) - 1);
    uint64_t pn = largest + 1 + (splitmix() % (1ull << (8 * pn_len - 2)));
    size_t pn_offset, len;
    size_t target = (i < 8) ? (size_t)(20 + i) : (i < 16 ? 1200 : rndu(64, 1350));
    if (long_hdr) {
      /* Initial: 0xc0|pn_len-1, version 1, DCID 8, SCID 8, token len 0, Length varint(2) */
      size_t pos = 0;
      plain[pos++] = (uint8_t)(0xc0 | (pn_len - 1));
      plain[pos++] = 0; plain[pos++] = 0; plain[pos++] = 0; plain[pos++] = 1;
      plain[pos++] = 8; rnd(plain + pos, 8); pos += 8;
      plain[pos++] = 8; rnd(plain + pos, 8); pos += 8;
      plain[pos++] = 0;
      if (target < pos + 2 + pn_len + 20) target = pos + 2 + pn_len + 20;
      size_t length_field = target - pos - 2;  /* PN + payload + tag */
      plain[pos++] = (uint8_t)(0x40 | (length_field >> 8)); plain[pos++] = (uint8_t)length_field;
      pn_offset = pos;
      len = target;
    } else {
      size_t dcid = (i % 5 == 0) ? 0 : (i % 5 == 1 ? 20 : 8);
      plain[0] = (uint8_t)(0x40 | ((i & 8) ? 0x04 : 0) | (pn_len - 1));
      rnd(plain + 1, dcid);
      pn_offset = 1 + dcid;
      if (target < pn_offset + pn_len + 16 + 4) target = pn_offset + 4 + 16;
      if (target < pn_offset + pn_len + 16) target = pn_offset + pn_len + 16;
      len = target;
    }
    for (size_t k = 0; k < pn_len; ++k) plain[pn_offset + k] = (uint8_t)(pn >> (8 * (pn_len - 1 - k)));
    size_t payload_len = len - pn_offset - pn_len - 16;
    rnd(plain + pn_offset + pn_len, payload_len);
    if (i == 8) memset(plain + pn_offset + pn_len, 0, payload_len);
    if (i == 9) memset(plain + pn_offset + pn_len, 0xff, payload_len);
    memset(plain + len - 16, 0, 16);  /* tag room */
    memcpy(prot, plain, len);
    protect(suite, key, iv, hp, prot, pn_offset, pn_len, pn, long_hdr, payload_len);
    /* receive side check with OpenSSL: it must open */
    {
      uint8_t nonce[12], tmp[2048];
      size_t hdr = pn_offset + pn_len;
      nonce_of(iv, pn, nonce);
      if (!aead_open(suite, key, nonce, plain, hdr, prot + hdr, len - hdr, tmp)) die("reopen");
    }
    char name[32];
    snprintf(name, sizeof name, "rand-%02d", i);
    emit_packet(f, &first, name, suite, key, iv, hp, plain, len, pn_offset, pn_len, pn, largest,
                long_hdr, prot);
  }
  /* RFC 9001 A.2 client Initial (keys from A.1; values: reference rfc/rfc9001.txt:2357-2458) */
  {
    uint8_t key[16], iv[12], hp[16];
    unhex("1f369613dd76d5467730efcbe3b1a22d", key);
    unhex("fa044b2f42a3fd3b46fb255c", iv);
    unhex("9f50449e04a0e810283a1e9933adedd2", hp);
    size_t h = unhex("c300000001088394c8f03e5157080000449e00000002", plain);
    const char* crypto =
        "060040f1010000ed0303ebf8fa56f12939b9584a3896472ec40bb863cfd3e86804fe3a47f06a2b69484c"
        "00000413011302010000c000000010000e00000b6578616d706c652e636f6dff01000100000a00080006"
        "001d0017001800100007000504616c706e000500050100000000003300260024001d00209370b2c9caa4"
        "7fbabaf4559fedba753de171fa71f50f1ce15d43e994ec74d748002b0003020304000d0010000e040305"
        "0306030203080408050806002d00020101001c00024001003900320408ffffffffffffffff05048000ff"
        "ff07048000ffff0801100104800075300901100f088394c8f03e51570806048000ffff";
    size_t c = unhex(crypto, plain + h);
    memset(plain + h + c, 0, 1162 - c);
    size_t len = h + 1162 + 16;
    memset(plain + h + 1162, 0, 16);
    memcpy(prot, plain, len);
    protect(1, key, iv, hp, prot, 18, 4, 2, 1, 1162);
    emit_packet(f, &first, "rfc9001-A.2", 1, key, iv, hp, plain, len, 18, 4, 2, 0, 1, prot);
  }
  /* RFC 9001 A.3 server Initial (rfc9001.txt:2461-2488) */
  {
    uint8_t key[16], iv[12], hp[16];
    unhex("cf3a5331653c364c88f0f379b6067e37", key);
    unhex("0ac1493ca1905853b0bba03e", iv);
    unhex("c206b8d9b9f0f37644430b490eeaa314", hp);
    size_t h = unhex("c1000000010008f067a5502a4262b50040750001", plain);
    size_t c = unhex("02000000000600405a020000560303eefce7f7b37ba1d1632e96677825ddf73988cfc79825"
                     "df566dc5430b9a045a1200130100002e00330024001d00209d3c940d89690b84d08a60993c"
                     "144eca684d1081287c834d5311bcf32bb9da1a002b00020304", plain + h);
    size_t len = h + c + 16;
    memset(plain + h + c, 0, 16);
    memcpy(prot, plain, len);
    protect(1, key, iv, hp, prot, 18, 2, 1, 1, c);
    emit_packet(f, &first, "rfc9001-A.3", 1, key, iv, hp, plain, len, 18, 2, 1, 0, 1, prot);
  }
  /* RFC 9001 A.5 ChaCha20-Poly1305 short header (rfc9001.txt:2496-2553) */
  {
    uint8_t key[32], iv[12], hp[32];
    unhex("c6d98ff3441c3fe1b2182094f69caa2ed4b716b65488960a7a984979fb23e1c8", key);
    unhex("e0459b3474bdd0e44a41c144", iv);
    unhex("25a282b9e82f06f21f488917a4fc8f1b73573685608597d0efcb076b0ab7a7a4", hp);
    size_t h = unhex("4200bff4", plain);
    plain[h] = 0x01;
    memset(plain + h + 1, 0, 16);
    size_t len = h + 1 + 16;
    memcpy(prot, plain, len);
    protect(2, key, iv, hp, prot, 1, 3, 654360564ull, 0, 1);
    /* largest_pn chosen so that decode_pn recovers 654360564 from the 3-byte encoding */
    emit_packet(f, &first, "rfc9001-A.5", 2, key, iv, hp, plain, len, 1, 3, 654360564ull,
                654360563ull, 0, prot);
  }
  fprintf(f, "\n]}\n");
  fclose(f);
}

int main(int argc, char** argv) {
  const char* dir = argc > 1 ? argv[1] : ".";
  gen_aead(dir);
  gen_hp(dir);
  gen_packets(dir);
  return 0;
}
