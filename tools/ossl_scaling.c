/* ossl_scaling.c — why the OpenSSL leg of bench.py's CPU baseline stops scaling.
 * MEASUREMENT TOOL ONLY (links libcrypto; never part of the product).
 *
 * Per packet the OpenSSL composite (oracle/ossl_baseline.c) re-initialises two EVP contexts with a
 * new IV: the AEAD (nonce = iv ^ pn) and the ChaCha20 header-protection block (IV = sample). This
 * program times, on 1..T threads with one pre-keyed context per thread and explicitly fetched
 * ciphers (per-thread, and optionally from a per-thread OSSL_LIB_CTX):
 *   mode 1: full ChaCha20-Poly1305 seal of a 1171-B payload with 13-B AAD (re-IV + update + final)
 *   mode 2: the HP mask alone (re-IV + 5-byte update)
 *   mode 4: the re-IV call alone (EVP_EncryptInit_ex(ctx, NULL, NULL, NULL, iv))
 * and prints kpackets/s per thread count. Build: gcc -O2 -o ossl_scaling ossl_scaling.c -lcrypto -lpthread
 * Usage: ./ossl_scaling MODE PERCTX MAXTHREADS */
#include <openssl/crypto.h>
#include <openssl/evp.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

static int MODE, PERCTX, NPKT = 100000;
static pthread_barrier_t bar;
static double tstart[1024], tend[1024];

static double now(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + t.tv_nsec * 1e-9;
}

static void* work(void* arg) {
  const int id = (int)(long)arg;
  OSSL_LIB_CTX* lc = PERCTX ? OSSL_LIB_CTX_new() : NULL;
  EVP_CIPHER* c = EVP_CIPHER_fetch(lc, "ChaCha20-Poly1305", NULL);
  EVP_CIPHER* h = EVP_CIPHER_fetch(lc, "ChaCha20", NULL);
  EVP_CIPHER_CTX* x = EVP_CIPHER_CTX_new();
  EVP_CIPHER_CTX* y = EVP_CIPHER_CTX_new();
  unsigned char key[32] = {1}, iv[16] = {2}, buf[1300], tag[16];
  int l;
  EVP_EncryptInit_ex(x, c, NULL, key, iv);
  EVP_EncryptInit_ex(y, h, NULL, key, iv);
  memset(buf, 3, sizeof buf);
  pthread_barrier_wait(&bar);
  tstart[id] = now();
  for (int i = 0; i < NPKT; i++) {
    iv[0] = (unsigned char)i;
    iv[1] = (unsigned char)(i >> 8);
    if (MODE & 1) {
      EVP_EncryptInit_ex(x, NULL, NULL, NULL, iv);
      EVP_EncryptUpdate(x, NULL, &l, buf, 13);
      EVP_EncryptUpdate(x, buf + 13, &l, buf + 13, 1171);
      EVP_EncryptFinal_ex(x, tag, &l);
      EVP_CIPHER_CTX_ctrl(x, 0x10, 16, tag);
    }
    if (MODE & 2) {
      EVP_EncryptInit_ex(y, NULL, NULL, NULL, iv);
      EVP_EncryptUpdate(y, tag, &l, buf, 5);
    }
    if (MODE & 4) EVP_EncryptInit_ex(x, NULL, NULL, NULL, iv);
  }
  tend[id] = now();
  EVP_CIPHER_CTX_free(x);
  EVP_CIPHER_CTX_free(y);
  EVP_CIPHER_free(c);
  EVP_CIPHER_free(h);
  if (lc) OSSL_LIB_CTX_free(lc);
  return NULL;
}

int main(int argc, char** argv) {
  if (argc < 4) {
    fprintf(stderr, "usage: %s MODE PERCTX MAXTHREADS\n", argv[0]);
    return 2;
  }
  MODE = atoi(argv[1]);
  PERCTX = atoi(argv[2]);
  const int maxt = atoi(argv[3]);
  for (int t = 1; t <= maxt && t <= 1024; t *= 2) {
    pthread_t th[1024];
    pthread_barrier_init(&bar, NULL, (unsigned)t);
    for (int i = 0; i < t; i++) pthread_create(&th[i], NULL, work, (void*)(long)i);
    for (int i = 0; i < t; i++) pthread_join(th[i], NULL);
    double a = 1e30, b = 0;
    for (int i = 0; i < t; i++) {
      if (tstart[i] < a) a = tstart[i];
      if (tend[i] > b) b = tend[i];
    }
    printf("mode %d perctx %d threads %4d: %8.0f kpkt/s (%.2f kpkt/s per thread)\n", MODE, PERCTX, t,
           t * NPKT / (b - a) / 1e3, NPKT / (b - a) / 1e3);
    pthread_barrier_destroy(&bar);
  }
  return 0;
}
