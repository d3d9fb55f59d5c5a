/*
 * mq_oracle.h — CPU restatement of milli-quic's packet-protection path.
 *
 * TEST INFRASTRUCTURE ONLY. This code is the parity checker for the HIP kernels in
 * milli_quic_amd/csrc. Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * may load it; the product library never links or calls it.
 *
 * The reference (computer-whisperer/milli-quic, Rust) delegates the arithmetic to
 * un-vendored crates pinned in its Cargo.lock: chacha20poly1305 0.10.1, chacha20 0.9.1,
 * poly1305 0.8.0, aes-gcm 0.10.3, aes 0.8.4, ghash 0.5.1 / polyval 0.6.2, ctr 0.9.2,
 * hkdf 0.12 / sha2 0.10. Those crates implement the published algorithms restated here:
 * RFC 8439 (ChaCha20, Poly1305, AEAD_CHACHA20_POLY1305), FIPS-197 (AES-128),
 * NIST SP 800-38D (GCM), RFC 5869 (HKDF), FIPS 180-4 (SHA-256), RFC 9001 §5 (QUIC packet
 * protection). The adapter semantics (argument checks, tag placement, error mapping) follow
 * the reference's own src/crypto/rustcrypto.rs; each function cites the line it restates.
 *
 * Parity pin: checked in tests/ against RFC 9001 Appendix A (A.1 keys, A.2/A.3 AES Initial
 * packets, A.5 ChaCha20 short-header packet; text at reference rfc/rfc9001.txt:2319-2553),
 * the reference's captured curl Initial (src/connection/mod.rs:2210), RFC 8439 §2.8.2 and
 * OpenSSL-generated vectors committed under tests/golden/.
 */
#ifndef MQ_ORACLE_H
#define MQ_ORACLE_H

#include <stddef.h>
#include <stdint.h>
#include "../include/mq_aead.h"

#ifdef __cplusplus
extern "C" {
#endif

/* primitives */
void orc_chacha20_block(const uint8_t key[32], uint32_t counter, const uint8_t nonce[12],
                        uint8_t out[64]);
void orc_poly1305(const uint8_t key[32], const uint8_t* msg, size_t len, uint8_t tag[16]);
void orc_aes128_expand(const uint8_t key[16], uint32_t rk[44]);
void orc_aes128_encrypt(const uint32_t rk[44], const uint8_t in[16], uint8_t out[16]);
void orc_gf128_mul(const uint8_t x[16], const uint8_t y[16], uint8_t out[16]);
void orc_ghash(const uint8_t h[16], const uint8_t* aad, size_t aad_len, const uint8_t* ct,
               size_t ct_len, uint8_t out[16]);
void orc_sha256(const uint8_t* msg, size_t len, uint8_t out[32]);
void orc_hmac_sha256(const uint8_t* key, size_t key_len, const uint8_t* msg, size_t len,
                     uint8_t out[32]);

/* Aead / HeaderProtection semantics (MQ_* status codes of include/mq_aead.h) */
int orc_aead_seal(uint32_t suite, const uint8_t* key, size_t key_len, const uint8_t* nonce,
                  size_t nonce_len, const uint8_t* aad, size_t aad_len, uint8_t* buf,
                  size_t buf_len, size_t payload_len, size_t* out_len, size_t* needed);
int orc_aead_open(uint32_t suite, const uint8_t* key, size_t key_len, const uint8_t* nonce,
                  size_t nonce_len, const uint8_t* aad, size_t aad_len, uint8_t* buf,
                  size_t buf_len, size_t ct_len, size_t* out_len);
int orc_hp_mask(uint32_t suite, const uint8_t* hp_key, size_t key_len, const uint8_t* sample,
                size_t sample_len, uint8_t mask[5]);
void orc_nonce(const uint8_t iv[12], uint64_t pn, uint8_t nonce[12]);

/* key schedule */
void orc_hkdf_extract(const uint8_t* salt, size_t salt_len, const uint8_t* ikm, size_t ikm_len,
                      uint8_t prk[32]);
int orc_hkdf_expand(const uint8_t* prk, size_t prk_len, const uint8_t* info, size_t info_len,
                    uint8_t* okm, size_t okm_len);
int orc_hkdf_expand_label(const uint8_t* secret, size_t secret_len, const uint8_t* label,
                          size_t label_len, const uint8_t* ctx, size_t ctx_len, uint8_t* out,
                          size_t out_len);
int orc_derive_initial_secrets(const uint8_t* dcid, size_t dcid_len, uint8_t client[32],
                               uint8_t server[32]);
int orc_derive_key_material(uint32_t suite, const uint8_t* secret, size_t secret_len,
                            mq_key_material* out);

/* packet-number helpers */
size_t orc_pn_length(uint64_t full_pn, uint64_t largest_acked);
uint64_t orc_decode_pn(uint32_t truncated, size_t pn_len, uint64_t largest_pn);

/* composites over one packet in `pkt` (len bytes as in mq_pkt_desc) */
int orc_protect_packet(const mq_key_material* km, uint8_t* pkt, const mq_pkt_desc* d);
int orc_unprotect_packet(const mq_key_material* km, uint8_t* pkt, const mq_pkt_desc* d,
                         uint64_t* pn_out);

/* send composite from frames (transmit.rs:499-755): header / PN encode, padding, seal, HP */
int orc_protect_frames(const mq_key_material* km, const mq_conn_send* c, const mq_send_req* r,
                       const uint8_t* frames, uint8_t* out, uint64_t out_cap, uint32_t* len);
void orc_batch_protect(const mq_key_material* rows, uint32_t n_rows, const mq_conn_send* conns,
                       uint32_t n_conns, const uint8_t* frames, uint64_t frames_len, uint8_t* out,
                       uint64_t out_len, const mq_send_req* req, uint32_t n, uint8_t* status,
                       uint32_t* pkt_len, uint32_t suite_hint);

/* receive composite over raw datagrams (recv.rs:189-510, 953-1025), conns updated in place */
void orc_batch_recv(const mq_key_material* rows, uint32_t n_rows, mq_conn_recv* conns, uint32_t n_conns,
                    uint8_t* arena, uint64_t arena_len, const mq_dgram* dg, uint32_t n_dgrams,
                    mq_recv_pkt* out, uint32_t max_pkts, uint32_t* n_pkts);
/* the same on `threads` threads (connections split over them; identical results) */
void orc_batch_recv_mt(const mq_key_material* rows, uint32_t n_rows, mq_conn_recv* conns, uint32_t n_conns,
                    uint8_t* arena, uint64_t arena_len, const mq_dgram* dg, uint32_t n_dgrams,
                    mq_recv_pkt* out, uint32_t max_pkts, uint32_t* n_pkts, int threads);

/* batch drivers with the product's descriptor semantics; `threads` <= 1 runs serially */
void orc_batch_seal(const mq_key_material* rows, uint32_t n_rows, uint8_t* arena,
                    uint64_t arena_len, const mq_pkt_desc* desc, uint32_t n, uint8_t* status,
                    uint32_t suite_hint, int threads);
void orc_batch_open(const mq_key_material* rows, uint32_t n_rows, uint8_t* arena,
                    uint64_t arena_len, const mq_pkt_desc* desc, uint32_t n, uint8_t* status,
                    uint64_t* pn_out, uint32_t suite_hint, int threads);

#ifdef __cplusplus
}
#endif
#endif
