/*
 * mq_aead.h — C ABI of the MI355X-native QUIC packet-protection library (libmq_aead.so).
 *
 * Drop-in boundary for milli-quic's packet-protection path (reference at
 * computer-whisperer/milli-quic; all file:line citations below are relative to that tree):
 *
 *   trait Aead              src/crypto/aead.rs:8-42          -> mq_aead_* (per-packet, in place)
 *   trait HeaderProtection  src/crypto/header_protection.rs:6-13 -> mq_hp_*
 *   trait CryptoProvider    src/crypto/mod.rs:38-51          -> mq_aead_new / mq_hp_new (suite + key)
 *   trait Hkdf + key_schedule src/crypto/hkdf.rs:7-16, src/crypto/key_schedule.rs:23-151 -> mq_hkdf_* / mq_derive_*
 *   DirectionalKeys::nonce  src/crypto/mod.rs:66-74          -> mq_nonce
 *
 * plus a device-resident BATCH API (mq_batch_*), which the reference lacks: it runs the send
 * composite of src/connection/transmit.rs:499-755 (seal + header protection) and the receive
 * composite of src/connection/recv.rs:340-421,953-1025 (header-protection removal, decode_pn,
 * open) over a whole arena of packets in HBM (8 packets per wave, 8 lanes per packet), ordered
 * on a HIP stream.
 *
 * All entry points take plain pointers and sizes. Every compute path runs on the GPU (gfx950);
 * there is no CPU fallback: without a usable device the calls return MQ_ERR_NO_DEVICE.
 */
#ifndef MQ_AEAD_H
#define MQ_AEAD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes (reference: src/error.rs:144-170) ------------------------------------- */
#define MQ_OK                    0  /* Ok(..)                                               */
#define MQ_ERR_CRYPTO            1  /* Error::Crypto: bad nonce length, short ciphertext,
                                       tag mismatch, bad key length, sample out of range     */
#define MQ_ERR_BUFFER_TOO_SMALL  2  /* Error::BufferTooSmall { needed }                     */
#define MQ_ERR_INVALID_ARG       3  /* cases where the reference panics (index out of range:
                                       rustcrypto.rs:83,154,180,201-204) or a NULL pointer   */
#define MQ_ERR_PROTOCOL          4  /* Error::Transport(ProtocolViolation): decoded pn > 2^62-1
                                       (recv.rs:393-395, 994-997)                             */
#define MQ_ERR_SUITE             5  /* packet's key suite differs from the launched kernel's  */
#define MQ_ERR_NO_DEVICE         6  /* no gfx950 device / HIP runtime failure                 */
#define MQ_ERR_HIP               7  /* HIP runtime error during a call                        */
#define MQ_ERR_TLS               8  /* Error::Tls: an opened TLS record whose plaintext has no
                                       valid inner content type (tcp_tls/connection.rs:546-556,
                                       record.rs:131-139); the plaintext IS in place, as in the
                                       reference (open_in_place succeeded before the scan)     */

/* ---- cipher suites (TLS_AES_128_GCM_SHA256 = 0x1301, TLS_CHACHA20_POLY1305_SHA256 = 0x1303;
 *      reference tls/handshake.rs:636-654 maps KEY_LEN 16 -> 0x1301, 32 -> 0x1303) ----------- */
#define MQ_SUITE_AES128GCM       1
#define MQ_SUITE_CHACHA20        2
#define MQ_SUITE_MIXED           0xFF /* batch hint: per-packet suite from the key table       */

#define MQ_NONCE_LEN 12
#define MQ_TAG_LEN   16
#define MQ_SAMPLE_LEN 16
#define MQ_MASK_LEN   5

/* ---- key material (host side; what CryptoProvider::aead + ::header_protection consume) ---- */
typedef struct mq_key_material {
  uint32_t suite;      /* MQ_SUITE_AES128GCM or MQ_SUITE_CHACHA20                              */
  uint32_t reserved;
  uint8_t  key[32];    /* AEAD key: 16 B (AES) or 32 B (ChaCha20)                              */
  uint8_t  iv[12];     /* DirectionalKeys::iv (src/crypto/mod.rs:57-59)                        */
  uint8_t  pad[4];
  uint8_t  hp[32];     /* header-protection key: 16 B (AES) or 32 B (ChaCha20)                 */
} mq_key_material;     /* 88 bytes */

/* ---- per-packet descriptor of the batch API (32 bytes, read once per packet) -------------- */
#define MQ_PKT_LONG_HEADER  0x01  /* header protection masks byte 0 with 0x0f (else 0x1f)     */
#define MQ_PKT_NO_HP        0x02  /* plain AEAD: no header protection, pn_len taken from the
                                     descriptor on open, AAD = bytes [0, pn_offset + pn_len)  */
#define MQ_PKT_TLS_RECORD   0x06  /* TLS 1.3 record (includes MQ_PKT_NO_HP): offset = the 5-byte
                                     record header, len = 5 + data + 1 + 16 (seal) or 5 + the
                                     header's length field (open), pn = sequence number
                                     (record.rs:70-78 nonce), pn_offset = 5, pn_len = 0, and on
                                     seal `reserved` = the inner content type. Seal writes the
                                     header (23, 0x0303, len - 5) and the inner content type
                                     byte, then seals with AAD = header (connection.rs:561-600) */
#define MQ_PKT_NO_RECV_LIMIT 0x08 /* open only: lift the receive composite's 2048-byte limit.
                                     By default, as in the reference — recv_short and
                                     decrypt_long_packet copy the packet into a 2048-B stack
                                     buffer and return Err(BufferTooSmall { needed: len })
                                     above that (recv.rs:356-360, 962-965) — a header-protected
                                     packet with len > 2048 gets MQ_ERR_BUFFER_TOO_SMALL
                                     (needed = its desc.len) and is left untouched. With this
                                     flag such packets are opened (a deliberate divergence for
                                     callers with larger receive buffers).                    */
#define MQ_RECV_MAX_PACKET 2048

typedef struct mq_pkt_desc {
  uint64_t offset;     /* byte offset of the packet's first header byte in the arena            */
  uint32_t len;        /* seal: bytes the protected packet occupies = pn_offset + pn_len +
                          payload_len + 16 (the arena must hold them);
                          open: protected length (pn_offset + Length for long headers)         */
  uint32_t key_id;     /* row of the key table                                                  */
  uint64_t pn;         /* seal: full packet number; open: largest_pn of the PN space (decode_pn) */
  uint16_t pn_offset;  /* offset of the packet-number field (= 1 + dcid_len for short headers)  */
  uint8_t  pn_len;     /* seal: encoded PN length 1..4 (already in the header); open: ignored
                          unless MQ_PKT_NO_HP                                                     */
  uint8_t  flags;      /* MQ_PKT_*                                                              */
  uint32_t reserved;
} mq_pkt_desc;

/* ---- send composite from frames (mq_batch_protect; transmit.rs:499-755) ------------------- */
#define MQ_LEVEL_INITIAL      0
#define MQ_LEVEL_HANDSHAKE    1
#define MQ_LEVEL_APPLICATION  2
#define MQ_SEND_PAD_TO_MIN    0x01  /* Initial: pad to MIN_INITIAL_PACKET_SIZE = 1200
                                       (build_and_encrypt_initial_packet's pad_to_min)          */

typedef struct mq_conn_send {       /* what the send path reads from a Connection             */
  uint8_t  dcid_len;                /* remote_cid (transmit.rs:513, 653), <= 20                */
  uint8_t  scid_len;                /* local_cids[0] or empty (:514-518, 654-658), <= 20       */
  uint8_t  key_phase;               /* keys.key_phase() for 1-RTT (:677-678)                   */
  uint8_t  reserved0;
  uint8_t  dcid[20];
  uint8_t  scid[20];
  uint32_t key_row[3];              /* key-table row of the send keys per level (Initial rows
                                       must be AES-128-GCM, keys.rs:131-136)                   */
  uint32_t reserved1[2];
} mq_conn_send;                     /* 64 bytes */

typedef struct mq_send_req {        /* one packet to build and protect                         */
  uint64_t frames_offset;           /* payload_frames in the frames arena                      */
  uint64_t out_offset;              /* where the packet is written in the output arena         */
  uint64_t pn;                      /* next_pn[level]                                          */
  uint64_t largest_acked;           /* largest_recv_pn[level].unwrap_or(0) (:509, 635): picks
                                       the PN length (number.rs:9-26)                          */
  uint32_t frame_len;
  uint32_t out_cap;                 /* bytes available at out_offset (the reference's out.len()) */
  uint32_t conn;                    /* row of the connection table                             */
  uint8_t  level;                   /* MQ_LEVEL_*                                               */
  uint8_t  flags;                   /* MQ_SEND_*                                                */
  uint16_t reserved;
} mq_send_req;                      /* 48 bytes */

/* ---- receive composite over raw datagrams (mq_batch_recv; recv.rs:189-510, 953-1025) ----- */
#define MQ_ERR_DEFERRED          9  /* mq_batch_recv: not processed because an earlier packet of
                                       its connection changed state differently than the batch
                                       speculated (or a second key update in one batch) — bytes
                                       untouched; resubmit after the batch                      */
#define MQ_RECV_HAS_INITIAL   0x01  /* mq_conn_recv.flags: which recv keys are installed         */
#define MQ_RECV_HAS_HANDSHAKE 0x02
#define MQ_RECV_HAS_APP       0x04  /* current 1-RTT keys (app_row[1])                           */
#define MQ_RECV_HAS_PREV      0x08  /* previous generation (app_row[0], keys.rs:585-589)          */
#define MQ_RECV_HAS_NEXT      0x10  /* next generation, derived ahead with "quic ku"
                                       (app_row[2]; keys.rs:498-522)                            */

typedef struct mq_dgram {           /* one received UDP datagram, in arrival order              */
  uint64_t offset;                  /* in the arena                                             */
  uint32_t len;
  uint32_t conn;                    /* row of the connection table (the caller's DCID lookup)    */
} mq_dgram;                         /* 16 bytes */

typedef struct mq_conn_recv {       /* receive-side connection state, updated in place           */
  uint32_t initial_row;             /* key-table rows of the recv keys (HP keys are shared by   */
  uint32_t handshake_row;           /* all 1-RTT generations, keys.rs:386-414)                  */
  uint32_t app_row[3];              /* 1-RTT: previous, current, next generation                */
  uint8_t  dcid_len;                /* local CID length for short headers (recv.rs:341-345)     */
  uint8_t  key_phase;               /* keys.key_phase() (keys.rs:364-366)                        */
  uint8_t  flags;                   /* MQ_RECV_HAS_*                                             */
  uint8_t  key_updates;             /* out: peer key updates confirmed by this batch             */
  uint64_t largest_pn[3];           /* largest_recv_pn per level; None == 0 (unwrap_or(0))       */
  uint64_t reserved[2];
} mq_conn_recv;                     /* 64 bytes */

typedef struct mq_recv_pkt {        /* one packet found in the datagrams, in arrival order       */
  uint64_t offset;                  /* packet start in the arena                                 */
  uint64_t pn;                      /* decoded packet number (MQ_OK)                             */
  uint32_t len;                     /* long: pn_offset + Length; short: rest of the datagram     */
  uint32_t dgram;                   /* datagram index                                            */
  uint16_t payload_offset;          /* MQ_OK: plaintext at offset + payload_offset, length
                                       len - payload_offset - 16                                 */
  uint8_t  level;                   /* MQ_LEVEL_*                                                 */
  uint8_t  status;                  /* MQ_* (the Result of recv_initial / _handshake / _short)   */
  uint8_t  key_gen;                 /* opened 1-RTT packets: keys of the 0 previous, 1 current,
                                       2 next generation (0 otherwise)                           */
  uint8_t  reserved[3];
} mq_recv_pkt;                      /* 32 bytes */

/* ---- opaque handles ---------------------------------------------------------------------- */
typedef struct mq_aead_ctx mq_aead_ctx;     /* one Aead instance (immutable after creation)      */
typedef struct mq_hp_ctx mq_hp_ctx;         /* one HeaderProtection instance                     */
typedef struct mq_keytable mq_keytable;     /* device-resident table of expanded keys            */

/* ---- library / device ---------------------------------------------------------------------- */
/* Devices. Every object is bound to the device it was created on: key tables (mq_keytable_create)
 * and AEAD / HP contexts (mq_aead_new, mq_hp_new) are created on the calling thread's device —
 * the one it selected with mq_device_init, else its current HIP device — and every later call on
 * them runs on THAT device, whichever thread makes it (a batch call's stream and buffers must
 * belong to the key table's device). The library never changes a thread's current HIP device,
 * except in mq_device_init, so one host thread can drive several GPUs, one key table (and stream)
 * per GPU, and threads on different GPUs never see each other's choice. */
const char* mq_version(void);
/* Selects (and makes current) the HIP device this thread creates objects on: MQ_OK, or
 * MQ_ERR_NO_DEVICE (no such device / not a gfx950; the thread's previous selection stays). */
int mq_device_init(int device);
/* The device this thread creates objects on (its selection, else its current HIP device), or -1
 * when that is not a usable gfx950. */
int mq_device_current(void);
/* The device a key table lives on (-1 for NULL). */
int mq_keytable_device(const mq_keytable* kt);
/* Mixed / multi-key batches run some tile kernels on side streams forked from and joined back
 * to the caller's stream (one set per device and caller stream, at most 64 sets, least recently
 * used dropped). Call before destroying a stream that such batches used, to free its set now. */
void mq_stream_release(void* stream);
/* Diagnostic: device-side phases (ns) of the last per-packet call served by device dev's resident
 * workgroup — the poll round trip that saw it, request + first 2 KiB loaded, rest loaded, first
 * half of the work (seal: cipher, open: MAC), second half, written back — then three host-side
 * ones: request written, waiting for `done` (0 if the call relaunched the server), result copied.
 * Writes min(n, 9) values and returns that count; 0 before any resident call. */
int mq_resident_phases(int device, uint32_t* ns, int n);
const char* mq_status_str(int status);
/* Diagnostic switches (A/B measurements and tests that run two kernel paths on one batch; no
 * switch changes a result): MQ_CC_NARROW, MQ_CC_LONG, MQ_CC_LIST, MQ_HP_FORK, MQ_AES_SEG,
 * MQ_PROTECT_FUSED, MQ_RESIDENT, MQ_RESIDENT_TIMEOUT_US, MQ_RECV_SEG, MQ_AES_HOT_SEG, MQ_AES_NARROW.
 * Each starts from the environment variable of that name (read once, at the first use of any
 * switch); value < 0 unsets it (the product behaviour). MQ_OK, or MQ_ERR_INVALID_ARG for an unknown name. A batch reads each
 * switch once per call. */
int mq_debug_option(const char* name, long value);
/* The switch's value: -1 unset, -2 unknown name. */
long mq_debug_option_get(const char* name);
/* The kernel family a flat single-suite ChaCha20 batch of n packets over arena_len bytes runs with
 * this suite_hint (MQ_BATCH_LEN_HINT included): 0 narrow tiles (short packets), 1 octet tiles over
 * 10-KiB images, 2 over 13-KiB, 3 over 20-KiB images; -1 for n = 0. (Diagnostic switches aside.) */
int mq_debug_chacha_flat_kind(uint64_t arena_len, uint32_t n, uint32_t suite_hint);
/* The same for a flat single-key AES-128-GCM batch: its lanes per packet — 2 (tiles of 32 short
 * packets), 4 (16 packets) or 8 (octet tiles); -1 for n = 0. */
int mq_debug_aes_flat_kind(uint64_t arena_len, uint32_t n, uint32_t suite_hint);

/* ---- CryptoProvider::aead / Aead (per packet, host buffers; runs the HIP kernels) ----------- */
/* provider.aead(key): key_len must equal KEY_LEN of the suite (rustcrypto.rs:234-236, 267-269) */
int mq_aead_new(uint32_t suite, const uint8_t* key, size_t key_len, mq_aead_ctx** out);
void mq_aead_free(mq_aead_ctx* ctx);
size_t mq_aead_key_len(uint32_t suite);     /* Aead::KEY_LEN (16 / 32), 0 for an unknown suite   */
/* Aead::seal_in_place (aead.rs:22-28, rustcrypto.rs:38-63 / 111-135): buf[..payload_len] holds
 * plaintext; on MQ_OK buf[..payload_len+16] holds ciphertext||tag and *out_len = payload_len+16.
 * MQ_ERR_CRYPTO if nonce_len != 12; MQ_ERR_BUFFER_TOO_SMALL (with *needed) if
 * buf_len < payload_len + 16. */
int mq_aead_seal_in_place(const mq_aead_ctx* ctx, const uint8_t* nonce, size_t nonce_len,
                          const uint8_t* aad, size_t aad_len, uint8_t* buf, size_t buf_len,
                          size_t payload_len, size_t* out_len, size_t* needed);
/* Aead::open_in_place (aead.rs:35-41, rustcrypto.rs:65-94 / 137-165): buf[..ct_len] holds
 * ciphertext||tag; on MQ_OK buf[..ct_len-16] holds plaintext and *out_len = ct_len - 16.
 * MQ_ERR_CRYPTO on nonce_len != 12, ct_len < 16, or tag mismatch (buffer left unchanged);
 * MQ_ERR_INVALID_ARG if ct_len > buf_len (the reference panics). */
int mq_aead_open_in_place(const mq_aead_ctx* ctx, const uint8_t* nonce, size_t nonce_len,
                          const uint8_t* aad, size_t aad_len, uint8_t* buf, size_t buf_len,
                          size_t ct_len, size_t* out_len);

/* ---- CryptoProvider::header_protection / HeaderProtection::mask ---------------------------- */
int mq_hp_new(uint32_t suite, const uint8_t* key, size_t key_len, mq_hp_ctx** out);
void mq_hp_free(mq_hp_ctx* ctx);
/* HeaderProtection::mask (header_protection.rs:12; rustcrypto.rs:175-186 / 197-220):
 * MQ_ERR_INVALID_ARG if sample_len < 16 (the reference panics). */
int mq_hp_mask(const mq_hp_ctx* ctx, const uint8_t* sample, size_t sample_len, uint8_t mask[5]);

/* ---- DirectionalKeys::nonce (src/crypto/mod.rs:66-74) -------------------------------------- */
void mq_nonce(const uint8_t iv[12], uint64_t packet_number, uint8_t nonce[12]);

/* ---- HKDF-SHA256 + QUIC key schedule (host; per connection, not per packet) ---------------- */
/* Hkdf::extract / Hkdf::expand (rustcrypto.rs:9-24) */
void mq_hkdf_extract(const uint8_t* salt, size_t salt_len, const uint8_t* ikm, size_t ikm_len,
                     uint8_t prk[32]);
int mq_hkdf_expand(const uint8_t* prk, size_t prk_len, const uint8_t* info, size_t info_len,
                   uint8_t* okm, size_t okm_len);
/* hkdf_expand_label (key_schedule.rs:23-55): MQ_ERR_CRYPTO if the info would exceed 80 bytes */
int mq_hkdf_expand_label(const uint8_t* secret, size_t secret_len, const uint8_t* label,
                         size_t label_len, const uint8_t* context, size_t context_len,
                         uint8_t* out, size_t out_len);
/* derive_initial_secrets (key_schedule.rs:60-72) */
int mq_derive_initial_secrets(const uint8_t* dcid, size_t dcid_len, uint8_t client_secret[32],
                              uint8_t server_secret[32]);
/* derive_packet_keys + derive_directional_keys (key_schedule.rs:79-90, 123-151): fills key
 * (KEY_LEN), iv, hp (max(KEY_LEN,16) bytes) of `out` for `suite` from a 32-byte secret */
int mq_derive_key_material(uint32_t suite, const uint8_t* secret, size_t secret_len,
                           mq_key_material* out);
/* derive_next_application_secret (key_schedule.rs:114-120), label "quic ku" */
int mq_derive_next_secret(const uint8_t* secret, size_t secret_len, uint8_t next[32]);

/* ---- device key table ----------------------------------------------------------------------- */
/* Expands every row (AES key schedules, GHASH subkey) on the host once and uploads the table. */
int mq_keytable_create(const mq_key_material* rows, uint32_t n_rows, mq_keytable** out);
int mq_keytable_update(mq_keytable* kt, uint32_t first_row, const mq_key_material* rows,
                       uint32_t n_rows);
uint32_t mq_keytable_rows(const mq_keytable* kt);
void mq_keytable_free(mq_keytable* kt);

/* Batched Initial key derivation on the GPU (server-side Initial floods): derive_initial
 * (connection/keys.rs:181-212 = key_schedule.rs:60-72 + derive_directional_keys :123-151 +
 * Aes128GcmProvider::aead / header_protection, rustcrypto.rs:232-252) for n client DCIDs.
 * dcids: device, 20-byte stride; dcid_lens: device, n bytes. Writes key-table rows
 * first_row + 2i (client keys) and first_row + 2i + 1 (server keys) directly on the device;
 * km_out (device, 2n entries, may be NULL) receives the same key material; status (device, n
 * bytes): MQ_OK, or MQ_ERR_INVALID_ARG for a DCID longer than 20 bytes (its rows get suite 0).
 * MQ_ERR_INVALID_ARG (nothing launched) if first_row + 2n exceeds the table. */
int mq_batch_derive_initial(mq_keytable* kt, uint32_t first_row, const uint8_t* dcids,
                            const uint8_t* dcid_lens, uint32_t n, mq_key_material* km_out,
                            uint8_t* status, void* stream);

/* ---- batch API (device pointers, stream-ordered, asynchronous) ------------------------------ */
/* Optional length hint, OR-ed into suite_hint of mq_batch_seal / mq_batch_open and the record
 * variants: the batch's typical (average) protected packet length in bytes (saturating at 65535).
 * Flat ChaCha20 batches choose their tile geometry from it (LDS image per 8-packet tile, or the
 * narrow tiles of short packets: mq_debug_chacha_flat_kind). Without it the library takes
 * arena_len / n, which is the batch's own figure only when the arena holds just this batch: a
 * batch over part of a larger arena (a ring buffer, one chunk of a pipeline) should pass the hint,
 * or it may run a kernel sized for longer packets. Results never depend on it. */
#define MQ_BATCH_LEN_HINT(len) ((uint32_t)((len) > 0xFFFF ? 0xFFFF : (len)) << 16)

/* `arena` is device memory of `arena_len` bytes holding the packets; `desc` (n entries) and
 * `status` (n bytes, written with MQ_* per packet) are device memory; `pn_out` (open only,
 * may be NULL) receives each packet's decoded packet number. `suite_hint` is
 * MQ_SUITE_CHACHA20 / MQ_SUITE_AES128GCM for a single-suite batch (one launch; rows of the
 * other suite get MQ_ERR_SUITE) or MQ_SUITE_MIXED (packets are partitioned on the device first
 * by suite and 64-B length class, so that a tile's packets need similar work; results do not
 * depend on the order; needs `workspace` of mq_batch_workspace_size(n) bytes of device memory;
 * at most 2^30 packets per mixed batch, else MQ_ERR_INVALID_ARG).
 * `workspace` is optional for single-suite batches; given to mq_batch_open it also enables the
 * header-protection pre-pass (one lane per packet computes the mask, so the packet kernel spends
 * no keystream slot on it), and given with an AES batch over a key table of several rows it
 * routes the batch through the same partition, which also groups AES packets by key (tiles of
 * one key run their GHASH through a table) — same results, faster. Workspace contents need not
 * be initialised.
 * `stream` is a hipStream_t (NULL = default stream). Returns MQ_OK once the work is enqueued. */
size_t mq_batch_workspace_size(uint32_t n);
int mq_batch_seal(const mq_keytable* kt, uint8_t* arena, uint64_t arena_len,
                  const mq_pkt_desc* desc, uint32_t n, uint8_t* status, uint32_t suite_hint,
                  void* workspace, void* stream);
int mq_batch_open(const mq_keytable* kt, uint8_t* arena, uint64_t arena_len,
                  const mq_pkt_desc* desc, uint32_t n, uint8_t* status, uint64_t* pn_out,
                  uint32_t suite_hint, void* workspace, void* stream);
/* Send composite from plaintext frames: per request, what
 * build_and_encrypt_initial_packet (transmit.rs:499-622) and build_and_encrypt_packet
 * (:625-755) do after frame assembly — PN length (number.rs:9-26), Initial / Handshake / short
 * header with the Length varint (long_header.rs:214-314, short_header.rs:33-47, first byte
 * 0x40 | key_phase << 2 | pn_len - 1), encode_pn, PADDING (Initial to 1200 with pad_to_min,
 * else pn_len + payload + tag >= 20), seal with AAD = header || PN, header protection — writing
 * the protected packet at out + req.out_offset. pkt_len[i] = packet length (MQ_OK), or the
 * reference's `needed` for MQ_ERR_BUFFER_TOO_SMALL, else 0. Packets that fail leave `out`
 * untouched. Per packet, in this order: MQ_ERR_INVALID_ARG for a bad conn / level / key row /
 * range; MQ_ERR_SUITE for a row of another suite than suite_hint (MQ_SUITE_MIXED: any) or an
 * Initial row that is not AES-128-GCM; MQ_ERR_INVALID_ARG for a CID over 20 bytes; then the
 * buffer checks; a row of neither suite fails the seal (MQ_ERR_SUITE). With MQ_SUITE_CHACHA20
 * the whole batch is one kernel that builds each packet in LDS and seals it there (the
 * workspace is then unused). `frames`, `out`, `conns`, `req`, `status`, `pkt_len` and
 * `workspace` (mq_batch_protect_workspace_size(n) bytes) are device memory; frames and out must
 * not overlap. */
size_t mq_batch_protect_workspace_size(uint32_t n);
int mq_batch_protect(const mq_keytable* kt, const mq_conn_send* conns, uint32_t n_conns,
                     const uint8_t* frames, uint64_t frames_len, uint8_t* out, uint64_t out_len,
                     const mq_send_req* req, uint32_t n, uint8_t* status, uint32_t* pkt_len,
                     uint32_t suite_hint, void* workspace, void* stream);

/* Receive composite over raw datagrams: Connection::recv's datagram loop
 * (recv.rs:189-265) without frame dispatch — CoalescedPackets splitting (packet/coalesce.rs:26-133),
 * long-header parsing (long_header.rs:92-206), header-protection removal, decode_pn against the
 * connection's running largest_recv_pn, the 1-RTT key-phase logic (current keys, previous keys
 * on failure, next keys + rotation on a phase flip; recv.rs:410-509) and open. Datagrams of one
 * connection are processed in arrival order (one sequential pass per connection on the device,
 * speculating that packets open; MQ_ERR_DEFERRED marks the rare packets whose inputs the
 * speculation got wrong). 0-RTT, Retry and Version Negotiation packets are skipped, as in the
 * reference (:221-226). Opened packets are decrypted in place (header unmasked); others keep
 * their bytes. pkts receives up to max_pkts records in arrival order, *n_pkts (device) their
 * count; conns is updated (largest_recv_pn, key phase / rotation). Initial keys must already be
 * installed (mq_batch_derive_initial). All pointers are device memory; workspace has
 * mq_batch_recv_workspace_size(n_dgrams, max_pkts, n_conns) bytes.
 * *n_pkts is the number of packets the datagrams split into, which can EXCEED max_pkts: only the
 * first max_pkts (in arrival order) are processed and recorded; the rest are neither opened nor
 * reflected in conns — resubmit their datagrams (or size max_pkts from *n_pkts).
 * A packet that opened under inputs other than the ones the sequential reference would have chosen
 * (possible only when an earlier packet of its connection failed where the batch speculated it
 * would open, e.g. a PN decoded against a largest PN the reference never reached) reports
 * MQ_ERR_CRYPTO, as the reference would, and is sealed again under the inputs that opened it, so
 * its bytes are exactly as received — like every packet that fails. */
size_t mq_batch_recv_workspace_size(uint32_t n_dgrams, uint32_t max_pkts, uint32_t n_conns);
int mq_batch_recv(const mq_keytable* kt, mq_conn_recv* conns, uint32_t n_conns, uint8_t* arena,
                  uint64_t arena_len, const mq_dgram* dgrams, uint32_t n_dgrams, mq_recv_pkt* pkts,
                  uint32_t max_pkts, uint32_t* n_pkts, void* workspace, void* stream);

/* Batched HeaderProtection::mask: masks[i*5..] = mask(key_table[key_ids[i]].hp, samples[i*16..]).
 * An entry whose key id is out of range or whose row holds no valid suite gets an all-zero mask
 * (the call still returns MQ_OK: validate key ids on the caller's side). */
int mq_batch_hp_mask(const mq_keytable* kt, const uint32_t* key_ids, const uint8_t* samples,
                     uint8_t* masks, uint32_t n, void* stream);

/* ---- TLS 1.3 record layer over the same AEAD (the reference's second caller of Aead:
 *      src/tcp_tls/record.rs:70-143, src/tcp_tls/connection.rs:264,306,546-600) ------------ */
/* seal_record (record.rs:88-113): buf[..payload_len] holds plaintext; writes the inner content
 * type at buf[payload_len] and seals payload_len + 1 bytes with AAD = (23, 0x0303,
 * payload_len + 17 as u16). *out_len = payload_len + 17. MQ_ERR_BUFFER_TOO_SMALL (+needed) if
 * buf_len < payload_len + 17; nonce rules as mq_aead_seal_in_place. */
int mq_record_seal(const mq_aead_ctx* ctx, const uint8_t* nonce, size_t nonce_len, uint8_t* buf,
                   size_t buf_len, size_t payload_len, uint8_t inner_type, size_t* out_len,
                   size_t* needed);
/* open_record (record.rs:122-143): opens buf[..ct_len] with AAD = header (the 5 received bytes),
 * then finds the inner content type (last non-zero byte): *data_len, *inner_type. MQ_ERR_TLS if
 * there is none or it is not 20..23 (plaintext left in place, as in the reference). */
int mq_record_open(const mq_aead_ctx* ctx, const uint8_t* nonce, size_t nonce_len, uint8_t* buf,
                   size_t buf_len, size_t ct_len, const uint8_t header[5], size_t* data_len,
                   uint8_t* inner_type);
/* Batched records: descriptors flagged MQ_PKT_TLS_RECORD (see above), any mix with QUIC packets
 * of the same suite hint. Open additionally runs find_inner_content_type (connection.rs:546-556)
 * per record: info[i] = data_len | (uint64_t)inner_type << 32 (QUIC rows: the decoded PN). */
int mq_batch_seal_records(const mq_keytable* kt, uint8_t* arena, uint64_t arena_len,
                          const mq_pkt_desc* desc, uint32_t n, uint8_t* status, uint32_t suite_hint,
                          void* workspace, void* stream);
int mq_batch_open_records(const mq_keytable* kt, uint8_t* arena, uint64_t arena_len,
                          const mq_pkt_desc* desc, uint32_t n, uint8_t* status, uint64_t* info,
                          uint32_t suite_hint, void* workspace, void* stream);

/* ---- timing hooks for bench.py (HIP events on the launch stream) ---------------------------- */
/* Time `iters` back-to-back (seal, open) pairs on `stream`; returns per-kernel average ms. */
int mq_batch_time_seal_open(const mq_keytable* kt, uint8_t* arena, uint64_t arena_len,
                            const mq_pkt_desc* desc, uint32_t n, uint8_t* status, uint64_t* pn_out,
                            uint32_t suite_hint, void* workspace, void* stream, int iters,
                            float* seal_ms, float* open_ms);

#ifdef __cplusplus
}
#endif
#endif /* MQ_AEAD_H */
