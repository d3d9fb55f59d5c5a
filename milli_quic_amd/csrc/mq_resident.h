// mq_resident.h — the resident per-packet server (mq_resident.hip): request / control layout in
// pinned host memory, shared by the host (mq_host.cpp) and the device kernel.
//
// The reference calls Aead::seal_in_place / open_in_place and HeaderProtection::mask once per
// packet, synchronously (transmit.rs:713-719, recv.rs:416-421). A kernel launch per call costs
// 30-40 us (r02), so per-packet calls go to one resident workgroup per device that polls this
// mailbox: the host writes the request and bumps `seq`; the kernel serves it and publishes `done`.
// The body sits at a 16-B aligned data offset (pay_off), so the workgroup's keystream words and
// MAC blocks are aligned LDS dwords.
#pragma once
#include <stdint.h>

namespace mq {

constexpr uint32_t kResMaxPkt = 16 * 1024 + 256;  // aad + body + tag of one call (TLS records fit)

enum ResOp : uint32_t { kResSeal = 0, kResOpen = 1, kResHp = 2 };
enum ResState : uint32_t { kResExited = 0, kResRunning = 1, kResExiting = 2 };
// phases of a request (ResCtl::phase): the poll round trip that saw it, request + first 2 KiB
// loaded, rest loaded, first half of the work (seal: cipher, open: MAC), second half, written
// back (before `done`)
constexpr int kResPhases = 6;

// control words, each on its own 64-B line
struct alignas(64) ResCtl {
  uint32_t seq;           // host: number of the latest request (written after the request)
  uint32_t stop;          // host: 1 = leave now (process exit); polled with seq in one 8-B load
  uint32_t pad0[14];
  uint32_t done;          // device: number of the latest request served
  uint32_t status;        // device: MQ_* of that request
  uint32_t mask0, mask1;  // device: header-protection mask (kResHp)
  uint32_t phase[kResPhases];  // device: wall-clock ticks of the last request's phases (diagnostic)
  uint32_t pad1[12 - kResPhases];
  uint32_t state;         // device: ResState (host sets kResRunning before a launch)
  uint32_t pad2[15];
};

// one request (host -> device)
struct alignas(64) ResReq {
  uint32_t op, suite, aad_len, body_len;  // body: plaintext (seal) / ciphertext || tag (open)
  uint32_t nonce[3];                      // the 12-B nonce as little-endian words
  uint32_t pay_off;                       // data offset of the body: aad_len rounded up to 16 B
  uint32_t key[8];                        // ChaCha20 AEAD key (LE words)
  uint32_t hp[8];                         // ChaCha20 HP key (LE words)
  uint32_t aes_rk[44];                    // AES-128 round keys, AEAD key (FIPS-197 BE words)
  uint32_t hp_rk[44];                     // AES-128 round keys, HP key
  uint32_t Hpow[64][4];                   // GHASH H^1 .. H^64 (BE words)
  uint32_t sample[4];                     // HP sample (LE words)
};

struct ResArea {
  ResCtl ctl;
  ResReq req;
  alignas(64) uint8_t data[kResMaxPkt];  // aad, then the body at pay_off (|| room for the tag)
};
static_assert(sizeof(ResReq) % 16 == 0 && sizeof(ResReq) <= 128 * 16, "the request: two 16-B loads per lane");

}  // namespace mq
