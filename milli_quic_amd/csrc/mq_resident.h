// mq_resident.h — the resident per-packet server (mq_resident.hip): mailbox layout in pinned host
// memory, shared by the host (mq_host.cpp) and the device kernel.
//
// The reference calls Aead::seal_in_place / open_in_place and HeaderProtection::mask once per
// packet, synchronously (transmit.rs:713-719, recv.rs:416-421). A kernel launch per call costs
// 30-40 us (r02), so per-packet calls go to one resident workgroup per device that polls this
// mailbox.
//
// r03 v2: the request HEADER travels in the poll itself. It is 64 stamped slots {word, sequence
// number}, each written by the host with one 8-B store and read by one lane of the polling wave
// with one 8-B load, so a slot is never torn; a request is complete when every slot it uses
// carries its number. The host writes the packet (and for AES-128-GCM the GHASH powers) first and
// slot 0 last, so once the kernel has seen the complete header, its loads of the packet see the
// packet — and they overlap the work that needs only the header (keystream, the one-time key, the
// powers of r, E_K(J0)). r03 v1 polled a sequence number and then loaded request and packet in a
// second PCIe round trip (2.8 us) before any work.
#pragma once
#include <stdint.h>

namespace mq {

constexpr uint32_t kResMaxPkt = 16 * 1024 + 256;  // aad + body + tag of one call (TLS records fit)

enum ResOp : uint32_t { kResSeal = 0, kResOpen = 1, kResHp = 2 };
enum ResState : uint32_t { kResExited = 0, kResRunning = 1, kResExiting = 2 };
// phases of a request (ResCtl::phase, diagnostic): header seen -> broadcast to the workgroup,
// first half of the work (needs only the header), packet landed in LDS, second half (seal: cipher
// and MAC, open: MAC and verdict), decryption applied (open), written back (before `done`)
constexpr int kResPhases = 6;

// header words (slot i carries word i)
enum ResHdrWord : uint32_t {
  kHwOp = 0,       // op | suite << 8
  kHwAad = 1,      // AAD bytes
  kHwBody = 2,     // body bytes: plaintext (seal) / ciphertext || tag (open)
  kHwPay = 3,      // data offset of the body: AAD rounded up to 16 B
  kHwNonce = 4,    // 3 words, the 12-B nonce as little-endian words
  kHwSample = 8,   // 4 words, the header-protection sample (little-endian words)
  kHwKey = 12,     // key material, 16-B aligned in LDS: ChaCha20 key (8 words: AEAD key, or the
                   // HP key for kResHp); AES-128 round keys (44 words, FIPS-197 big-endian; HP
                   // key's for kResHp)
  kHwStop = 56,    // host: 1 = leave now (process exit); its stamp is never checked
};
constexpr int kResHdrSlots = 64;  // slots 57..63 unused (lanes 57..63 of a poll read the stop slot)
constexpr uint32_t kSuiteAesRes = 1;  // MQ_SUITE_AES128GCM (include/mq_aead.h)
__host__ __device__ constexpr uint32_t res_hdr_words(uint32_t suite) {
  return kHwKey + (suite == kSuiteAesRes ? 44u : 8u);
}

// device -> host control words, each group on its own 64-B line
struct alignas(64) ResCtl {
  // one 16-B store per request (a single PCIe write: the host sees all four words or none)
  uint32_t done;          // number of the latest request served
  uint32_t status;        // MQ_* of that request
  uint32_t mask0, mask1;  // header-protection mask (kResHp)
  uint32_t phase[kResPhases];  // wall-clock ticks of the last request's phases (diagnostic)
  uint32_t pad1[12 - kResPhases];
  uint32_t state;         // ResState (host sets kResRunning before a launch)
  uint32_t pad2[15];
};

struct ResArea {
  uint64_t hdr[kResHdrSlots];          // host -> device: word | sequence number << 32
  ResCtl ctl;                          // device -> host
  alignas(64) uint32_t Hpow[64][4];    // AES-128-GCM: GHASH H^1 .. H^64 (BE words), read after the header
  alignas(64) uint8_t data[kResMaxPkt];  // aad, then the body at pay_off (|| room for the tag)
};

// the host's image of a context's request: key material filled once, op / lengths / nonce /
// sample per call (mq_host.cpp); mq_resident_call turns it into header slots
struct ResReq {
  uint32_t op, suite, aad_len, body_len;
  uint32_t nonce[3];
  uint32_t sample[4];
  uint32_t key[8];       // ChaCha20 AEAD key (LE words)
  uint32_t hp[8];        // ChaCha20 HP key (LE words)
  uint32_t aes_rk[44];   // AES-128 round keys, AEAD key (FIPS-197 BE words)
  uint32_t hp_rk[44];    // AES-128 round keys, HP key
  uint32_t Hpow[64][4];  // GHASH H^1 .. H^64 (BE words)
};

}  // namespace mq
