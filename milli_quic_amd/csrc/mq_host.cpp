// mq_host.cpp — C ABI of libmq_aead.so (include/mq_aead.h).
//
// Host side of the drop-in boundary: key contexts (CryptoProvider::aead/header_protection,
// reference src/crypto/rustcrypto.rs:225-287), per-packet Aead/HeaderProtection calls that run
// the HIP kernels on a batch of one, the HKDF/QUIC key schedule (src/crypto/key_schedule.rs),
// device key tables and the stream-ordered batch API. No CPU fallback exists for any
// cryptographic transform on packets: without a gfx950 device the calls fail with
// MQ_ERR_NO_DEVICE.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "mq_device.h"
#include "mq_opts.h"
#include "mq_resident.h"
#include "mq_runtime.h"

using mq::KeyRow;

int mq_chacha_flat_kind(uint64_t bpp);  // mq_chacha.hip
int mq_aes_flat_lanes(uint64_t bpp);    // mq_aes.hip

// ---- diagnostic switches (mq_opts.h) ---------------------------------------------------------
namespace {
const char* const kOptNames[(int)mq::Opt::Count] = {
    "MQ_CC_NARROW", "MQ_CC_LONG",  "MQ_CC_LIST",           "MQ_HP_FORK", "MQ_AES_SEG",
    "MQ_PROTECT_FUSED", "MQ_RESIDENT", "MQ_RESIDENT_TIMEOUT_US", "MQ_RECV_SEG", "MQ_AES_HOT_SEG", "MQ_AES_NARROW"};
std::atomic<long> g_opts[(int)mq::Opt::Count];
std::once_flag g_opts_once;
void opts_init() {  // once: the environment's values (shell-driven diagnostics keep working)
  std::call_once(g_opts_once, [] {
    for (int k = 0; k < (int)mq::Opt::Count; ++k) {
      const char* e = std::getenv(kOptNames[k]);
      long v = -1;
      if (e && *e) {
        char* end = nullptr;
        v = std::strtol(e, &end, 10);
        if (end == e || v < 0) v = -1;  // not a number: unset
      }
      g_opts[k].store(v, std::memory_order_relaxed);
    }
  });
}
}  // namespace

long mq::opt(mq::Opt o) {
  opts_init();
  return g_opts[(int)o].load(std::memory_order_relaxed);
}

extern "C" int mq_debug_option(const char* name, long value) {
  if (!name) return MQ_ERR_INVALID_ARG;
  opts_init();
  for (int k = 0; k < (int)mq::Opt::Count; ++k)
    if (std::strcmp(name, kOptNames[k]) == 0) {
      g_opts[k].store(value < 0 ? -1 : value, std::memory_order_relaxed);
      return MQ_OK;
    }
  return MQ_ERR_INVALID_ARG;
}

extern "C" int mq_debug_chacha_flat_kind(uint64_t arena_len, uint32_t n, uint32_t suite_hint) {
  const uint64_t len_hint = suite_hint >> 16;
  if (n == 0) return -1;
  return mq_chacha_flat_kind(len_hint ? len_hint : (arena_len + n - 1) / n);
}

extern "C" int mq_debug_aes_flat_kind(uint64_t arena_len, uint32_t n, uint32_t suite_hint) {
  const uint64_t len_hint = suite_hint >> 16;
  if (n == 0) return -1;
  return mq_aes_flat_lanes(len_hint ? len_hint : (arena_len + n - 1) / n);
}

extern "C" long mq_debug_option_get(const char* name) {
  if (!name) return -2;
  for (int k = 0; k < (int)mq::Opt::Count; ++k)
    if (std::strcmp(name, kOptNames[k]) == 0) return mq::opt((mq::Opt)k);
  return -2;
}

// launchers defined in the .hip translation units
hipError_t mq_launch_chacha(bool open, const KeyRow* kt, uint32_t n_rows, uint8_t* arena,
                            uint64_t arena_len, const mq_pkt_desc* desc, uint32_t n,
                            const uint32_t* index, const uint32_t* n_dev, uint8_t* status,
                            uint64_t* pn_out, uint2* hpm, bool own_hp, hipStream_t s, int cus, uint32_t* sched,
                            int64_t single_row, bool persistent, const uint32_t* reg, uint64_t bpp);
const uint32_t* mq_partition_regions(const uint32_t* counts);
hipError_t mq_launch_chacha_hp(const KeyRow* kt, uint32_t n_rows, const uint32_t* key_ids,
                               const uint8_t* samples, uint8_t* masks, uint32_t n, hipStream_t s);
hipError_t mq_launch_aes(bool open, const KeyRow* kt, uint32_t n_rows, uint8_t* arena,
                         uint64_t arena_len, const mq_pkt_desc* desc, uint32_t n,
                         const uint32_t* index, const uint32_t* n_dev, const uint32_t* hot,
                         uint8_t* status, uint64_t* pn_out, uint2* hpm, bool own_hp, hipStream_t s,
                         hipStream_t hot_stream, int cus, const uint32_t* rowseg, uint32_t* sched_s,
                         uint32_t* sched_hs, uint64_t bpp = 0);
const uint32_t* mq_partition_rowseg(uint32_t n, uint32_t n_rows, const uint32_t* counts);
hipError_t mq_launch_mixed_open_hp(const KeyRow* kt, uint32_t n_rows, const uint8_t* arena, uint64_t arena_len,
                                   const mq_pkt_desc* desc, uint32_t n, uint2* hpm, hipStream_t s);
hipError_t mq_launch_aes_hp(const KeyRow* kt, uint32_t n_rows, const uint32_t* key_ids,
                            const uint8_t* samples, uint8_t* masks, uint32_t n, hipStream_t s);
hipError_t mq_launch_partition(const KeyRow* kt, uint32_t n_rows, const mq_pkt_desc* desc, uint32_t n,
                               uint32_t* list, uint32_t* codes, uint32_t* counts, hipStream_t s, bool skip_unkeyed,
                               const uint32_t* live);
size_t mq_partition_workspace(uint32_t n);
void mq_partition_layout(uint32_t n, size_t* codes_off, size_t* counts_off);
uint32_t mq_partition_list_cap(uint32_t n);
hipError_t mq_launch_derive_initial(const mq::MQDeriveConsts& k, const uint8_t* dcids, const uint8_t* dcid_lens,
                                    uint32_t n, KeyRow* rows, mq_key_material* km_out, uint8_t* status,
                                    hipStream_t s);
hipError_t mq_launch_build(const KeyRow* kt, uint32_t n_rows, const mq_conn_send* conns, uint32_t n_conns,
                           const uint8_t* frames, uint64_t frames_len, uint8_t* out, uint64_t out_len,
                           const mq_send_req* req, uint32_t n, mq_pkt_desc* desc, uint8_t* bstatus,
                           uint32_t* pkt_len, uint32_t suite_hint, hipStream_t s);
hipError_t mq_launch_send_status(const uint8_t* bstatus, uint8_t* status, uint32_t n, hipStream_t s);
hipError_t mq_launch_chacha_protect(const KeyRow* kt, uint32_t n_rows, const mq_conn_send* conns, uint32_t n_conns,
                                    const uint8_t* frames, uint64_t frames_len, uint8_t* out, uint64_t out_len,
                                    const mq_send_req* req, uint32_t n, uint32_t suite_hint, uint8_t* status,
                                    uint32_t* pkt_len, hipStream_t s);
size_t mq_recv_workspace(uint32_t n_dgrams, uint32_t max_pkts, uint32_t n_conns, size_t open_ws_bytes);
void mq_recv_trace(const char* what, uint32_t n_dgrams, uint32_t max_pkts, uint32_t n_conns, void* ws_ptr,
                   size_t open_ws_bytes, uint32_t seg, hipStream_t s);
uint32_t mq_recv_seg_len();
hipError_t mq_recv_front(const KeyRow* kt, uint32_t n_rows, mq_conn_recv* conns, uint32_t n_conns, uint8_t* arena,
                         uint64_t arena_len, const mq_dgram* dg, uint32_t n_dgrams, uint32_t max_pkts,
                         uint32_t* n_pkts, mq_recv_pkt* out, void* ws_ptr, size_t open_ws_bytes, mq::MQRecvPass* pass,
                         uint32_t seg, hipStream_t s);
hipError_t mq_recv_walk(const KeyRow* kt, uint32_t n_rows, mq_conn_recv* conns, uint32_t n_conns,
                        uint32_t n_dgrams, uint32_t max_pkts, mq_recv_pkt* out, void* ws_ptr, size_t open_ws_bytes,
                        bool final_walk, bool verify, uint32_t walk_idx, uint32_t seg, hipStream_t s);
hipError_t mq_recv_retry(uint32_t n_dgrams, uint32_t max_pkts, uint32_t n_conns, void* ws_ptr, size_t open_ws_bytes,
                         hipStream_t s);
hipError_t mq_recv_outcomes(uint32_t n_dgrams, uint32_t max_pkts, uint32_t n_conns, void* ws_ptr,
                            size_t open_ws_bytes, hipStream_t s);
hipError_t mq_launch_record_inner(const uint8_t* arena, uint64_t arena_len, const mq_pkt_desc* desc, uint32_t n,
                                  uint8_t* status, uint64_t* info, hipStream_t s);
int mq_resident_call(int dev, const mq::ResReq& q, uint64_t uid, const uint8_t* aad, const uint8_t* body, uint8_t* out,
                     size_t out_off, size_t out_len, int* status, uint32_t* mask);
#ifdef MQ_STAMPS
void mq_stamps_set_chacha(uint64_t* p);
void mq_stamps_set_aes(uint64_t* p);
void mq_stamps_set_part(uint64_t* p);
#endif

namespace {

// ---------------------------------------------------------------------------------------------
// device selection (per thread) and side streams (per device and caller stream): mq_runtime.h
struct HipBackend {
  typedef hipStream_t Stream;
  typedef hipEvent_t Event;
  static int count() {
    int n = 0;
    return hipGetDeviceCount(&n) == hipSuccess ? n : 0;
  }
  static bool usable(int dev) {
    hipDeviceProp_t prop;
    return hipGetDeviceProperties(&prop, dev) == hipSuccess && std::strncmp(prop.gcnArchName, "gfx950", 6) == 0;
  }
  static int cus(int dev) {
    int v = 0;
    return hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess ? v : 0;
  }
  static int get() {
    int d = -1;
    return hipGetDevice(&d) == hipSuccess ? d : -1;
  }
  static bool set(int dev) { return hipSetDevice(dev) == hipSuccess; }
  static bool stream_create(Stream* s) { return hipStreamCreateWithFlags(s, hipStreamNonBlocking) == hipSuccess; }
  static void stream_destroy(Stream s) {
    (void)hipStreamSynchronize(s);
    (void)hipStreamDestroy(s);
  }
  static bool event_create(Event* e) { return hipEventCreateWithFlags(e, hipEventDisableTiming) == hipSuccess; }
  static void event_destroy(Event e) { (void)hipEventDestroy(e); }
  static bool record(Event e, Stream s) { return hipEventRecord(e, s) == hipSuccess; }
  static bool wait(Stream s, Event e) { return hipStreamWaitEvent(s, e, 0) == hipSuccess; }
  static void* alloc_zeroed(size_t bytes) {
    void* p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess) return nullptr;
    if (hipMemset(p, 0, bytes) != hipSuccess || hipDeviceSynchronize() != hipSuccess) return nullptr;  // leaked
    return p;
  }
  static void stream_sync(Stream s) { (void)hipStreamSynchronize(s); }
};
typedef mq::DeviceRegistry<HipBackend> Devices;
typedef Devices::Guard DeviceGuard;
// Constructed on first use and never destroyed: side streams and device state may be touched from
// other libraries' static destructors, after which the HIP runtime may already be gone.
Devices& devices() {
  static Devices* d = new Devices();
  return *d;
}
// Dynamic tile schedule slots of the persistent AES kernels, per (device, stream): mq_runtime.h,
// mq_tile.h TileSched. MQ_SCHED=0 (diagnostic) selects the static stride.
mq::SchedSlots<HipBackend>& sched_slots() {
  static auto* s = new mq::SchedSlots<HipBackend>(1024, mq::kSchedSlotBytes);
  return *s;
}
// Side streams hand their schedule slots back when their entry goes (evicted or released), so a
// server that keeps creating and dropping caller streams never runs out of slots.
mq::SideStreams<HipBackend>& side_streams() {
  static auto* s = new mq::SideStreams<HipBackend>(64, [](hipStream_t side) { sched_slots().release(side); });
  return *s;
}
uint32_t* sched_slot(int dev, hipStream_t s) {
  static const bool on = [] {
#ifdef MQ_SCHED_STATIC  // diagnostic builds (tools/build_variant.sh)
    return false;
#endif
    const char* e = std::getenv("MQ_SCHED");
    return !(e && e[0] == '0');
  }();
  if (!on) return nullptr;
  // A slot assumes that kernels on its handle never overlap. Two handles break that:
  // hipStreamPerThread is one value naming a different stream on every host thread, and the legacy
  // handle is shared in the same way; and a stream under capture records kernels into a graph that
  // may be replayed concurrently or on another stream. Those launches take the static stride.
  if (s == hipStreamPerThread || s == hipStreamLegacy) return nullptr;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
  return (uint32_t*)sched_slots().get(dev, s);
}

// The device a new object (key table, AEAD / HP context) is created on: the thread's selection,
// else its current HIP device; -1 (MQ_ERR_NO_DEVICE) when that is not a gfx950.
int creation_device() { return devices().current(); }

// Forked tile kernels: MQ_FORK=0 runs every kernel of a batch on the caller's stream (diagnostic)
bool fork_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("MQ_FORK");
    return !(e && e[0] == '0');
  }();
  return on;
}


// ---------------------------------------------------------------------------------------------
// AES-128 key expansion / block encryption (FIPS-197), host side: the reference computes the
// key schedule and GHASH H once at construction (rustcrypto.rs:232-252); so does the key table.
uint8_t g_sbox[256];
std::once_flag g_sbox_once;

uint8_t gmul(uint8_t a, uint8_t b) {
  uint8_t r = 0;
  while (b) {
    if (b & 1) r ^= a;
    a = (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0));
    b >>= 1;
  }
  return r;
}

void init_sbox() {
  // walk the multiplicative group with generator 3 to get inverses, then the affine map
  uint8_t p = 1, qv = 1;
  do {
    p = (uint8_t)(p ^ (p << 1) ^ ((p & 0x80) ? 0x1b : 0));
    qv ^= (uint8_t)(qv << 1); qv ^= (uint8_t)(qv << 2); qv ^= (uint8_t)(qv << 4);
    if (qv & 0x80) qv ^= 0x09;
    const uint8_t x = (uint8_t)(qv ^ ((qv << 1) | (qv >> 7)) ^ ((qv << 2) | (qv >> 6)) ^
                                ((qv << 3) | (qv >> 5)) ^ ((qv << 4) | (qv >> 4)));
    g_sbox[p] = x ^ 0x63;
  } while (p != 1);
  g_sbox[0] = 0x63;
}

const uint8_t* sbox() {
  std::call_once(g_sbox_once, init_sbox);
  return g_sbox;
}

uint32_t be32(const uint8_t* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}
uint32_t le32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

void aes_expand(const uint8_t key[16], uint32_t rk[44]) {
  const uint8_t* S = sbox();
  uint8_t rcon = 1;
  for (int i = 0; i < 4; ++i) rk[i] = be32(key + 4 * i);
  for (int i = 4; i < 44; ++i) {
    uint32_t t = rk[i - 1];
    if (i % 4 == 0) {
      t = (t << 8) | (t >> 24);
      t = ((uint32_t)S[t >> 24] << 24) | ((uint32_t)S[(t >> 16) & 0xff] << 16) |
          ((uint32_t)S[(t >> 8) & 0xff] << 8) | S[t & 0xff];
      t ^= (uint32_t)rcon << 24;
      rcon = gmul(rcon, 2);
    }
    rk[i] = rk[i - 4] ^ t;
  }
}

void aes_encrypt(const uint32_t rk[44], const uint8_t in[16], uint8_t out[16]) {
  const uint8_t* S = sbox();
  uint8_t s[16], t[16];
  for (int c = 0; c < 4; ++c) {
    uint32_t w = be32(in + 4 * c) ^ rk[c];
    s[4 * c] = (uint8_t)(w >> 24); s[4 * c + 1] = (uint8_t)(w >> 16);
    s[4 * c + 2] = (uint8_t)(w >> 8); s[4 * c + 3] = (uint8_t)w;
  }
  for (int r = 1; r <= 10; ++r) {
    for (int c = 0; c < 4; ++c)
      for (int i = 0; i < 4; ++i) t[4 * c + i] = S[s[4 * ((c + i) & 3) + i]];
    if (r < 10) {
      for (int c = 0; c < 4; ++c) {
        const uint8_t a0 = t[4 * c], a1 = t[4 * c + 1], a2 = t[4 * c + 2], a3 = t[4 * c + 3];
        s[4 * c] = gmul(a0, 2) ^ gmul(a1, 3) ^ a2 ^ a3;
        s[4 * c + 1] = a0 ^ gmul(a1, 2) ^ gmul(a2, 3) ^ a3;
        s[4 * c + 2] = a0 ^ a1 ^ gmul(a2, 2) ^ gmul(a3, 3);
        s[4 * c + 3] = gmul(a0, 3) ^ a1 ^ a2 ^ gmul(a3, 2);
      }
    } else {
      std::memcpy(s, t, 16);
    }
    for (int c = 0; c < 4; ++c) {
      const uint32_t k = rk[4 * r + c];
      s[4 * c] ^= (uint8_t)(k >> 24); s[4 * c + 1] ^= (uint8_t)(k >> 16);
      s[4 * c + 2] ^= (uint8_t)(k >> 8); s[4 * c + 3] ^= (uint8_t)k;
    }
  }
  std::memcpy(out, s, 16);
}

// GF(2^128) product in GCM bit order (SP 800-38D Alg. 1)
void gf128_mul(const uint8_t x[16], const uint8_t y[16], uint8_t out[16]) {
  uint8_t z[16] = {0}, v[16];
  std::memcpy(v, y, 16);
  for (int i = 0; i < 128; ++i) {
    if ((x[i >> 3] >> (7 - (i & 7))) & 1)
      for (int k = 0; k < 16; ++k) z[k] ^= v[k];
    const int lsb = v[15] & 1;
    for (int k = 15; k > 0; --k) v[k] = (uint8_t)((v[k] >> 1) | (v[k - 1] << 7));
    v[0] >>= 1;
    if (lsb) v[0] ^= 0xe1;
  }
  std::memcpy(out, z, 16);
}

size_t suite_key_len(uint32_t suite) {
  return suite == MQ_SUITE_AES128GCM ? 16 : suite == MQ_SUITE_CHACHA20 ? 32 : 0;
}

// Build one device row from host key material. Returns false on a bad suite.
bool build_row(const mq_key_material& km, KeyRow& row) {
  std::memset(&row, 0, sizeof row);
  if (!suite_key_len(km.suite)) return false;
  row.suite = km.suite;
  for (int i = 0; i < 3; ++i) row.iv[i] = le32(km.iv + 4 * i);
  for (int i = 0; i < 8; ++i) row.key[i] = le32(km.key + 4 * i);
  for (int i = 0; i < 8; ++i) row.hp[i] = le32(km.hp + 4 * i);
  if (km.suite == MQ_SUITE_AES128GCM) {
    aes_expand(km.key, row.aes_rk);
    aes_expand(km.hp, row.hp_rk);
    uint8_t h[8][16], zero[16] = {0};
    aes_encrypt(row.aes_rk, zero, h[0]);  // H = E_K(0^128), then H^2..H^8
    for (int p = 1; p < 8; ++p) gf128_mul(h[p - 1], h[0], h[p]);
    for (int p = 0; p < 8; ++p)
      for (int w = 0; w < 4; ++w) row.H[p][w] = be32(h[p] + 4 * w);
  }
  return true;
}

// ---------------------------------------------------------------------------------------------
// SHA-256 / HMAC / HKDF (FIPS 180-4, RFC 2104, RFC 5869): Hkdf trait, rustcrypto.rs:9-24
const uint32_t kK256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

struct Sha256 {
  uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                   0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  uint8_t buf[64];
  size_t fill = 0;
  uint64_t total = 0;

  static uint32_t ror(uint32_t x, int r) { return (x >> r) | (x << (32 - r)); }
  void block(const uint8_t* p) {
    uint32_t w[64];
    for (int i = 0; i < 16; ++i) w[i] = be32(p + 4 * i);
    for (int i = 16; i < 64; ++i)
      w[i] = w[i - 16] + (ror(w[i - 15], 7) ^ ror(w[i - 15], 18) ^ (w[i - 15] >> 3)) + w[i - 7] +
             (ror(w[i - 2], 17) ^ ror(w[i - 2], 19) ^ (w[i - 2] >> 10));
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
    for (int i = 0; i < 64; ++i) {
      const uint32_t t1 = hh + (ror(e, 6) ^ ror(e, 11) ^ ror(e, 25)) + ((e & f) ^ (~e & g)) + kK256[i] + w[i];
      const uint32_t t2 = (ror(a, 2) ^ ror(a, 13) ^ ror(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
      hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
  }
  void update(const uint8_t* p, size_t n) {
    total += n;
    while (n) {
      const size_t k = std::min(n, (size_t)64 - fill);
      std::memcpy(buf + fill, p, k);
      fill += k; p += k; n -= k;
      if (fill == 64) { block(buf); fill = 0; }
    }
  }
  void final(uint8_t out[32]) {
    const uint64_t bits = total * 8;
    const uint8_t one = 0x80, zero = 0;
    update(&one, 1);
    while (fill != 56) update(&zero, 1);
    uint8_t len[8];
    for (int i = 0; i < 8; ++i) len[i] = (uint8_t)(bits >> (56 - 8 * i));
    update(len, 8);
    for (int i = 0; i < 8; ++i) {
      out[4 * i] = (uint8_t)(h[i] >> 24); out[4 * i + 1] = (uint8_t)(h[i] >> 16);
      out[4 * i + 2] = (uint8_t)(h[i] >> 8); out[4 * i + 3] = (uint8_t)h[i];
    }
  }
};

void hmac_sha256(const uint8_t* key, size_t key_len, const uint8_t* m1, size_t l1, const uint8_t* m2,
                 size_t l2, const uint8_t* m3, size_t l3, uint8_t out[32]) {
  uint8_t k[64] = {0}, pad[64], inner[32];
  if (key_len > 64) { Sha256 s; s.update(key, key_len); s.final(k); }
  else std::memcpy(k, key, key_len);
  Sha256 si, so;
  for (int i = 0; i < 64; ++i) pad[i] = k[i] ^ 0x36;
  si.update(pad, 64); si.update(m1, l1); si.update(m2, l2); si.update(m3, l3); si.final(inner);
  for (int i = 0; i < 64; ++i) pad[i] = k[i] ^ 0x5c;
  so.update(pad, 64); so.update(inner, 32); so.final(out);
}

// ---------------------------------------------------------------------------------------------
// Scratch of the per-packet (batch of one) calls: [row][desc 32][status 16][pn 8][pad][packet ...]
// in pinned host memory. Zero-copy (default): the buffer is mapped into the device's address
// space and the kernel reads and writes it over PCIe directly — a call is one kernel launch and
// one stream sync, no copies. MQ_PER_PACKET_COPY=1 selects the copy path instead (a device mirror,
// H2D before and D2H after the kernel), kept for comparison (tools/bench_latency.py).
struct Scratch {
  int device = -1;          // the owning context's device (every call runs there)
  hipStream_t stream = nullptr;
  uint8_t* dev = nullptr;   // what the kernel addresses: device mirror, or the mapped host buffer
  uint8_t* host = nullptr;  // pinned host buffer
  size_t cap = 0;
  bool zero_copy = true;
  std::mutex mu;

  static constexpr size_t kDesc = sizeof(KeyRow);  // descriptor (AEAD) / key id (HP)
  static constexpr size_t kStatus = kDesc + 32;     // status (AEAD) / mask (HP)
  static constexpr size_t kPn = kStatus + 16;       // decoded pn (AEAD)
  static constexpr size_t kSample = kDesc + 16;     // HP sample
  static constexpr size_t kHdr = 1024;              // the packet
  static_assert(kPn + 8 <= kHdr && kPn % 8 == 0, "scratch header layout");

  void release() {
    if (dev && !zero_copy) (void)hipFree(dev);
    if (host) (void)hipHostFree(host);
    dev = nullptr; host = nullptr; cap = 0;
  }
  int ensure(size_t pkt_bytes) {
    const size_t need = kHdr + ((pkt_bytes + 255) & ~(size_t)255) + 256;
    if (!stream) {
      if (hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) != hipSuccess) return MQ_ERR_HIP;
      const char* e = std::getenv("MQ_PER_PACKET_COPY");
      zero_copy = !(e && e[0] == '1');
    }
    if (need <= cap) return MQ_OK;
    release();
    if (zero_copy) {
      if (hipHostMalloc(&host, need, hipHostMallocMapped) != hipSuccess) return MQ_ERR_HIP;
      if (hipHostGetDevicePointer((void**)&dev, host, 0) != hipSuccess) { release(); return MQ_ERR_HIP; }
    } else {
      if (hipMalloc(&dev, need) != hipSuccess) return MQ_ERR_HIP;
      if (hipHostMalloc(&host, need, hipHostMallocDefault) != hipSuccess) { release(); return MQ_ERR_HIP; }
    }
    cap = need;
    return MQ_OK;
  }
  // host -> what the kernel reads (no-op when zero-copy)
  int upload(size_t bytes) {
    if (zero_copy) return MQ_OK;
    return hipMemcpyAsync(dev, host, bytes, hipMemcpyHostToDevice, stream) == hipSuccess ? MQ_OK : MQ_ERR_HIP;
  }
  // [off, off + bytes) back to the host buffer (no-op when zero-copy), then wait for the stream
  int finish(size_t off, size_t bytes) {
    if (!zero_copy && hipMemcpyAsync(host + off, dev + off, bytes, hipMemcpyDeviceToHost, stream) != hipSuccess)
      return MQ_ERR_HIP;
    return hipStreamSynchronize(stream) == hipSuccess ? MQ_OK : MQ_ERR_HIP;
  }
  ~Scratch() {
    if (!stream && !host) return;
    DeviceGuard g(device);
    release();
    if (stream) (void)hipStreamDestroy(stream);
  }
};

// Run one packet through the seal/open kernel of `row.suite`. The packet is aad || body, where
// body = `body_len` bytes of buf (plaintext for seal, ciphertext || tag for open), staged straight
// into the pinned scratch (no heap allocation per call); `pkt_len` = aad_len + body_len (+ 16 on
// seal: the tag area). Descriptor in NO_HP mode with pn = 0 (the caller's nonce sits in row.iv).
// On MQ_OK the transformed body (`out_len` bytes) is copied back into buf. Runs on the scratch's
// (its context's) device.
int run_one(Scratch& sc, const KeyRow& row, const uint8_t* aad, uint32_t aad_len, uint8_t* buf,
            uint32_t body_len, uint32_t pkt_len, uint32_t out_len, bool open) {
  DeviceGuard g(sc.device);
  if (!g.ok()) return MQ_ERR_NO_DEVICE;
  int rc = sc.ensure(pkt_len);
  if (rc) return rc;
  std::memcpy(sc.host, &row, sizeof row);
  mq_pkt_desc d;
  std::memset(&d, 0, sizeof d);
  d.offset = Scratch::kHdr;
  d.len = pkt_len;
  d.key_id = 0;
  d.pn = 0;
  d.pn_offset = (uint16_t)aad_len;
  d.pn_len = 0;
  d.flags = MQ_PKT_NO_HP;
  std::memcpy(sc.host + Scratch::kDesc, &d, sizeof d);
  std::memset(sc.host + Scratch::kStatus, 0xff, 16);
  uint8_t* pkt = sc.host + Scratch::kHdr;
  if (aad_len) std::memcpy(pkt, aad, aad_len);
  std::memcpy(pkt + aad_len, buf, body_len);
  if (pkt_len > aad_len + body_len) std::memset(pkt + aad_len + body_len, 0, pkt_len - aad_len - body_len);
  const size_t bytes = Scratch::kHdr + pkt_len;
  if ((rc = sc.upload(bytes)) != MQ_OK) return rc;
  const KeyRow* kt = (const KeyRow*)sc.dev;
  const mq_pkt_desc* dd = (const mq_pkt_desc*)(sc.dev + Scratch::kDesc);
  uint8_t* st = sc.dev + Scratch::kStatus;
  uint64_t* pn = (uint64_t*)(sc.dev + Scratch::kPn);
  // the arena is the whole scratch buffer; the packet sits at offset kHdr. NO_HP: no header
  // protection pass to launch (own_hp false)
  hipError_t e = row.suite == MQ_SUITE_CHACHA20
                     ? mq_launch_chacha(open, kt, 1, sc.dev, bytes, dd, 1, nullptr, nullptr, st, pn, nullptr, false, sc.stream,
                                        0, nullptr, -1, false, nullptr, bytes)
                     : mq_launch_aes(open, kt, 1, sc.dev, bytes, dd, 1, nullptr, nullptr, nullptr, st, pn, nullptr, false,
                                     sc.stream, sc.stream, devices().cus(sc.device), nullptr, nullptr, nullptr);
  if (e != hipSuccess) return MQ_ERR_HIP;
  // status and the transformed packet in one read-back (the status sits before the packet)
  if ((rc = sc.finish(Scratch::kStatus, Scratch::kHdr - Scratch::kStatus + pkt_len)) != MQ_OK) return rc;
  const int status = sc.host[Scratch::kStatus];
  if (status == MQ_OK) std::memcpy(buf, pkt + aad_len, out_len);
  return status;
}

// Per-packet calls go to the device's resident kernel (mq_resident.hip: no launch per call) unless
// MQ_RESIDENT=0 or the packet exceeds its buffer; then run_one's batch of one.
bool resident_enabled(size_t bytes) {
  // tests and tools/bench_latency.py switch it (mq_debug_option)
  return mq::opt(mq::Opt::Resident) != 0 && bytes + 31 <= mq::kResMaxPkt;  // + the body's alignment pad and the tag
}

// The resident request image of a context: suite and key material (and for AES-128-GCM the GHASH
// powers H^1..H^64 of its 64-lane Horner), filled once at creation; `uid` names the context to the
// mailbox (its GHASH powers are copied there only when another context used it last).
std::atomic<uint64_t> g_res_uid{0};
mq::ResReq* res_image(const KeyRow& row, bool aead, uint64_t& uid) {
  uid = ++g_res_uid;
  mq::ResReq* q = new mq::ResReq();
  std::memset(q, 0, sizeof *q);
  q->suite = row.suite;
  std::memcpy(q->key, row.key, sizeof q->key);
  std::memcpy(q->hp, row.hp, sizeof q->hp);
  std::memcpy(q->aes_rk, row.aes_rk, sizeof q->aes_rk);
  std::memcpy(q->hp_rk, row.hp_rk, sizeof q->hp_rk);
  if (aead && row.suite == MQ_SUITE_AES128GCM) {
    uint8_t h[16], x[16], zero[16] = {0};
    aes_encrypt(row.aes_rk, zero, h);  // H = E_K(0^128)
    std::memcpy(x, h, 16);
    for (int p = 0; p < 64; ++p) {
      for (int w = 0; w < 4; ++w) q->Hpow[p][w] = be32(x + 4 * w);
      uint8_t y[16];
      gf128_mul(x, h, y);
      std::memcpy(x, y, 16);
    }
  }
  return q;
}

}  // namespace

// =============================================================================================
// opaque handle definitions
struct mq_aead_ctx {
  uint32_t suite;
  KeyRow row;  // key schedule, H powers; iv is overwritten by the per-call nonce
  mutable Scratch sc;
  mq::ResReq* res = nullptr;  // resident request image (mutated per call under sc.mu)
  uint64_t res_uid = 0;
  ~mq_aead_ctx() { delete res; }
};
struct mq_hp_ctx {
  uint32_t suite;
  KeyRow row;
  mutable Scratch sc;
  mq::ResReq* res = nullptr;
  uint64_t res_uid = 0;
  ~mq_hp_ctx() { delete res; }
};
struct mq_keytable {
  KeyRow* dev = nullptr;
  uint32_t rows = 0;
  int device = -1;  // where the rows live; every batch call on this table runs there
  // host view of the rows' suites (as last written by mq_keytable_update; a device-side write —
  // mq_batch_derive_initial — only turns rows into AES-128-GCM ones, so the count of non-AES rows
  // is never underestimated): a table with ONE non-AES row puts every packet of a mixed batch's
  // second list on that row, and the ChaCha20 list kernels take the single-key path
  std::vector<uint8_t> suite;
  uint32_t non_aes = 0;
  bool derived = false;  // rows written on the device (their suites unknown here): no single-key path
  int64_t single_row() const {
    if (derived || non_aes != 1) return -1;
    for (uint32_t r = 0; r < rows; ++r)
      if (suite[r] != MQ_SUITE_AES128GCM) return r;
    return -1;
  }
};

// the host view of rows [first, first + n) after a write (suite_of(i): row first + i's new suite)
template <class F>
static void kt_mirror(mq_keytable* kt, uint32_t first, uint32_t n, F suite_of) {
  if (kt->suite.size() != kt->rows) {
    kt->suite.assign(kt->rows, 0);
    kt->non_aes = kt->rows;
  }
  for (uint32_t i = 0; i < n; ++i) {
    const uint8_t o = kt->suite[first + i], v = suite_of(i);
    kt->non_aes += (v != MQ_SUITE_AES128GCM) - (o != MQ_SUITE_AES128GCM);
    kt->suite[first + i] = v;
  }
}

extern "C" {

const char* mq_version(void) { return "mq_aead 0.2.0 (gfx950)"; }

int mq_device_init(int device) { return devices().select(device) ? MQ_OK : MQ_ERR_NO_DEVICE; }

int mq_device_current(void) { return devices().current(); }

int mq_keytable_device(const mq_keytable* kt) { return kt ? kt->device : -1; }

void mq_stream_release(void* stream) {
  side_streams().release((hipStream_t)stream);
  sched_slots().release((hipStream_t)stream);
}

const char* mq_status_str(int status) {
  switch (status) {
    case MQ_OK: return "ok";
    case MQ_ERR_CRYPTO: return "crypto";
    case MQ_ERR_BUFFER_TOO_SMALL: return "buffer too small";
    case MQ_ERR_INVALID_ARG: return "invalid argument";
    case MQ_ERR_PROTOCOL: return "protocol violation";
    case MQ_ERR_SUITE: return "suite mismatch";
    case MQ_ERR_NO_DEVICE: return "no gfx950 device";
    case MQ_ERR_HIP: return "hip runtime error";
    case MQ_ERR_TLS: return "tls";
    default: return "unknown";
  }
}

size_t mq_aead_key_len(uint32_t suite) { return suite_key_len(suite); }

int mq_aead_new(uint32_t suite, const uint8_t* key, size_t key_len, mq_aead_ctx** out) {
  if (!out) return MQ_ERR_INVALID_ARG;
  *out = nullptr;
  if (!suite_key_len(suite) || !key || key_len != suite_key_len(suite)) return MQ_ERR_CRYPTO;
  const int dev = creation_device();
  if (dev < 0) return MQ_ERR_NO_DEVICE;
  mq_key_material km;
  std::memset(&km, 0, sizeof km);
  km.suite = suite;
  std::memcpy(km.key, key, key_len);
  mq_aead_ctx* c = new mq_aead_ctx();
  c->sc.device = dev;
  c->suite = suite;
  build_row(km, c->row);
  c->res = res_image(c->row, true, c->res_uid);
  *out = c;
  return MQ_OK;
}

void mq_aead_free(mq_aead_ctx* ctx) { delete ctx; }

int mq_aead_seal_in_place(const mq_aead_ctx* ctx, const uint8_t* nonce, size_t nonce_len,
                          const uint8_t* aad, size_t aad_len, uint8_t* buf, size_t buf_len,
                          size_t payload_len, size_t* out_len, size_t* needed) {
  if (!ctx) return MQ_ERR_INVALID_ARG;
  if (!nonce || nonce_len != 12) return MQ_ERR_CRYPTO;  // rustcrypto.rs:48-50,120-122
  const size_t total = payload_len + 16;
  if (buf_len < total) {  // rustcrypto.rs:51-54,123-126
    if (needed) *needed = total;
    return MQ_ERR_BUFFER_TOO_SMALL;
  }
  if ((aad_len && !aad) || !buf || aad_len > 0xffff || aad_len + total > 0xffffffffu) return MQ_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(ctx->sc.mu);
  if (resident_enabled(aad_len + total)) {
    DeviceGuard g(ctx->sc.device);
    if (!g.ok()) return MQ_ERR_NO_DEVICE;
    mq::ResReq& q = *ctx->res;
    q.op = mq::kResSeal;
    q.aad_len = (uint32_t)aad_len;
    q.body_len = (uint32_t)payload_len;
    for (int i = 0; i < 3; ++i) q.nonce[i] = le32(nonce + 4 * i);
    int st = MQ_ERR_HIP;
    const int rc = mq_resident_call(ctx->sc.device, q, ctx->res_uid, aad, buf, buf, 0, total, &st, nullptr);
    if (rc) return rc;
    if (st) return st;
    if (out_len) *out_len = total;
    return MQ_OK;
  }
  KeyRow row = ctx->row;
  for (int i = 0; i < 3; ++i) row.iv[i] = le32(nonce + 4 * i);
  const int rc = run_one(ctx->sc, row, aad, (uint32_t)aad_len, buf, (uint32_t)payload_len,
                         (uint32_t)(aad_len + total), (uint32_t)total, false);
  if (rc) return rc;
  if (out_len) *out_len = total;
  return MQ_OK;
}

int mq_aead_open_in_place(const mq_aead_ctx* ctx, const uint8_t* nonce, size_t nonce_len,
                          const uint8_t* aad, size_t aad_len, uint8_t* buf, size_t buf_len,
                          size_t ct_len, size_t* out_len) {
  if (!ctx) return MQ_ERR_INVALID_ARG;
  if (!nonce || nonce_len != 12) return MQ_ERR_CRYPTO;  // rustcrypto.rs:75-77,146-148
  if (ct_len < 16) return MQ_ERR_CRYPTO;                // :78-80,149-151
  if (ct_len > buf_len) return MQ_ERR_INVALID_ARG;      // the reference panics (:83,154)
  if ((aad_len && !aad) || !buf || aad_len > 0xffff || aad_len + ct_len > 0xffffffffu) return MQ_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(ctx->sc.mu);
  if (resident_enabled(aad_len + ct_len)) {
    DeviceGuard g(ctx->sc.device);
    if (!g.ok()) return MQ_ERR_NO_DEVICE;
    mq::ResReq& q = *ctx->res;
    q.op = mq::kResOpen;
    q.aad_len = (uint32_t)aad_len;
    q.body_len = (uint32_t)ct_len;
    for (int i = 0; i < 3; ++i) q.nonce[i] = le32(nonce + 4 * i);
    int st = MQ_ERR_HIP;
    const int rc = mq_resident_call(ctx->sc.device, q, ctx->res_uid, aad, buf, buf, 0, ct_len - 16, &st, nullptr);
    if (rc) return rc;
    if (st) return st;  // buffer untouched on failure
    if (out_len) *out_len = ct_len - 16;
    return MQ_OK;
  }
  KeyRow row = ctx->row;
  for (int i = 0; i < 3; ++i) row.iv[i] = le32(nonce + 4 * i);
  const int rc = run_one(ctx->sc, row, aad, (uint32_t)aad_len, buf, (uint32_t)ct_len, (uint32_t)(aad_len + ct_len),
                         (uint32_t)(ct_len - 16), true);
  if (rc) return rc;  // buffer untouched on failure
  if (out_len) *out_len = ct_len - 16;
  return MQ_OK;
}

int mq_hp_new(uint32_t suite, const uint8_t* key, size_t key_len, mq_hp_ctx** out) {
  if (!out) return MQ_ERR_INVALID_ARG;
  *out = nullptr;
  const size_t want = suite == MQ_SUITE_AES128GCM ? 16 : suite == MQ_SUITE_CHACHA20 ? 32 : 0;
  if (!want || !key || key_len != want) return MQ_ERR_CRYPTO;  // rustcrypto.rs:247-249,280-282
  const int dev = creation_device();
  if (dev < 0) return MQ_ERR_NO_DEVICE;
  mq_key_material km;
  std::memset(&km, 0, sizeof km);
  km.suite = suite;
  std::memcpy(km.hp, key, key_len);
  if (suite == MQ_SUITE_AES128GCM) std::memset(km.key, 0, 16);
  mq_hp_ctx* c = new mq_hp_ctx();
  c->sc.device = dev;
  c->suite = suite;
  build_row(km, c->row);
  c->res = res_image(c->row, false, c->res_uid);
  *out = c;
  return MQ_OK;
}

void mq_hp_free(mq_hp_ctx* ctx) { delete ctx; }

int mq_hp_mask(const mq_hp_ctx* ctx, const uint8_t* sample, size_t sample_len, uint8_t mask[5]) {
  if (!ctx || !mask || !sample || sample_len < 16) return MQ_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(ctx->sc.mu);
  Scratch& sc = ctx->sc;
  DeviceGuard g(sc.device);
  if (!g.ok()) return MQ_ERR_NO_DEVICE;
  if (resident_enabled(0)) {
    mq::ResReq& q = *ctx->res;
    q.op = mq::kResHp;
    q.aad_len = q.body_len = 0;
    for (int i = 0; i < 4; ++i) q.sample[i] = le32(sample + 4 * i);
    int st = MQ_ERR_HIP;
    uint32_t m[2] = {0, 0};
    const int rc = mq_resident_call(sc.device, q, ctx->res_uid, nullptr, nullptr, nullptr, 0, 0, &st, m);
    if (rc) return rc;
    if (st) return st;
    for (int b = 0; b < 4; ++b) mask[b] = (uint8_t)(m[0] >> (8 * b));
    mask[4] = (uint8_t)m[1];
    return MQ_OK;
  }
  int rc = sc.ensure(64);
  if (rc) return rc;
  // layout: row | key id (4) @kDesc | sample 16 @kSample | mask 5 @kStatus
  std::memcpy(sc.host, &ctx->row, sizeof(KeyRow));
  const uint32_t kid = 0;
  std::memcpy(sc.host + Scratch::kDesc, &kid, 4);
  std::memcpy(sc.host + Scratch::kSample, sample, 16);
  std::memset(sc.host + Scratch::kStatus, 0, 8);
  if ((rc = sc.upload(Scratch::kStatus + 8)) != MQ_OK) return rc;
  const KeyRow* kt = (const KeyRow*)sc.dev;
  const uint32_t* kids = (const uint32_t*)(sc.dev + Scratch::kDesc);
  hipError_t e = ctx->suite == MQ_SUITE_CHACHA20
                     ? mq_launch_chacha_hp(kt, 1, kids, sc.dev + Scratch::kSample, sc.dev + Scratch::kStatus, 1, sc.stream)
                     : mq_launch_aes_hp(kt, 1, kids, sc.dev + Scratch::kSample, sc.dev + Scratch::kStatus, 1, sc.stream);
  if (e != hipSuccess) return MQ_ERR_HIP;
  if ((rc = sc.finish(Scratch::kStatus, 8)) != MQ_OK) return rc;
  std::memcpy(mask, sc.host + Scratch::kStatus, 5);
  return MQ_OK;
}

void mq_nonce(const uint8_t iv[12], uint64_t packet_number, uint8_t nonce[12]) {
  std::memcpy(nonce, iv, 12);
  for (int i = 0; i < 8; ++i) nonce[4 + i] ^= (uint8_t)(packet_number >> (56 - 8 * i));
}

void mq_hkdf_extract(const uint8_t* salt, size_t salt_len, const uint8_t* ikm, size_t ikm_len,
                     uint8_t prk[32]) {
  hmac_sha256(salt, salt_len, ikm, ikm_len, nullptr, 0, nullptr, 0, prk);
}

int mq_hkdf_expand(const uint8_t* prk, size_t prk_len, const uint8_t* info, size_t info_len,
                   uint8_t* okm, size_t okm_len) {
  if (prk_len < 32 || okm_len > 255 * 32 || (!okm && okm_len)) return MQ_ERR_CRYPTO;
  uint8_t t[32];
  size_t tlen = 0, done = 0;
  for (uint8_t i = 1; done < okm_len; ++i) {
    hmac_sha256(prk, prk_len, t, tlen, info, info_len, &i, 1, t);
    tlen = 32;
    const size_t n = std::min(okm_len - done, (size_t)32);
    std::memcpy(okm + done, t, n);
    done += n;
  }
  return MQ_OK;
}

int mq_hkdf_expand_label(const uint8_t* secret, size_t secret_len, const uint8_t* label,
                         size_t label_len, const uint8_t* context, size_t context_len,
                         uint8_t* out, size_t out_len) {
  // key_schedule.rs:23-55: HkdfLabel = u16 length || u8 len || "tls13 " label || u8 len || ctx
  const size_t full = 6 + label_len, info_len = 2 + 1 + full + 1 + context_len;
  if (info_len > 80) return MQ_ERR_CRYPTO;
  uint8_t info[80];
  info[0] = (uint8_t)(out_len >> 8);
  info[1] = (uint8_t)out_len;
  info[2] = (uint8_t)full;
  std::memcpy(info + 3, "tls13 ", 6);
  if (label_len) std::memcpy(info + 9, label, label_len);
  info[3 + full] = (uint8_t)context_len;
  if (context_len) std::memcpy(info + 4 + full, context, context_len);
  return mq_hkdf_expand(secret, secret_len, info, info_len, out, out_len);
}

int mq_derive_initial_secrets(const uint8_t* dcid, size_t dcid_len, uint8_t client_secret[32],
                              uint8_t server_secret[32]) {
  static const uint8_t salt[20] = {0x38, 0x76, 0x2c, 0xf7, 0xf5, 0x59, 0x34, 0xb3, 0x4d, 0x17,
                                   0x9a, 0xe6, 0xa4, 0xc8, 0x0c, 0xad, 0xcc, 0xbb, 0x7f, 0x0a};
  uint8_t initial[32];
  mq_hkdf_extract(salt, 20, dcid, dcid_len, initial);
  int rc = mq_hkdf_expand_label(initial, 32, (const uint8_t*)"client in", 9, nullptr, 0, client_secret, 32);
  if (rc) return rc;
  return mq_hkdf_expand_label(initial, 32, (const uint8_t*)"server in", 9, nullptr, 0, server_secret, 32);
}

int mq_derive_key_material(uint32_t suite, const uint8_t* secret, size_t secret_len,
                           mq_key_material* out) {
  const size_t klen = suite_key_len(suite);
  if (!klen || !out) return MQ_ERR_CRYPTO;
  std::memset(out, 0, sizeof *out);
  out->suite = suite;
  int rc = mq_hkdf_expand_label(secret, secret_len, (const uint8_t*)"quic key", 8, nullptr, 0, out->key, klen);
  if (!rc) rc = mq_hkdf_expand_label(secret, secret_len, (const uint8_t*)"quic iv", 7, nullptr, 0, out->iv, 12);
  if (!rc)  // hp_key_len = max(KEY_LEN, 16), key_schedule.rs:133
    rc = mq_hkdf_expand_label(secret, secret_len, (const uint8_t*)"quic hp", 7, nullptr, 0, out->hp,
                              klen > 16 ? klen : 16);
  return rc;
}

int mq_derive_next_secret(const uint8_t* secret, size_t secret_len, uint8_t next[32]) {
  return mq_hkdf_expand_label(secret, secret_len, (const uint8_t*)"quic ku", 7, nullptr, 0, next, 32);
}

int mq_keytable_create(const mq_key_material* rows, uint32_t n_rows, mq_keytable** out) {
  if (!out || (!rows && n_rows)) return MQ_ERR_INVALID_ARG;
  *out = nullptr;
  const int dev = creation_device();
  if (dev < 0) return MQ_ERR_NO_DEVICE;
  DeviceGuard g(dev);
  if (!g.ok()) return MQ_ERR_NO_DEVICE;
  mq_keytable* kt = new mq_keytable();
  kt->rows = n_rows;
  kt->device = dev;
  if (hipMalloc(&kt->dev, sizeof(KeyRow) * (n_rows ? n_rows : 1)) != hipSuccess) {
    delete kt;
    return MQ_ERR_HIP;
  }
  int rc = mq_keytable_update(kt, 0, rows, n_rows);
  if (rc) {
    mq_keytable_free(kt);
    return rc;
  }
  *out = kt;
  return MQ_OK;
}

int mq_keytable_update(mq_keytable* kt, uint32_t first_row, const mq_key_material* rows, uint32_t n_rows) {
  if (!kt || (uint64_t)first_row + n_rows > kt->rows) return MQ_ERR_INVALID_ARG;
  if (!n_rows) return MQ_OK;
  std::vector<KeyRow> host(n_rows);
  for (uint32_t i = 0; i < n_rows; ++i)
    if (!build_row(rows[i], host[i])) std::memset(&host[i], 0, sizeof(KeyRow));  // suite 0: rejected per packet
  DeviceGuard g(kt->device);
  if (!g.ok()) return MQ_ERR_NO_DEVICE;
  if (hipMemcpy(kt->dev + first_row, host.data(), sizeof(KeyRow) * n_rows, hipMemcpyHostToDevice) != hipSuccess)
    return MQ_ERR_HIP;
  kt_mirror(kt, first_row, n_rows, [&](uint32_t i) { return (uint8_t)host[i].suite; });
  return MQ_OK;
}

uint32_t mq_keytable_rows(const mq_keytable* kt) { return kt ? kt->rows : 0; }

void mq_keytable_free(mq_keytable* kt) {
  if (!kt) return;
  if (kt->dev) {
    DeviceGuard g(kt->device);
    (void)hipFree(kt->dev);
  }
  delete kt;
}

// workspace: [open pre-pass HP masks, 8 B per packet][partition lists (mixed batches)]
static size_t ws_align(size_t b) { return (b + 255) & ~(size_t)255; }
size_t mq_batch_workspace_size(uint32_t n) { return ws_align(8 * (size_t)n) + mq_partition_workspace(n); }

// recv_pass (mq_batch_recv's AEAD passes): descriptors without a valid key row are skipped —
// no status is written for them; the receive composite reads only what it attempted. live (receive
// passes): device word with the pass's number of keyed descriptors, 0 = the partition publishes
// empty lists at once (mq_partition.hip). hpm_ready: the open pre-pass values are already in the
// workspace (the receive walk writes them), so no header-protection pre-pass runs.
static int batch(bool open, const mq_keytable* kt, uint8_t* arena, uint64_t arena_len,
                 const mq_pkt_desc* desc, uint32_t n, uint8_t* status, uint64_t* pn_out,
                 uint32_t suite_hint, void* workspace, void* stream, bool recv_pass = false,
                 const uint32_t* live = nullptr, bool hpm_ready = false) {
  if (!kt || (n && (!arena || !desc || !status))) return MQ_ERR_INVALID_ARG;
  if (((uintptr_t)arena & 15) != 0) return MQ_ERR_INVALID_ARG;  // 16-B staging chunks
  DeviceGuard g(kt->device);  // the table's device; `stream` must belong to it
  if (!g.ok()) return MQ_ERR_NO_DEVICE;
  if (n == 0) return MQ_OK;
  // MQ_BATCH_LEN_HINT in the high half; without it the arena's bytes per packet stand in for the
  // batch's (right when the arena holds just this batch)
  const uint64_t len_hint = suite_hint >> 16;
  suite_hint &= 0xFFFFu;
  const uint64_t bpp = len_hint ? len_hint : (arena_len + n - 1) / n;
  const int cus = devices().cus(kt->device);
  hipStream_t s = (hipStream_t)stream;
  hipError_t e = hipSuccess;
  uint8_t* ws = (uint8_t*)workspace;
  // open with a workspace: header-protection masks come from the one-lane-per-packet pre-pass
  uint2* hpm = (open && ws) ? (uint2*)ws : nullptr;
  if (suite_hint == MQ_SUITE_CHACHA20) {
    e = mq_launch_chacha(open, kt->dev, kt->rows, arena, arena_len, desc, n, nullptr, nullptr, status, pn_out, hpm, true,
                         s, cus, nullptr, -1, false, nullptr, bpp);
  } else if (suite_hint == MQ_SUITE_AES128GCM && (kt->rows == 1 || !ws || n > (1u << 30))) {
    e = mq_launch_aes(open, kt->dev, kt->rows, arena, arena_len, desc, n, nullptr, nullptr, nullptr, status, pn_out,
                      hpm, true, s, s, cus, nullptr, sched_slot(kt->device, s), nullptr, bpp);
  } else if (suite_hint == MQ_SUITE_MIXED || suite_hint == MQ_SUITE_AES128GCM) {
    // the two index lists (2 x mq_partition_list_cap(n) entries, holes included) are addressed
    // with 32-bit positions: up to 2^30 packets per mixed batch. An AES batch over several key
    // rows takes the partition too, for its key-uniform tiles; whatever it puts in the second
    // list (packets of other suites, bad key ids) goes to the AES kernel as well, which rejects
    // it exactly as the flat launch would.
    if (!ws || n > (1u << 30)) return MQ_ERR_INVALID_ARG;
    const bool aes_only = suite_hint == MQ_SUITE_AES128GCM;
    uint8_t* pw = ws + ws_align(8 * (size_t)n);
    uint32_t* list = (uint32_t*)pw;
    size_t codes_off, counts_off;
    mq_partition_layout(n, &codes_off, &counts_off);
    uint32_t* codes = (uint32_t*)(pw + codes_off);
    uint32_t* counts = (uint32_t*)(pw + counts_off);
    // list mode: the grids cover the list capacity; the kernels read the real lengths from counts
    const uint32_t cap = mq_partition_list_cap(n);
    // open: one header-protection pre-pass over the whole batch in descriptor order, both suites,
    // before the tiles (seal needs none: the tiles mask their own packets). It runs on a side
    // stream beside the partition (r05: the partition no longer has a single-workgroup launch for
    // its blocks to delay — r03f measured that scan 27 -> 85 us and no gain); MQ_HP_FORK=0
    // (diagnostic, mq_opts.h) runs it on s after the partition, as r04 did.
    {
      const bool hp = open && hpm && !hpm_ready;
      auto hfork = hp && fork_enabled() && mq::opt(mq::Opt::HpFork) != 0 ? side_streams().fork(kt->device, s, 1)
                                                                          : mq::SideStreams<HipBackend>::Fork();
      if (hp && hfork) e = mq_launch_mixed_open_hp(kt->dev, kt->rows, arena, arena_len, desc, n, hpm, hfork.side(0));
      if (e == hipSuccess) e = mq_launch_partition(kt->dev, kt->rows, desc, n, list, codes, counts, s, recv_pass, live);
      if (e == hipSuccess && hp && !hfork) e = mq_launch_mixed_open_hp(kt->dev, kt->rows, arena, arena_len, desc, n, hpm, s);
      if (!hfork.join() && e == hipSuccess) e = hipErrorUnknown;
    }  // the fork's entry lock is released before the AES fork below takes it
    if (e != hipSuccess) return MQ_ERR_HIP;
    // The hot AES key's segment (counts + 2: its row and segment length, list 0's front;
    // single-key kernel) runs on a side stream beside the other AES keys' tiles on s: each CU moves
    // on to the other kernel's workgroups as its own finish (r02: E 2.794 -> 2.749 ms). List 1
    // (ChaCha20, or the AES hint's leftovers) follows on s: forked as well it cost E 15 % (r03a:
    // 1.346 -> 1.562 ms seal), because its 40-KiB workgroups take CUs that the persistent AES
    // grids (one 152-KiB workgroup per CU) then wait for. Side streams are per (device, caller
    // stream): mq_runtime.h.
    // Keys with many packets each (on average >= kSegPackets per row, keyed layout): the
    // key-segmented single-key kernels run list 0 whole, no fork (mq_aes.hip aes_seg_tiles)
    constexpr uint32_t kSegPackets = 512;
    const long seg_opt = mq::opt(mq::Opt::AesSeg);  // diagnostic: 0 = never, 1 = whenever keyed
    const bool seg_force = seg_opt == 1;
    const uint32_t* rowseg = seg_opt == 0 || (!seg_force && (uint64_t)n < (uint64_t)kSegPackets * kt->rows)
                                 ? nullptr
                                 : mq_partition_rowseg(n, kt->rows, counts);
    auto fork = fork_enabled() && !rowseg ? side_streams().fork(kt->device, s, 1) : mq::SideStreams<HipBackend>::Fork();
    // list 1 stays on s: after the hot segment on its side stream instead it cost E 2 % (the slice
    // kernel) to 10 % (the tile kernel) (profiles/r06r_ab_e_list1_after_hot_rejected.txt)
    hipStream_t s_hot = fork ? fork.side(0) : s, s_list1 = s;
    uint32_t* sched_s = sched_slot(kt->device, s);
    e = mq_launch_aes(open, kt->dev, kt->rows, arena, arena_len, desc, cap, list, counts, counts + 2, status, pn_out,
                      hpm, false, s, s_hot, cus, rowseg, sched_s, s_hot != s ? sched_slot(kt->device, s_hot) : nullptr);
    if (e == hipSuccess && aes_only)
      e = mq_launch_aes(open, kt->dev, kt->rows, arena, arena_len, desc, cap, list + cap, counts + 1, nullptr, status,
                        pn_out, hpm, false, s_list1, s_list1, cus, nullptr, sched_slot(kt->device, s_list1), nullptr);
    else if (e == hipSuccess)
      e = mq_launch_chacha(open, kt->dev, kt->rows, arena, arena_len, desc, cap, list + cap, counts + 1, status,
                           pn_out, hpm, false, s_list1, cus, sched_slot(kt->device, s_list1), kt->single_row(),
                           recv_pass, mq_partition_regions(counts), bpp);
    // join even after a failed launch, so no side stream runs ahead of s
    if (!fork.join() && e == hipSuccess) e = hipErrorUnknown;
  } else {
    return MQ_ERR_INVALID_ARG;
  }
  return e == hipSuccess ? MQ_OK : MQ_ERR_HIP;
}

int mq_batch_seal(const mq_keytable* kt, uint8_t* arena, uint64_t arena_len, const mq_pkt_desc* desc,
                  uint32_t n, uint8_t* status, uint32_t suite_hint, void* workspace, void* stream) {
  return batch(false, kt, arena, arena_len, desc, n, status, nullptr, suite_hint, workspace, stream);
}

int mq_batch_open(const mq_keytable* kt, uint8_t* arena, uint64_t arena_len, const mq_pkt_desc* desc,
                  uint32_t n, uint8_t* status, uint64_t* pn_out, uint32_t suite_hint, void* workspace,
                  void* stream) {
  return batch(true, kt, arena, arena_len, desc, n, status, pn_out, suite_hint, workspace, stream);
}

}  // extern "C"

// ---- batched Initial key derivation (keys.rs:181-212 per new client DCID) ---------------------
namespace {
// The padded second block of HMAC(secret, HkdfLabel(label, "", L) || 0x01) (key_schedule.rs:23-55;
// one HKDF-Expand block since L <= 32), as 16 big-endian words.
void label_block(const char* label, uint16_t out_len, uint32_t w[16]) {
  uint8_t b[64] = {0};
  const size_t ll = std::strlen(label);
  size_t n = 0;
  b[n++] = (uint8_t)(out_len >> 8);
  b[n++] = (uint8_t)out_len;
  b[n++] = (uint8_t)(6 + ll);
  std::memcpy(b + n, "tls13 ", 6);
  n += 6;
  std::memcpy(b + n, label, ll);
  n += ll;
  b[n++] = 0;     // empty context
  b[n++] = 0x01;  // HKDF-Expand block counter
  b[n] = 0x80;
  const uint64_t bits = (64 + n) * 8;
  for (int i = 0; i < 8; ++i) b[56 + i] = (uint8_t)(bits >> (56 - 8 * i));
  for (int i = 0; i < 16; ++i) w[i] = be32(b + 4 * i);
}

const mq::MQDeriveConsts& derive_consts() {
  static mq::MQDeriveConsts k;
  static std::once_flag once;
  std::call_once(once, [] {
    static const uint8_t salt[20] = {0x38, 0x76, 0x2c, 0xf7, 0xf5, 0x59, 0x34, 0xb3, 0x4d, 0x17,
                                     0x9a, 0xe6, 0xa4, 0xc8, 0x0c, 0xad, 0xcc, 0xbb, 0x7f, 0x0a};
    uint8_t pad[64];
    Sha256 si, so;
    for (int i = 0; i < 64; ++i) pad[i] = (i < 20 ? salt[i] : 0) ^ 0x36;
    si.block(pad);
    for (int i = 0; i < 64; ++i) pad[i] = (i < 20 ? salt[i] : 0) ^ 0x5c;
    so.block(pad);
    for (int i = 0; i < 8; ++i) { k.salt_ist[i] = si.h[i]; k.salt_ost[i] = so.h[i]; }
    label_block("client in", 32, k.lbl[0]);
    label_block("server in", 32, k.lbl[1]);
    label_block("quic key", 16, k.lbl[2]);
    label_block("quic iv", 12, k.lbl[3]);
    label_block("quic hp", 16, k.lbl[4]);
  });
  return k;
}
}  // namespace

extern "C" {

int mq_batch_derive_initial(mq_keytable* kt, uint32_t first_row, const uint8_t* dcids, const uint8_t* dcid_lens,
                            uint32_t n, mq_key_material* km_out, uint8_t* status, void* stream) {
  if (!kt || (n && (!dcids || !dcid_lens || !status))) return MQ_ERR_INVALID_ARG;
  if ((uint64_t)first_row + 2ull * n > kt->rows) return MQ_ERR_INVALID_ARG;
  DeviceGuard g(kt->device);
  if (!g.ok()) return MQ_ERR_NO_DEVICE;
  // the derived rows are AES-128-GCM, or suite 0 for an over-long DCID — unknown here, so the table
  // leaves the single-key list path for good (a per-row host update cost 0.8 ms per 2^21 rows)
  kt->derived = kt->derived || n > 0;
  return mq_launch_derive_initial(derive_consts(), dcids, dcid_lens, n, kt->dev + first_row, km_out, status,
                                  (hipStream_t)stream) == hipSuccess
             ? MQ_OK
             : MQ_ERR_HIP;
}

// ---- send composite from frames (transmit.rs:499-755) -----------------------------------------
// workspace: [descriptors 32 B x n][build status n][seal workspace]
size_t mq_batch_protect_workspace_size(uint32_t n) {
  return ws_align(sizeof(mq_pkt_desc) * (size_t)n) + ws_align(n) + mq_batch_workspace_size(n);
}

int mq_batch_protect(const mq_keytable* kt, const mq_conn_send* conns, uint32_t n_conns, const uint8_t* frames,
                     uint64_t frames_len, uint8_t* out, uint64_t out_len, const mq_send_req* req, uint32_t n,
                     uint8_t* status, uint32_t* pkt_len, uint32_t suite_hint, void* workspace, void* stream) {
  if (!kt || (n && (!conns || !frames || !out || !req || !status || !pkt_len || !workspace)))
    return MQ_ERR_INVALID_ARG;
  suite_hint &= 0xFFFFu;  // a length hint (MQ_BATCH_LEN_HINT) is not used here
  if (((uintptr_t)out & 15) != 0) return MQ_ERR_INVALID_ARG;
  DeviceGuard g(kt->device);
  if (!g.ok()) return MQ_ERR_NO_DEVICE;
  if (n == 0) return MQ_OK;
  hipStream_t s = (hipStream_t)stream;
  // ChaCha20 batches (r04): one fused kernel builds each tile's packets into LDS and seals them
  // there (mq_chacha.hip); MQ_PROTECT_FUSED=0 (diagnostic, mq_opts.h: tests compare both) keeps
  // the two-kernel composite below
  if (mq::opt(mq::Opt::ProtectFused) != 0 && suite_hint == MQ_SUITE_CHACHA20)
    return mq_launch_chacha_protect(kt->dev, kt->rows, conns, n_conns, frames, frames_len, out, out_len, req, n,
                                    suite_hint, status, pkt_len, s) == hipSuccess
               ? MQ_OK
               : MQ_ERR_HIP;
  uint8_t* ws = (uint8_t*)workspace;
  mq_pkt_desc* desc = (mq_pkt_desc*)ws;
  uint8_t* bstatus = ws + ws_align(sizeof(mq_pkt_desc) * (size_t)n);
  void* seal_ws = bstatus + ws_align(n);
  // Pipelined (r04): the batch in kProtectChunks chunks, each built on the caller's stream and sealed
  // on a side stream once its build is done, so chunk k's seal (VALU-bound) runs beside chunk
  // k + 1's build (memory-bound). r03 built the whole batch, then sealed it: 1.35 + 1.14 ms at
  // 2^20 x 1200 B (profiles/r04g_kernel_stats_protect.csv). Small batches, or without a side
  // stream, run build then seal on the caller's stream.
  constexpr uint32_t kProtectChunks = 4;
  auto fork = (fork_enabled() && n >= (1u << 15)) ? side_streams().fork(kt->device, s, 1)
                                                  : mq::SideStreams<HipBackend>::Fork();
  if (!fork) {
    if (mq_launch_build(kt->dev, kt->rows, conns, n_conns, frames, frames_len, out, out_len, req, n, desc, bstatus,
                        pkt_len, suite_hint, s) != hipSuccess)
      return MQ_ERR_HIP;
    const int sr = batch(false, kt, out, out_len, desc, n, status, nullptr, suite_hint, seal_ws, stream);
    if (sr != MQ_OK) return sr;
    return mq_launch_send_status(bstatus, status, n, s) == hipSuccess ? MQ_OK : MQ_ERR_HIP;
  }
  hipStream_t hs = fork.side(0);
  int rc = MQ_OK;
  for (uint32_t k = 0; k < kProtectChunks && rc == MQ_OK; ++k) {
    const uint32_t lo = (uint32_t)((uint64_t)n * k / kProtectChunks), hi = (uint32_t)((uint64_t)n * (k + 1) / kProtectChunks);
    if (mq_launch_build(kt->dev, kt->rows, conns, n_conns, frames, frames_len, out, out_len, req + lo, hi - lo,
                        desc + lo, bstatus + lo, pkt_len + lo, suite_hint, s) != hipSuccess ||
        !fork.hand_off((int)k, 0)) {
      rc = MQ_ERR_HIP;
      break;
    }
    // the seal workspace is used by one chunk after the other (all on hs)
    rc = batch(false, kt, out, out_len, desc + lo, hi - lo, status + lo, nullptr, suite_hint, seal_ws, hs);
  }
  if (!fork.join() && rc == MQ_OK) rc = MQ_ERR_HIP;  // s waits for the seals, even after a failure
  if (rc != MQ_OK) return rc;
  return mq_launch_send_status(bstatus, status, n, s) == hipSuccess ? MQ_OK : MQ_ERR_HIP;
}

// ---- receive composite over raw datagrams (recv.rs:189-510, 953-1025) --------------------------
size_t mq_batch_recv_workspace_size(uint32_t n_dgrams, uint32_t max_pkts, uint32_t n_conns) {
  return mq_recv_workspace(n_dgrams, max_pkts, n_conns, mq_batch_workspace_size(max_pkts));
}

int mq_batch_recv(const mq_keytable* kt, mq_conn_recv* conns, uint32_t n_conns, uint8_t* arena, uint64_t arena_len,
                  const mq_dgram* dgrams, uint32_t n_dgrams, mq_recv_pkt* pkts, uint32_t max_pkts, uint32_t* n_pkts,
                  void* workspace, void* stream) {
  if (!kt || !n_pkts || !workspace || (n_conns && !conns) || (n_dgrams && (!arena || !dgrams)) ||
      (max_pkts && !pkts))
    return MQ_ERR_INVALID_ARG;
  if (((uintptr_t)arena & 15) != 0) return MQ_ERR_INVALID_ARG;
  DeviceGuard g(kt->device);
  if (!g.ok()) return MQ_ERR_NO_DEVICE;
  hipStream_t s = (hipStream_t)stream;
  const size_t open_ws = mq_batch_workspace_size(max_pkts);
  mq::MQRecvPass p;
  const uint32_t seg = mq_recv_seg_len();  // once per batch: every walk uses the same segment layout
  if (mq_recv_front(kt->dev, kt->rows, conns, n_conns, arena, arena_len, dgrams, n_dgrams, max_pkts, n_pkts, pkts,
                    workspace, open_ws, &p, seg, s) != hipSuccess)
    return MQ_ERR_HIP;
  if (!max_pkts) return MQ_OK;
  mq_recv_trace("walk 1", n_dgrams, max_pkts, n_conns, workspace, open_ws, seg, s);
  // walk -> AEAD passes -> walk ...: the first walk speculates that every packet opens, later walks
  // re-attempt what the real outcomes changed (rare: after a failed packet); the last walk defers
  // anything still unresolved. Fixed rounds keep the call asynchronous (no host read-back).
  // Passes with nothing keyed (live word 0: in a batch where every packet opens, everything after
  // the first pass) cost a few empty launches; the walks write the open pre-pass values.
  constexpr int kRounds = 2;
  for (int round = 0; round < kRounds; ++round) {
    int r = batch(true, kt, arena, arena_len, p.d1, max_pkts, p.st1, nullptr, MQ_SUITE_MIXED, p.open_ws, stream, true,
                  p.live1, true);
    if (r != MQ_OK) return r;
    if (mq_recv_retry(n_dgrams, max_pkts, n_conns, workspace, open_ws, s) != hipSuccess) return MQ_ERR_HIP;
    r = batch(true, kt, arena, arena_len, p.d2, max_pkts, p.st2, nullptr, MQ_SUITE_MIXED, p.open_ws, stream, true,
              p.live2, true);
    if (r != MQ_OK) return r;
    if (mq_recv_outcomes(n_dgrams, max_pkts, n_conns, workspace, open_ws, s) != hipSuccess) return MQ_ERR_HIP;
    if (mq_recv_walk(kt->dev, kt->rows, conns, n_conns, n_dgrams, max_pkts, pkts, workspace, open_ws,
                     round + 1 == kRounds, true, (uint32_t)round + 1, seg, s) != hipSuccess)
      return MQ_ERR_HIP;
    mq_recv_trace(round + 1 == kRounds ? "final walk" : "walk 2", n_dgrams, max_pkts, n_conns, workspace, open_ws,
                  seg, s);
  }
  // Re-seal pass: a packet that opened under the speculation's inputs but fails under the
  // reference's (MQ_ERR_CRYPTO) holds plaintext; the final walk left its opening key row and PN in
  // d1 (every other entry has no key row and is skipped), and sealing it again under them restores
  // its bytes as received. Statuses land in the st1 scratch.
  return batch(false, kt, arena, arena_len, p.d1, max_pkts, p.st1, nullptr, MQ_SUITE_MIXED, p.open_ws, stream, true,
               p.live1);
}

// ---- TLS 1.3 records (tcp_tls/record.rs:88-143, connection.rs:546-600) -----------------------
int mq_record_seal(const mq_aead_ctx* ctx, const uint8_t* nonce, size_t nonce_len, uint8_t* buf,
                   size_t buf_len, size_t payload_len, uint8_t inner_type, size_t* out_len,
                   size_t* needed) {
  if (!ctx || !buf) return MQ_ERR_INVALID_ARG;
  const size_t inner_len = payload_len + 1;  // plaintext || inner content type
  if (buf_len < inner_len + 16) {            // record.rs:97-99
    if (needed) *needed = inner_len + 16;
    return MQ_ERR_BUFFER_TOO_SMALL;
  }
  const uint16_t outer = (uint16_t)(inner_len + 16);  // `as u16`, record.rs:103
  const uint8_t aad[5] = {23, 3, 3, (uint8_t)(outer >> 8), (uint8_t)outer};
  buf[payload_len] = inner_type;  // record.rs:100, before the seal (kept on a seal error too)
  return mq_aead_seal_in_place(ctx, nonce, nonce_len, aad, 5, buf, buf_len, inner_len, out_len, needed);
}

int mq_record_open(const mq_aead_ctx* ctx, const uint8_t* nonce, size_t nonce_len, uint8_t* buf,
                   size_t buf_len, size_t ct_len, const uint8_t header[5], size_t* data_len,
                   uint8_t* inner_type) {
  if (!ctx || !buf || !header) return MQ_ERR_INVALID_ARG;
  size_t pt_len = 0;
  const int rc = mq_aead_open_in_place(ctx, nonce, nonce_len, header, 5, buf, buf_len, ct_len, &pt_len);
  if (rc != MQ_OK) return rc;
  size_t pos = pt_len;  // find_inner_content_type (connection.rs:546-556)
  while (pos > 0 && buf[pos - 1] == 0) --pos;
  if (pos == 0 || buf[pos - 1] < 20 || buf[pos - 1] > 23) return MQ_ERR_TLS;
  if (data_len) *data_len = pos - 1;
  if (inner_type) *inner_type = buf[pos - 1];
  return MQ_OK;
}

int mq_batch_seal_records(const mq_keytable* kt, uint8_t* arena, uint64_t arena_len, const mq_pkt_desc* desc,
                          uint32_t n, uint8_t* status, uint32_t suite_hint, void* workspace, void* stream) {
  return batch(false, kt, arena, arena_len, desc, n, status, nullptr, suite_hint, workspace, stream);
}

int mq_batch_open_records(const mq_keytable* kt, uint8_t* arena, uint64_t arena_len, const mq_pkt_desc* desc,
                          uint32_t n, uint8_t* status, uint64_t* info, uint32_t suite_hint, void* workspace,
                          void* stream) {
  int rc = batch(true, kt, arena, arena_len, desc, n, status, info, suite_hint, workspace, stream);
  if (rc != MQ_OK || n == 0) return rc;
  return mq_launch_record_inner(arena, arena_len, desc, n, status, info, (hipStream_t)stream) == hipSuccess
             ? MQ_OK
             : MQ_ERR_HIP;
}

int mq_batch_hp_mask(const mq_keytable* kt, const uint32_t* key_ids, const uint8_t* samples,
                     uint8_t* masks, uint32_t n, void* stream) {
  if (!kt || (n && (!key_ids || !samples || !masks))) return MQ_ERR_INVALID_ARG;
  DeviceGuard g(kt->device);
  if (!g.ok()) return MQ_ERR_NO_DEVICE;
  hipStream_t s = (hipStream_t)stream;
  hipError_t e = mq_launch_chacha_hp(kt->dev, kt->rows, key_ids, samples, masks, n, s);
  if (e == hipSuccess) e = mq_launch_aes_hp(kt->dev, kt->rows, key_ids, samples, masks, n, s);
  return e == hipSuccess ? MQ_OK : MQ_ERR_HIP;
}

int mq_batch_time_seal_open(const mq_keytable* kt, uint8_t* arena, uint64_t arena_len,
                            const mq_pkt_desc* desc, uint32_t n, uint8_t* status, uint64_t* pn_out,
                            uint32_t suite_hint, void* workspace, void* stream, int iters,
                            float* seal_ms, float* open_ms) {
  if (!kt || iters <= 0 || !seal_ms || !open_ms) return MQ_ERR_INVALID_ARG;
  DeviceGuard g(kt->device);
  if (!g.ok()) return MQ_ERR_NO_DEVICE;
  int rc = MQ_OK;
  hipStream_t s = (hipStream_t)stream;
  std::vector<hipEvent_t> ev(2 * iters + 1, nullptr);
  auto destroy = [&] {
    for (auto& x : ev)
      if (x) (void)hipEventDestroy(x);
  };
  for (auto& x : ev)
    if (hipEventCreate(&x) != hipSuccess) {
      x = nullptr;
      destroy();
      return MQ_ERR_HIP;
    }
  if (hipEventRecord(ev[0], s) != hipSuccess) {
    destroy();
    return MQ_ERR_HIP;
  }
  for (int i = 0; i < iters; ++i) {
    rc = mq_batch_seal(kt, arena, arena_len, desc, n, status, suite_hint, workspace, stream);
    if (rc == MQ_OK && hipEventRecord(ev[2 * i + 1], s) != hipSuccess) rc = MQ_ERR_HIP;
    if (rc == MQ_OK) rc = mq_batch_open(kt, arena, arena_len, desc, n, status, pn_out, suite_hint, workspace, stream);
    if (rc == MQ_OK && hipEventRecord(ev[2 * i + 2], s) != hipSuccess) rc = MQ_ERR_HIP;
    if (rc != MQ_OK) {  // nothing meaningful to time: drain what was enqueued and stop
      (void)hipStreamSynchronize(s);
      destroy();
      return rc;
    }
  }
  if (hipEventSynchronize(ev[2 * iters]) != hipSuccess) {
    destroy();
    return MQ_ERR_HIP;
  }
  double ts = 0, to = 0;
  for (int i = 0; i < iters; ++i) {
    float a = 0, b = 0;
    (void)hipEventElapsedTime(&a, ev[2 * i], ev[2 * i + 1]);
    (void)hipEventElapsedTime(&b, ev[2 * i + 1], ev[2 * i + 2]);
    ts += a;
    to += b;
  }
  destroy();
  *seal_ms = (float)(ts / iters);
  *open_ms = (float)(to / iters);
  return MQ_OK;
}

#ifdef MQ_STAMPS
// Diagnostic build only: route phase stamps to a device buffer of tiles x 8 uint64.
void mq_debug_set_stamps(uint64_t* dev) {
  mq_stamps_set_chacha(dev);
  mq_stamps_set_aes(dev);
}
// the partition kernels' stamps (2 x blocks x 8 uint64: count, then scatter; mq_partition.hip)
void mq_debug_set_part_stamps(uint64_t* dev) { mq_stamps_set_part(dev); }
#endif

}  // extern "C"
