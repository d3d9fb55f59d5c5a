// mq_resident.hip — per-packet Aead / HeaderProtection calls without a kernel launch per call.
//
// The reference's call sites are synchronous and per packet: Aead::seal_in_place
// (transmit.rs:713-718), open_in_place (recv.rs:416-421) and HeaderProtection::mask
// (transmit.rs:729, recv.rs:370) through rustcrypto.rs:38-220. Launching a kernel per call (r02:
// a batch of one) costs 30-40 us; here one resident workgroup per device (one wave) polls a mailbox
// in pinned host memory (mq_resident.h) and serves each call with all 64 lanes on ONE packet:
//   ChaCha20-Poly1305: keystream block b on lane b (b = 0: the Poly1305 key), the MAC as a 64-way
//     interleaved Horner (multiplier r^64, lane j's final multiplier r^(64-j) from a 6-step power
//     ladder), lanes summed in 64-bit limbs;
//   AES-128-GCM: CTR block b on lane b through the wide T-table (built once when the kernel starts),
//     GHASH as a 64-way Horner with the bit-holed product (multiplier H^64, final H^(64-j); the
//     host precomputes H^1 .. H^64 per context), lanes XOR-reduced;
//   header protection: one block on lane 0.
// The packet is copied host -> LDS once, processed in LDS, copied back; open verifies before it
// decrypts (a failed packet is never written back). Memory ordering: the host writes the request
// then `seq`; the wave polls `seq` with system-scope atomic loads (vector memory, never the scalar
// cache), takes a system-scope acquire fence, reads the request with vector loads, and after the
// results a system-scope release fence precedes `done`. The kernel leaves when the host asks (stop),
// or after `idle` ticks without a request (or `life` ticks in all) — an exit claimed with a
// Dekker-style handshake on `state` / `seq`, so a request posted meanwhile is either served or
// finds the kernel gone (the host then relaunches it).
#include "mq_aes.h"
#include "mq_resident.h"

#include <atomic>
#include <chrono>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

namespace mq {

__device__ __forceinline__ uint32_t ld_sys(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint32_t ld_sys_sc(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys_sc(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint32_t uni(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }

// LDS of the resident wave: the request, the packet, scratch
constexpr uint32_t kResReqWords = sizeof(ResReq) / 4;
__shared__ __attribute__((aligned(16))) uint32_t s_req[kResReqWords];
__shared__ __attribute__((aligned(16))) uint8_t s_pkt[kResMaxPkt + 64];
__shared__ __attribute__((aligned(16))) uint32_t s_scr[16];  // one-time key / E_K(J0)
#define REQ (*(const ResReq*)s_req)

// 64-bit lane sums of Poly1305 limbs -> the accumulator mod 2^130 - 5 in 26-bit limbs
__device__ __forceinline__ P26 p26_from_sums(const uint64_t (&s)[5]) {
  uint64_t t[5] = {s[0], s[1], s[2], s[3], s[4]};
  for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
    for (int l = 0; l < 4; ++l) {
      t[l + 1] += t[l] >> 26;
      t[l] &= 0x3ffffff;
    }
    t[0] += (t[4] >> 26) * 5;
    t[4] &= 0x3ffffff;
  }
  P26 h;
#pragma unroll
  for (int l = 0; l < 5; ++l) h.l[l] = (uint32_t)t[l];
  return h;
}

// Poly1305 of AAD||pad||C||pad||lens over the LDS packet (aad at 0, ciphertext at pay), 64 lanes
__device__ void res_poly(uint32_t aad_len, uint32_t pay, uint32_t ct_len, const uint32_t* otk, int lane,
                         uint32_t (&tag)[4]) {
  const LdsSpace sp{s_pkt};
  const P26 r = p26_from_words(otk[0] & 0x0fffffffu, otk[1] & 0x0ffffffcu, otk[2] & 0x0ffffffcu,
                               otk[3] & 0x0ffffffcu, 0);
  // powers by a prefix product over the lanes: after step s lane j holds r^(min(j, 2^(s+1) - 1) + 1)
  // (6 multiplies, not 6 squarings + 6 conditional multiplies); r^64 = lane 63's r^64
  P26 v = r;
#pragma unroll 1
  for (int s = 0; s < 6; ++s) {
    P26 u;
#pragma unroll
    for (int l = 0; l < 5; ++l) u.l[l] = (uint32_t)__shfl((int)v.l[l], max(lane - (1 << s), 0), 64);
    P26 t = v;
    p26_mul(t, p26_mult(u));
    if (lane >= (1 << s)) v = t;
  }
  P26 e;
#pragma unroll
  for (int l = 0; l < 5; ++l) e.l[l] = (uint32_t)__builtin_amdgcn_readlane((int)v.l[l], 63);
  const P26m m64 = p26_mult(e);
  P26 last;
#pragma unroll
  for (int l = 0; l < 5; ++l) last.l[l] = (uint32_t)__shfl((int)v.l[l], 63 - lane, 64);  // r^(64 - lane)
  const P26m ml = p26_mult(last);
  const uint32_t A = (aad_len + 15) >> 4, T = (ct_len + 15) >> 4, nb = A + T + 1;
  const uint32_t K = (nb + 63) / 64;
  const int z = (int)(64 * K) - (int)nb;
  P26 acc;
#pragma unroll
  for (int l = 0; l < 5; ++l) acc.l[l] = 0;
#pragma unroll 1
  for (uint32_t k = 0; k < K; ++k) {
    const int i = (int)(64 * k) + lane - z;
    uint32_t m[4] = {0, 0, 0, 0};
    uint32_t hib = 1;
    if (i < 0) {
      hib = 0;
    } else if (i < (int)A) {
      load_words<4>(sp, 16u * (uint32_t)i, m);
      const int rem = (int)aad_len - 16 * i;
#pragma unroll
      for (int w = 0; w < 4; ++w) m[w] &= byte_mask(rem, w);
    } else if (i < (int)(A + T)) {
      const uint32_t o = 16u * (uint32_t)(i - (int)A);
      load_words<4>(sp, pay + o, m);
      const int rem = (int)(ct_len - o);
#pragma unroll
      for (int w = 0; w < 4; ++w) m[w] &= byte_mask(rem, w);
    } else {
      m[0] = aad_len; m[2] = ct_len;
    }
    const P26 x = p26_from_words(m[0], m[1], m[2], m[3], hib);
#pragma unroll
    for (int l = 0; l < 5; ++l) acc.l[l] += x.l[l];
    p26_mul(acc, k + 1 < K ? m64 : ml);
  }
  uint64_t s[5];
#pragma unroll
  for (int l = 0; l < 5; ++l) {
    uint64_t x = acc.l[l];
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
    s[l] = x;
  }
  const uint32_t sk[4] = {otk[4], otk[5], otk[6], otk[7]};
  p26_finish(p26_from_sums(s), sk, tag);
}

// ChaCha20-Poly1305 seal / open of the LDS packet (aad at 0, body at aad_len); returns MQ_*
__device__ int res_chacha(bool open, uint32_t aad_len, uint32_t body_len, int lane) {
  const LdsSpace sp{s_pkt};
  uint32_t key[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) key[k] = REQ.key[k];
  const uint32_t n0 = REQ.nonce[0], n1 = REQ.nonce[1], n2 = REQ.nonce[2];
  const uint32_t P = open ? body_len - 16 : body_len, pay = aad_len;
  const uint32_t nblk = 1 + (P + 63) / 64;  // block 0: the Poly1305 key
  auto xor_blocks = [&](bool with_otk) {
#pragma unroll 1
    for (uint32_t b0 = 0; b0 < nblk; b0 += 64) {
      const uint32_t b = b0 + (uint32_t)lane;
      uint32_t raw[17];
      load_raw<16>(sp, b >= 1 && b < nblk ? pay + 64 * (b - 1) : 0u, raw);
      uint32_t ks[16];
      chacha20_block(key, b, n0, n1, n2, ks);
      if (b == 0 && with_otk) {
#pragma unroll
        for (int q = 0; q < 8; ++q) s_scr[q] = ks[q];
      } else if (b >= 1 && b < nblk) {
        xor_words<16>(sp, pay + 64 * (b - 1), ks, (int)min(64u, P - 64 * (b - 1)), raw);
      }
    }
    wave_sync();
  };
  uint32_t tag[4];
  if (!open) {
    xor_blocks(true);
    uint32_t otk[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) otk[q] = s_scr[q];
    res_poly(aad_len, pay, P, otk, lane, tag);
    if (lane == 0) store_words<4>(sp, pay + P, tag);
    wave_sync();
    return MQ_OK;
  }
  if (lane == 0) {  // the one-time key only: the MAC reads the untouched ciphertext
    uint32_t ks[16];
    chacha20_block(key, 0, n0, n1, n2, ks);
#pragma unroll
    for (int q = 0; q < 8; ++q) s_scr[q] = ks[q];
  }
  wave_sync();
  uint32_t otk[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) otk[q] = s_scr[q];
  res_poly(aad_len, pay, P, otk, lane, tag);
  uint32_t got[4];
  load_words<4>(sp, pay + P, got);
  const uint32_t diff = uni((tag[0] ^ got[0]) | (tag[1] ^ got[1]) | (tag[2] ^ got[2]) | (tag[3] ^ got[3]));
  if (diff) return MQ_ERR_CRYPTO;  // rustcrypto.rs:156-163; nothing decrypted
  wave_sync();
  xor_blocks(false);
  return MQ_OK;
}

// AES-128-GCM seal / open of the LDS packet
__device__ int res_aes(bool open, uint32_t aad_len, uint32_t body_len, int lane) {
  const LdsSpace sp{s_pkt};
  const TwLane L = tw_lane();
  const RkLds key{REQ.aes_rk};
  const uint32_t nb0 = bswap32(REQ.nonce[0]), nb1 = bswap32(REQ.nonce[1]), nb2 = bswap32(REQ.nonce[2]);
  const uint32_t P = open ? body_len - 16 : body_len, pay = aad_len;
  const uint32_t nblk = 1 + (P + 15) / 16;  // slot 0: E_K(J0), slot b >= 1: CTR block with counter b + 1
  auto ctr_pass = [&](bool with_j0) {
#pragma unroll 1
    for (uint32_t b0 = 0; b0 < nblk; b0 += 64) {
      const uint32_t b = b0 + (uint32_t)lane;
      uint32_t s[4] = {nb0, nb1, nb2, b == 0 ? 1u : b + 1};
      aes128_enc(key, L, s);
      uint32_t ks[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) ks[q] = bswap32(s[q]);
      if (b == 0 && with_j0) {
#pragma unroll
        for (int q = 0; q < 4; ++q) s_scr[8 + q] = ks[q];
      } else if (b >= 1 && b < nblk) {
        uint32_t raw[5];
        const uint32_t o = pay + 16 * (b - 1);
        load_raw<4>(sp, o, raw);
        xor_words<4>(sp, o, ks, (int)min(16u, P - 16 * (b - 1)), raw);
      }
    }
    wave_sync();
  };
  // GHASH(AAD || C || lens) in the reflected basis (mq_aes.h), lane j: blocks 64k + j - z
  auto ghash = [&](uint32_t (&g)[4]) {
    const uint32_t A = (aad_len + 15) >> 4, T = (P + 15) >> 4, nb = A + T + 1;
    const uint32_t K = (nb + 63) / 64;
    const int z = (int)(64 * K) - (int)nb;
    uint32_t h[4];
#pragma unroll
    for (int w = 0; w < 4; ++w) h[w] = brev(REQ.Hpow[63][w]);
    const GfOp m64 = gf_prepare(h);
    uint32_t acc[4] = {0, 0, 0, 0};
#pragma unroll 1
    for (uint32_t k = 0; k < K; ++k) {
      const int i = (int)(64 * k) + lane - z;
      uint32_t m[4] = {0, 0, 0, 0};
      if (i >= 0 && i < (int)A) {
        load_words<4>(sp, 16u * (uint32_t)i, m);
        const int rem = (int)aad_len - 16 * i;
#pragma unroll
        for (int w = 0; w < 4; ++w) m[w] = refl(m[w] & byte_mask(rem, w));
      } else if (i >= (int)A && i < (int)(A + T)) {
        const uint32_t o = 16u * (uint32_t)(i - (int)A);
        load_words<4>(sp, pay + o, m);
        const int rem = (int)(P - o);
#pragma unroll
        for (int w = 0; w < 4; ++w) m[w] = refl(m[w] & byte_mask(rem, w));
      } else if (i == (int)(A + T)) {
        const uint64_t ab = (uint64_t)aad_len * 8, cb = (uint64_t)P * 8;
        m[0] = brev((uint32_t)(ab >> 32)); m[1] = brev((uint32_t)ab);
        m[2] = brev((uint32_t)(cb >> 32)); m[3] = brev((uint32_t)cb);
      }
#pragma unroll
      for (int w = 0; w < 4; ++w) acc[w] ^= m[w];
      if (k + 1 < K) gf_mul(acc, m64);
    }
    uint32_t hl[4];  // H^(64 - lane)
#pragma unroll
    for (int w = 0; w < 4; ++w) hl[w] = brev(REQ.Hpow[63 - lane][w]);
    gf_mul(acc, gf_prepare(hl));
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      uint32_t x = acc[w];
#pragma unroll
      for (int d = 32; d >= 1; d >>= 1) x ^= (uint32_t)__shfl_xor((int)x, d, 64);
      g[w] = x;
    }
  };
  uint32_t g[4], tag[4];
  if (!open) {
    ctr_pass(true);
    ghash(g);
#pragma unroll
    for (int w = 0; w < 4; ++w) tag[w] = bswap32(brev(g[w])) ^ s_scr[8 + w];
    if (lane == 0) store_words<4>(sp, pay + P, tag);
    wave_sync();
    return MQ_OK;
  }
  if (lane == 0) {  // E_K(J0) only: GHASH reads the untouched ciphertext
    uint32_t s[4] = {nb0, nb1, nb2, 1u};
    aes128_enc(key, L, s);
#pragma unroll
    for (int q = 0; q < 4; ++q) s_scr[8 + q] = bswap32(s[q]);
  }
  wave_sync();
  ghash(g);
  uint32_t got[4];
  load_words<4>(sp, pay + P, got);
  uint32_t diff = 0;
#pragma unroll
  for (int w = 0; w < 4; ++w) diff |= (bswap32(brev(g[w])) ^ s_scr[8 + w]) ^ got[w];
  if (uni(diff)) return MQ_ERR_CRYPTO;  // rustcrypto.rs:85-91; nothing decrypted
  wave_sync();
  ctr_pass(false);
  return MQ_OK;
}

__device__ void res_hp(uint32_t suite, int lane, uint32_t& m0, uint32_t& m1) {
  const uint32_t smp[4] = {REQ.sample[0], REQ.sample[1], REQ.sample[2], REQ.sample[3]};
  if (suite == MQ_SUITE_CHACHA20) {  // rustcrypto.rs:197-220
    uint32_t hk[8], blk[16];
#pragma unroll
    for (int k = 0; k < 8; ++k) hk[k] = REQ.hp[k];
    chacha20_block(hk, smp[0], smp[1], smp[2], smp[3], blk);
    m0 = blk[0];
    m1 = blk[1] & 0xffu;
  } else {  // rustcrypto.rs:175-186
    uint32_t s[4] = {bswap32(smp[0]), bswap32(smp[1]), bswap32(smp[2]), bswap32(smp[3])};
    aes128_enc(RkLds{REQ.hp_rk}, tw_lane(), s);
    m0 = bswap32(s[0]);
    m1 = s[1] >> 24;
  }
  (void)lane;
}

}  // namespace mq

using namespace mq;

extern "C" __global__ __launch_bounds__(64) void mq_resident_kernel(ResArea* area, uint64_t idle_ticks,
                                                                    uint64_t life_ticks) {
  const int lane = (int)threadIdx.x;
  ResCtl* ctl = &area->ctl;
  build_tw(lane, 64);  // the wide AES T-table, once per kernel
  wave_sync();
  uint32_t done = uni(ld_sys(&ctl->done));
  const uint64_t t0 = wall_clock64();
  uint64_t t_last = t0;
  for (;;) {
    // seq and stop in one 8-B system-scope load: one PCIe round trip per poll
    const uint64_t ss = __hip_atomic_load((const uint64_t*)&ctl->seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const uint32_t seq = uni((uint32_t)ss);
    if (uni((uint32_t)(ss >> 32))) break;
    if (seq == done) {
      const uint64_t now = wall_clock64();
      if (now - t_last > idle_ticks || now - t0 > life_ticks) {
        // claim the exit, then look once more: a request posted meanwhile is served first
        if (lane == 0) st_sys_sc(&ctl->state, kResExiting);
        wave_sync();
        if (uni(ld_sys_sc(&ctl->seq)) == done) break;
        if (lane == 0) st_sys_sc(&ctl->state, kResRunning);
        t_last = now;
        continue;
      }
      __builtin_amdgcn_s_sleep(1);  // the poll itself is a PCIe round trip (~1 us)
      continue;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope: the request written before seq
    // One round trip: the request (two 16-B loads per lane) and the packet's first 2 KiB (two
    // more), all in flight together; a longer packet's rest follows below. Vector loads with
    // per-lane addresses after the acquire fence (never the scalar cache).
    constexpr uint32_t kReq16 = sizeof(ResReq) / 16, kFirst16 = 128;
    const uint4* rq4 = (const uint4*)&area->req;
    const uint4* src = (const uint4*)area->data;
    const uint4 z4 = make_uint4(0, 0, 0, 0);
    const uint4 q0 = (uint32_t)lane < kReq16 ? rq4[lane] : z4, q1 = (uint32_t)lane + 64 < kReq16 ? rq4[lane + 64] : z4;
    const uint4 d0 = src[lane], d1 = src[lane + 64];
    if ((uint32_t)lane < kReq16) ((uint4*)s_req)[lane] = q0;
    if ((uint32_t)lane + 64 < kReq16) ((uint4*)s_req)[lane + 64] = q1;
    ((uint4*)s_pkt)[lane] = d0;
    ((uint4*)s_pkt)[lane + 64] = d1;
    wave_sync();
    const uint32_t op = uni(REQ.op), suite = uni(REQ.suite), aad_len = uni(REQ.aad_len), body_len = uni(REQ.body_len);
    const uint32_t tot = op == kResHp ? 0u : aad_len + body_len + (op == kResSeal ? 16u : 0u);
    const uint32_t nch = (tot + 15) / 16;
#pragma unroll 1
    for (uint32_t c0 = kFirst16; c0 < nch; c0 += 256) {  // the rest: 4 loads in flight per lane
      uint4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const uint32_t c = c0 + 64 * u + (uint32_t)lane;
        v[u] = c < nch ? src[c] : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const uint32_t c = c0 + 64 * u + (uint32_t)lane;
        if (c < nch) *(uint4*)(s_pkt + 16 * c) = v[u];
      }
    }
    wave_sync();
    int st = MQ_OK;
    uint32_t m0 = 0, m1 = 0;
    if (op == kResHp) {
      res_hp(suite, lane, m0, m1);
    } else if (tot > kResMaxPkt || (op == kResOpen && body_len < 16)) {
      st = MQ_ERR_INVALID_ARG;  // the host checks these; never trust the mailbox
    } else if (suite == MQ_SUITE_CHACHA20) {
      st = res_chacha(op == kResOpen, aad_len, body_len, lane);
    } else if (suite == MQ_SUITE_AES128GCM) {
      st = res_aes(op == kResOpen, aad_len, body_len, lane);
    } else {
      st = MQ_ERR_INVALID_ARG;
    }
    if (st == MQ_OK && op != kResHp) {  // the whole packet back (failed opens are not copied)
      uint4* dst = (uint4*)area->data;
#pragma unroll 1
      for (uint32_t c = (uint32_t)lane; c < nch; c += 64) dst[c] = *(const uint4*)(s_pkt + 16 * c);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: results before done
    if (lane == 0) {
      st_sys(&ctl->status, (uint32_t)st);
      st_sys(&ctl->mask0, m0);
      st_sys(&ctl->mask1, m1);
      __hip_atomic_store(&ctl->done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    done = seq;
    t_last = wall_clock64();
  }
  if (lane == 0) st_sys_sc(&ctl->state, kResExited);
}

// ---- host ------------------------------------------------------------------------------------------
namespace {

struct Resident {
  int dev = -1;
  ResArea* host = nullptr;  // pinned, coherent, mapped
  ResArea* dptr = nullptr;
  hipStream_t stream = nullptr;
  uint32_t seq = 0;
  bool launched = false;
  uint64_t idle = 0, life = 0;
  std::mutex mu;
};

std::mutex g_res_mu;
std::vector<Resident*> g_res;  // per device; never freed (the kernel may outlive static destructors)

void stop_all() {  // atexit: ask every resident kernel to leave (plain stores, no HIP call)
  for (Resident* r : g_res)
    if (r && r->host) __atomic_store_n(&r->host->ctl.stop, 1u, __ATOMIC_SEQ_CST);
}

Resident* resident(int dev) {
  std::lock_guard<std::mutex> lk(g_res_mu);
  if ((size_t)dev >= g_res.size()) g_res.resize((size_t)dev + 1, nullptr);
  if (!g_res[(size_t)dev]) {
    static bool hooked = false;
    if (!hooked) {
      hooked = true;
      std::atexit(stop_all);
    }
    g_res[(size_t)dev] = new Resident();
    g_res[(size_t)dev]->dev = dev;
  }
  return g_res[(size_t)dev];
}

uint32_t load_acq(const uint32_t* p) { return __atomic_load_n(p, __ATOMIC_ACQUIRE); }

}  // namespace

// One call through the resident kernel of device `dev` (the caller holds a device guard on it).
// `q` is the request with keys, nonce / sample, op, suite and lengths filled in; aad || body are
// the packet bytes. Returns MQ_OK when the call was served (*status = its result, out[0, out_len)
// = data bytes [out_off, out_off + out_len) of the processed packet when *status is MQ_OK, mask =
// the header-protection mask words), else an MQ_ERR_* of the transport.
int mq_resident_call(int dev, const ResReq& q, const uint8_t* aad, const uint8_t* body, uint8_t* out,
                     size_t out_off, size_t out_len, int* status, uint32_t* mask) {
  Resident* r = resident(dev);
  std::lock_guard<std::mutex> lk(r->mu);
  if (!r->host) {
    if (hipHostMalloc((void**)&r->host, sizeof(ResArea), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
      r->host = nullptr;
      return MQ_ERR_HIP;
    }
    std::memset(r->host, 0, sizeof(ResArea));
    if (hipHostGetDevicePointer((void**)&r->dptr, r->host, 0) != hipSuccess ||
        hipStreamCreateWithFlags(&r->stream, hipStreamNonBlocking) != hipSuccess)
      return MQ_ERR_HIP;
    int khz = 0;
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz <= 0) khz = 100000;
    const char* e = std::getenv("MQ_RESIDENT_IDLE_US");
    const uint64_t idle_us = e ? (uint64_t)std::strtoull(e, nullptr, 10) : 2000;  // 2 ms without a call
    r->idle = idle_us * (uint64_t)khz / 1000;
    r->life = 10ull * 1000 * (uint64_t)khz;  // 10 s, then leave at the next idle moment
  }
  ResArea* a = r->host;
  std::memcpy(&a->req, &q, sizeof q);
  if (q.op != kResHp) {
    if (q.aad_len) std::memcpy(a->data, aad, q.aad_len);
    if (q.body_len) std::memcpy(a->data + q.aad_len, body, q.body_len);
  }
  const uint32_t seq = ++r->seq;
  __atomic_store_n(&a->ctl.seq, seq, __ATOMIC_SEQ_CST);
  const auto t0 = std::chrono::steady_clock::now();
  for (uint32_t spins = 0;; ++spins) {
    if (load_acq(&a->ctl.done) == seq) break;
    if (!r->launched || __atomic_load_n(&a->ctl.state, __ATOMIC_SEQ_CST) == kResExited) {
      if (r->launched && hipStreamSynchronize(r->stream) != hipSuccess) return MQ_ERR_HIP;  // it has left
      if (load_acq(&a->ctl.done) == seq) break;  // served on its way out
      __atomic_store_n(&a->ctl.state, (uint32_t)kResRunning, __ATOMIC_SEQ_CST);
      __atomic_store_n(&a->ctl.stop, 0u, __ATOMIC_SEQ_CST);
      hipLaunchKernelGGL(mq_resident_kernel, dim3(1), dim3(64), 0, r->stream, r->dptr, r->idle, r->life);
      if (hipGetLastError() != hipSuccess) {
        __atomic_store_n(&a->ctl.state, (uint32_t)kResExited, __ATOMIC_SEQ_CST);
        return MQ_ERR_HIP;
      }
      r->launched = true;
    }
    if ((spins & 1023) == 1023 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(10)) return MQ_ERR_HIP;
  }
  *status = (int)__atomic_load_n(&a->ctl.status, __ATOMIC_ACQUIRE);
  if (mask) {
    mask[0] = a->ctl.mask0;
    mask[1] = a->ctl.mask1;
  }
  if (*status == MQ_OK && out_len) std::memcpy(out, a->data + out_off, out_len);
  return MQ_OK;
}
