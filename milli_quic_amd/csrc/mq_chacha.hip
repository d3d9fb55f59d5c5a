// mq_chacha.hip — AEAD_CHACHA20_POLY1305 packet protection (RFC 8439 / RFC 9001 §5) on gfx950.
//
// Replaces, per packet of a batch, the reference's ChaCha20Poly1305Aead::seal_in_place /
// open_in_place (src/crypto/rustcrypto.rs:111-165) plus ChaChaHeaderProtection::mask
// (:197-220), composed the way src/connection/transmit.rs:625-755 (send) and
// src/connection/recv.rs:340-421,953-1025 (receive) compose them.
//
// Per tile (8 packets, one octet of lanes per packet; see mq_tile.h):
//   seal: keystream block ctr on lane ctr % 8 (ctr 0 = Poly1305 one-time key) XORed into LDS
//         (blocks >= 16 and the header-protection block through the workgroup's keystream pool)
//         -> interleaved Poly1305 over AAD||pad||CT||pad||lens -> tag -> header mask applied
//   open: HP mask -> unmask byte 0 / PN -> decode_pn -> nonce -> first keystream block (lane 0:
//         one-time key) -> Poly1305 over the untouched ciphertext -> tag check -> only then the
//         keystream XOR (held first block + the rest); failed packets are never stored.
#include "mq_tile.h"
#include "mq_build.h"
#include "mq_opts.h"

#include <cstdlib>

namespace mq {

// Byte stride between the LDS images of a packet's consecutive keystream blocks: 64. The
// MQ_PROF_SKIP & 128 diagnostic build (never the product) uses 68 — a 17-dword stride, so the
// eight lanes of a packet hit eight distinct LDS banks — computing garbage with the same
// instructions: its time minus the product's is what the keystream XOR's bank conflicts cost.
#if MQ_PROF_SKIP & 128
constexpr uint32_t kKsStride = 68;
#else
constexpr uint32_t kKsStride = 64;
#endif

// Interleaved Poly1305 of the AEAD MAC input for the octet's packet (RFC 8439 §2.8: AAD||pad16||
// CT||pad16||LE64(len AAD)||LE64(len CT)): lane j takes MAC blocks 8k + j, Horner with r^8, one
// final multiply by r^(8-j), then the octet sum. Every lane of the octet returns the same tag.
template <class S>
__device__ __forceinline__ void poly_tag(const S& sp, typename S::off_t pkt, typename S::off_t pay,
                                         uint32_t aad_len, uint32_t ct_len,
                                         const uint32_t* otk_lds, int j, bool act,
                                         uint32_t (&tag)[4]) {
#if MQ_PROF_SKIP & 2
  for (int w = 0; w < 4; ++w) tag[w] = otk_lds[4 + w] ^ aad_len ^ ct_len;
  return;
#endif
  const uint4 rk = *(const uint4*)otk_lds;  // one-time key r || s, written by octet lane 0
  const P26 r = p26_from_words(rk.x & 0x0fffffffu, rk.y & 0x0ffffffcu, rk.z & 0x0ffffffcu,
                               rk.w & 0x0ffffffcu, 0);
  // powers by an octet prefix: v = r^(j+1) after three multiplies (r^2, then x r^2 on lanes with
  // bit 1 of j, then x r^4 — taken from octet lane 3 — on lanes with bit 2); r^8 is octet lane 7's
  // v, and the final multiplier r^(8-j) is lane 7-j's v (DPP row_half_mirror)
  P26 v = r, t = r;
  p26_mul(t, p26_mult(r));  // r^2
#pragma unroll
  for (int l = 0; l < 5; ++l) v.l[l] = (j & 1) ? t.l[l] : v.l[l];
  {
    P26 u = v;
    p26_mul(u, p26_mult(t));
#pragma unroll
    for (int l = 0; l < 5; ++l) v.l[l] = (j & 2) ? u.l[l] : v.l[l];
  }
  {
    P26 r4, u = v;
#pragma unroll
    for (int l = 0; l < 5; ++l) r4.l[l] = oct_lane3(v.l[l]);
    p26_mul(u, p26_mult(r4));
#pragma unroll
    for (int l = 0; l < 5; ++l) v.l[l] = (j & 4) ? u.l[l] : v.l[l];
  }
  P26 r8, rj;
#pragma unroll
  for (int l = 0; l < 5; ++l) {
    r8.l[l] = oct_lane7(v.l[l]);
    rj.l[l] = half_mirror(v.l[l]);
  }
  const P26m m8 = p26_mult(r8), mlast = p26_mult(rj);

  const uint32_t A = (aad_len + 15) >> 4, T = (ct_len + 15) >> 4, nb = A + T + 1;
  const uint32_t K = (nb + kLanesPerPkt - 1) / kLanesPerPkt;
  const uint32_t Kmax = wave_max_u32(act ? K : 0u);
  // prepend zero blocks (no 2^128 bit) so every packet of the wave runs exactly Kmax steps
  const int z = (int)(kLanesPerPkt * Kmax) - (int)nb;
  P26 acc;
#pragma unroll
  for (int l = 0; l < 5; ++l) acc.l[l] = 0;

  // MAC block i = 8k + j - z of this lane: where it lives, how many of its bytes are real
  struct Blk { typename S::off_t src; int rem; bool pre, lens; };
  auto where = [&](int i) {
    Blk b;
    const bool aad = i < (int)A;
    b.pre = i < 0;  // prepended zero block
    b.lens = i == (int)(A + T);
    b.src = aad ? pkt + 16 * (uint32_t)max(i, 0) : pay + 16 * (uint32_t)(i - (int)A);
    b.rem = aad ? (int)aad_len - 16 * i : (int)ct_len - 16 * (i - (int)A);
    if (b.pre || b.lens) b.src = pkt;
    return b;
  };
  auto absorb = [&](const Blk& b, uint32_t (&m)[4]) {
    // wave-uniform fast path: every active lane holds a whole AAD / ciphertext block
    if (wave_any(act && (b.pre || b.lens || b.rem < 16))) {
#pragma unroll
      for (int w = 0; w < 4; ++w) m[w] &= byte_mask(b.pre ? 0 : b.rem, w);
      if (b.lens) { m[0] = aad_len; m[1] = 0; m[2] = ct_len; m[3] = 0; }
    }
    const P26 x = p26_from_words(m[0], m[1], m[2], m[3], b.pre ? 0u : 1u);
#pragma unroll
    for (int l = 0; l < 5; ++l) acc.l[l] += x.l[l];
  };
  if (Kmax > 0) {
    int i = j - z;
    Blk b = where(i);
    uint32_t m[4];
    load_words<4>(sp, b.src, m);
    // steady state: every active lane moves from one whole ciphertext block to the next one 8
    // blocks on (src + 128, payload alignment fixed), so the address and realignment selector
    // need no per-step recomputation
    const uint32_t sel_pay = sel_load((uint32_t)(pay & 3));
    const int ct_full_end = (int)A + (int)(ct_len >> 4);  // first index past the whole CT blocks
    // lean steps k in [k_lo, k_hi): every active lane absorbs a whole ciphertext block and loads
    // the next whole one (8j + ... - z in [A, ct_full_end - 8)), so no masks, 2^128 bit selects
    // or address recomputation
    const int zA = (int)A + z;
    const uint32_t k_lo = act ? (uint32_t)((zA + kLanesPerPkt - 1) / kLanesPerPkt) : 0u;
    const int hi = ct_full_end + z - 2 * kLanesPerPkt + 1;  // lean iff 8k + 15 - z < ct_full_end
    const uint32_t k_hi = !act ? 0xFFFFFFFFu : (hi <= 0 ? 0u : (uint32_t)((hi + kLanesPerPkt - 1) / kLanesPerPkt));
    const uint32_t klo = wave_max_u32(k_lo), khi = min(~wave_max_u32(~k_hi), Kmax - 1);
    for (uint32_t k = 0; k + 1 < Kmax; ++k) {
      if (k == klo && k < khi) {  // wave-uniform: the lean stretch, steps klo .. khi - 1
        // only the block address advances; i, src and rem catch up once at the end
        typename S::off_t a = b.src & ~(typename S::off_t)3;
        uint32_t sel = sel_pay;
        pin(sel);  // keep the selector in a register (hipcc rematerialised it every step)
        for (; k < khi; ++k) {
          const P26 x = p26_from_words(m[0], m[1], m[2], m[3], 1u);
#pragma unroll
          for (int l = 0; l < 5; ++l) acc.l[l] += x.l[l];
          a += 128;
          load_words_sel<4>(sp, a, sel, m);
          p26_mul(acc, m8);
        }
        const uint32_t nl = khi - klo;
        i += (int)(kLanesPerPkt * nl);
        b.src += 128 * nl;
        b.rem -= (int)(128 * nl);
        if (k + 1 >= Kmax) break;
      }
      absorb(b, m);
      const bool steady = !act || (i >= (int)A && i + kLanesPerPkt < ct_full_end);
      i += kLanesPerPkt;
      if (!wave_any(!steady)) {
        b.src += 128;
        b.rem -= 128;
        load_words_sel<4>(sp, b.src & ~(typename S::off_t)3, sel_pay, m);
      } else {
        b = where(i);
        load_words<4>(sp, b.src, m);  // next block's LDS reads overlap this multiply
      }
      p26_mul(acc, m8);
    }
    absorb(b, m);
    p26_mul(acc, mlast);
  }
#pragma unroll
  for (int l = 0; l < 5; ++l) acc.l[l] = oct_sum(acc.l[l]);
  const uint4 sk = *(const uint4*)(otk_lds + 4);
  const uint32_t s[4] = {sk.x, sk.y, sk.z, sk.w};
  p26_finish(acc, s, tag);
}

__device__ __forceinline__ void load_key8(const uint32_t* src, uint32_t (&k)[8]) {
  const uint4 a = *(const uint4*)src, b = *(const uint4*)(src + 4);
  k[0] = a.x; k[1] = a.y; k[2] = a.z; k[3] = a.w; k[4] = b.x; k[5] = b.y; k[6] = b.z; k[7] = b.w;
}

// ---- keystream pool of a workgroup (kCcWaves waves, one staged tile each) ---------------------
// A 1200-B packet takes 20 ChaCha20 blocks (one-time key and 19 keystream; open's header-protection
// block runs in the one-packet-per-lane pre-pass, seal's in this pool, below), but an octet runs 24
// slots in three iterations, so 1/6 of the rounds went idle. Each wave runs
// iterations 0 and 1 of its own packets; every later keystream block (slot >= 16) goes to the
// workgroup's pool, which all its lanes work off together between two barriers (open: once the
// MACs have read the ciphertext; seal: before the MACs): 4 waves x 8 packets x 4 blocks = 128
// blocks, two wave-iterations for the four instead of a 4/8-full third one each. (Measured at 2,
// 4 and 8 waves: 8 in lockstep lose most of the gain to staging waits that no longer overlap.
// Seal with the HP block kept in the tile measured no gain: 21 blocks = 2.625 iterations per
// tile leave a 3-iteration wave in every workgroup, profiles/r02_ab_chacha_seal_pool_b_rejected.txt.)
#ifndef MQ_CC_WAVES
#define MQ_CC_WAVES 4
#endif
constexpr int kCcWaves = MQ_CC_WAVES;
#ifndef MQ_CC_POOL_ITERS
#define MQ_CC_POOL_ITERS 2
#endif
constexpr uint32_t kCcOwnIters = MQ_CC_POOL_ITERS;  // a wave's own iterations before the pool
constexpr uint32_t kCcPoolSlot = kCcOwnIters * kLanesPerPkt;  // first pooled slot

// Seal also pools every packet's header-protection block (RFC 9001 §5.4.4: ChaCha20 under the HP
// key, counter and nonce from the 16-B ciphertext sample at pn_offset + 4), as the packet's last
// pool entry: the sample is ciphertext of keystream block 1, in place after iteration 0, and the
// pool's second wave-iteration is otherwise idle for waves 2-3 of a 1200-B workgroup (128 keystream
// blocks + 32 HP blocks = 160 entries < 3 x 64), so the mask costs no extra time and no pass over
// the batch (r02 ran it as a post-pass kernel: 63 us and 0.23 GB per 2^20 packets). The mask waits
// in the record until the MAC has read the unprotected header; octet lane 0 then applies it.
//
// this packet's 32-B pool record in its wave's scratch: [0] pooled keystream blocks | the PN
// length << 8 when the header-protection block is pooled too, [1] payload LDS offset (workgroup)
// | P << 17, [2] / [7] mask words 0 / 1 (written by the pool), [3] key row, [4..6] nonce words
struct CcPool {
  bool on;              // wave-uniform: staged tile whose slots >= 16 go to the pool
  uint8_t* wg;          // the workgroup's LDS
  uint32_t base;        // this wave's region in it
  uint32_t* rec;        // this packet's record
  const KeyRow* kt;
};

// IMG: bytes of LDS per wave (kLdsBytes; the long-packet kernels' larger images, chacha_tile);
// W: waves of the workgroup sharing the pool
template <bool SINGLE, uint32_t IMG = kLdsBytes, uint32_t W = kCcWaves>
__device__ __forceinline__ void cc_pool_run(const CcPool& pool, uint32_t tid = threadIdx.x) {
  constexpr uint32_t kQ = kPktsPerTile * W;  // packets of the workgroup
  static_assert(kQ <= kWave, "one packet per lane in the pool scan");
  const int lane = tid & (kWave - 1);
  const uint32_t w = tid >> 6;
  auto rec = [&](uint32_t q) -> uint32_t* {
    return (uint32_t*)(pool.wg + (q >> 3) * IMG + (IMG - kScratchBytes) + 32u * (q & 7));
  };
  const uint32_t r0l = (uint32_t)lane < kQ ? rec((uint32_t)lane)[0] : 0u;  // lane q: packet q
  const uint32_t nq = (r0l & 0xffu) + ((r0l >> 8) ? 1u : 0u);
  const uint32_t incl = wave_incl_scan(nq), excl = incl - nq;
  const uint32_t T = lane_u32(incl, kWave - 1);
  const LdsSpace sp{pool.wg};
  for (uint32_t e0 = kWave * w; e0 < T; e0 += kWave * W) {  // wave-uniform
    const uint32_t e = e0 + (uint32_t)lane;
    uint32_t q = 0;  // the packet of entry e: the last q with excl[q] <= e
#pragma unroll
    for (uint32_t step = kQ / 2; step >= 1; step >>= 1) {
      const uint32_t v = (uint32_t)__shfl((int)excl, (int)(q + step), kWave);
      if (v <= e) q += step;
    }
    const uint32_t eq = (uint32_t)__shfl((int)excl, (int)q, kWave);
    const bool act = e < T;
    uint32_t* r = rec(q);
    const uint32_t r0 = r[0], r1 = r[1], pay = r1 & 0x1ffffu, P = r1 >> 17;
    const uint32_t idx = e - eq, pn_len = r0 >> 8;
    const bool hp = act && idx == (r0 & 0xffu);  // the packet's last entry: its HP block
    const uint32_t cb = kCcPoolSlot + idx, o = kKsStride * (cb - 1);
    const KeyRow* row = SINGLE || !act ? pool.kt : pool.kt + r[3];  // an idle lane's record may be stale
    uint32_t key[8];
    if (SINGLE) {  // both keys wave-uniform (SGPRs); pick per lane
      uint32_t kd[8], kh[8];
      load_key8(row->key, kd);
      load_key8(row->hp, kh);
#pragma unroll
      for (int k = 0; k < 8; ++k) key[k] = hp ? kh[k] : kd[k];
    } else {
      load_key8(hp ? row->hp : row->key, key);
    }
    uint32_t raw[17], smp[4];
    load_raw<16>(sp, act && !hp ? pay + o : 0u, raw);  // in flight during the rounds
    // the sample: 16 bytes at pn_offset + 4 = payload - pn_len + 4 (ciphertext of block 1)
    load_words<4>(sp, hp ? pay + 4u - pn_len : 0u, smp);
    uint32_t ks[16];
    chacha20_block(key, hp ? smp[0] : cb, hp ? smp[1] : r[4], hp ? smp[2] : r[5], hp ? smp[3] : r[6], ks);
    if (hp) {
      r[2] = ks[0];
      r[7] = ks[1];
    } else if (act) {
      xor_words<16>(sp, pay + o, ks, (int)min(64u, P - o), raw);
    }
  }
}

// RFC 9001 §5.4.1: XOR the mask into the first byte (low 4 / 5 bits) and the PN bytes of a sealed
// packet whose MAC has been computed (octet lane 0)
template <class S>
__device__ __forceinline__ void apply_hp(const S& sp, typename S::off_t pkt, const mq_pkt_desc& d, uint32_t m0,
                                         uint32_t m1) {
  sp.st8(pkt, (uint8_t)(sp.ld8(pkt) ^ ((uint8_t)m0 & ((d.flags & MQ_PKT_LONG_HEADER) ? 0x0f : 0x1f))));
  const uint32_t mk = (m0 >> 8) | (m1 << 24);
  for (uint32_t b = 0; b < d.pn_len; ++b)
    sp.st8(pkt + d.pn_offset + b, (uint8_t)(sp.ld8(pkt + d.pn_offset + b) ^ (uint8_t)(mk >> (8 * b))));
}

struct ChaChaPolicy {
  static constexpr uint32_t kSuite = MQ_SUITE_CHACHA20;

  // raw LDS/HBM dwords under keystream block `ctr` (>= 1): payload [64(ctr-1), min(64 ctr, P))
  template <class S>
  static __device__ __forceinline__ void load_block(const S& sp, typename S::off_t pay, uint32_t ctr,
                                                    uint32_t (&raw)[17]) {
    load_raw<16>(sp, pay + kKsStride * (ctr > 0 ? ctr - 1 : 0), raw);
  }
  template <class S>
  static __device__ __forceinline__ void store_block(const S& sp, typename S::off_t pay, uint32_t ctr, uint32_t P,
                                                     const uint32_t (&ks)[16], const uint32_t (&raw)[17]) {
    const uint32_t o = kKsStride * (ctr - 1);
    xor_words<16>(sp, pay + o, ks, (int)min(64u, P - o), raw);
  }

  static __device__ __forceinline__ void store_otk(uint32_t* otk, const uint32_t (&ks)[16]) {
    *(uint4*)otk = make_uint4(ks[0], ks[1], ks[2], ks[3]);
    *(uint4*)(otk + 4) = make_uint4(ks[4], ks[5], ks[6], ks[7]);
  }

  // ChaChaHeaderProtection::mask (rustcrypto.rs:197-220): block(hp, ctr = sample[0..4] LE,
  // nonce = sample[4..16]); the mask is keystream bytes 0..4.
  static __device__ __forceinline__ void hp_mask_words(const uint32_t (&smp)[4], const KeyRow* row, uint32_t& m0,
                                                       uint32_t& m1) {
    uint32_t hk[8], blk[16];
    load_key8(row->hp, hk);
    chacha20_block(hk, smp[0], smp[1], smp[2], smp[3], blk);
    m0 = blk[0];
    m1 = blk[1];
  }
  template <class S>
  static __device__ __forceinline__ void hp_mask(const S& sp, typename S::off_t sample_at,
                                                 const KeyRow* row, uint32_t& m0, uint32_t& m1) {
    uint32_t smp[4];
    load_words<4>(sp, sample_at, smp);
    hp_mask_words(smp, row, m0, m1);
  }

  // send composite (transmit.rs:625-755): keystream block ctr of the packet runs on lane ctr % 8 in
  // iteration ctr / 8 (ctr 0 = the Poly1305 key); with the pool, blocks >= 16 and the
  // header-protection block (its sample is ciphertext of block 1) run in the workgroup's pool
  // before the MACs, and the mask is applied once the MAC has read the unprotected header.
  template <bool SINGLE, class S, class G, uint32_t IMG = kLdsBytes, uint32_t W = kCcWaves>
  static __device__ __forceinline__ void seal(const S& sp, typename S::off_t pkt, PktCtx& c, const KeyRow* row, int j,
                                              G& stg, const CcPool& pool) {
    const mq_pkt_desc& d = c.d;
    uint32_t key[8];
    load_key8(row->key, key);
    const uint32_t aad_len = c.act ? (uint32_t)d.pn_offset + d.pn_len : 0u;
    const uint32_t P = c.act ? d.len - aad_len - 16 : 0u;
    const typename S::off_t pay = pkt + aad_len;
    // DirectionalKeys::nonce (src/crypto/mod.rs:66-74): iv ^ (0^32 || BE64(pn))
    uint32_t n0 = row->iv[0], n1 = row->iv[1] ^ bswap32((uint32_t)(c.pn >> 32)), n2 = row->iv[2] ^ bswap32((uint32_t)c.pn);
#pragma unroll
    for (int k = 0; k < 8; ++k) pin(key[k]);
    pin(n0); pin(n1); pin(n2);
    stg.issue();  // packet bytes stream into LDS while the first keystream block is computed
    const uint32_t nblk = 1 + (P + 63) / 64;  // block 0 = Poly1305 key, 1.. = keystream
    const uint32_t kst = pool.on ? min(nblk, kCcPoolSlot) : nblk;  // blocks of this wave's own slots
    const uint32_t Imax = wave_max_u32(c.act ? (kst + kLanesPerPkt - 1) / kLanesPerPkt : 0u);
    for (uint32_t it = 0; it < Imax; ++it) {
      const uint32_t ctr = (uint32_t)j + kLanesPerPkt * it;
      const bool a = c.act && ctr < kst;
      uint32_t w[17];
      if (it > 0) load_block(sp, pay, a ? ctr : 0u, w);  // LDS reads in flight during the block function
      uint32_t ks[16];
      chacha20_block(key, ctr, n0, n1, n2, ks);
      if (it == 0) {
        stg.complete();
        MQ_STAMP(c.tile, 2);
        const bool rec = c.act && is_record(d);
        if (wave_any(rec)) {  // TLS record: header (AAD) and inner content type before any use
          if (rec && j == 0) write_record_header(sp, pkt, d);
          wave_sync();
        }
        load_block(sp, pay, a ? ctr : 0u, w);
      }
      if (a && ctr == 0) {
        store_otk(c.otk, ks);  // the Poly1305 key waits in LDS until the MAC
      } else if (a) {
        store_block(sp, pay, ctr, P, ks, w);
      }
      wave_sync();
    }
    if (Imax == 0) stg.complete();
    const bool hp = c.act && !(d.flags & MQ_PKT_NO_HP);  // records and plain AEAD rows have none
    // the pool takes the HP block when the sample (payload bytes [4 - pn_len, 20 - pn_len)) is all
    // ciphertext; for tiny payloads it reaches into the tag, which only the MAC below produces
    const bool hp_pool = pool.on && hp && P + d.pn_len >= 20u;
    if (j == 0) {  // pool record: keystream blocks >= 16 and the HP block
      const uint32_t np = pool.on && c.act && nblk > kCcPoolSlot ? nblk - kCcPoolSlot : 0u;
      const uint32_t hpn = hp_pool ? (uint32_t)d.pn_len : 0u;  // 1..4 (validated)
      pool.rec[0] = np | hpn << 8;
      if (np || hpn) {
        pool.rec[1] = (pool.base + (uint32_t)pay) | P << 17;
        pool.rec[3] = d.key_id;
        pool.rec[4] = n0; pool.rec[5] = n1; pool.rec[6] = n2;
      }
    }
    __syncthreads();  // every wave's records
    cc_pool_run<SINGLE, IMG, W>(pool);
    __syncthreads();  // every pooled block (and mask) is in place before any MAC reads it
    MQ_STAMP(c.tile, 3);
    uint32_t tag[4];
    poly_tag(sp, pkt, pay, aad_len, P, c.otk, j, c.act, tag);
    if (c.act && j == 0) store_words<4>(sp, pay + P, tag);
    // header protection (transmit.rs:713-738), now that the MAC has read the unprotected header
    uint32_t m0 = 0, m1 = 0;
    if (hp_pool) {
      m0 = pool.rec[2];
      m1 = pool.rec[7];
    }
    const bool late = hp && !hp_pool;  // direct path, or a sample that reaches into the tag
    if (wave_any(late)) {  // this wave computes those masks itself
      wave_sync();  // ciphertext and tags are in place
      uint32_t a0, a1;
      hp_mask(sp, pkt + d.pn_offset + 4, row, a0, a1);
      if (late) {
        m0 = a0;
        m1 = a1;
      }
    }
    if (hp && j == 0) apply_hp(sp, pkt, d, m0, m1);
    wave_sync();
    MQ_STAMP(c.tile, 4);
  }

  // receive composite (recv.rs:340-421 / 953-1025): HP removal, decode_pn, open.
  template <bool SINGLE, class S, class G, uint32_t IMG = kLdsBytes, uint32_t W = kCcWaves>
  static __device__ __forceinline__ void open(const S& sp, typename S::off_t pkt, PktCtx& c, const KeyRow* row, int j,
                              bool direct, G& stg, const CcPool& pool) {
    const mq_pkt_desc& d = c.d;
    stg.issue();
    uint32_t pn_len = d.pn_len, trunc = 0;
    uint8_t orig_b0 = 0, b0 = 0;
    uint32_t orig_pn = 0;
    const bool hp = c.act && !(d.flags & MQ_PKT_NO_HP);
    // recv.rs:363-395 / :968-997: mask, unmask byte 0, pn_len, unmask PN, decode_pn. With the
    // pre-pass (wave-uniform) those values arrive with the descriptor, so the nonce and the first
    // keystream block are computed while the packet is still landing in LDS.
    if (c.pre_hp) {
      if (hp) b0 = header_from_prepass(c, pn_len, trunc);
    } else {
      stg.complete();
      if (hp) {
        uint32_t m0, m1;
        hp_mask(sp, pkt + d.pn_offset + 4, row, m0, m1);
        b0 = header_from_mask(sp, pkt, c, m0, m1, pn_len, trunc);
      }
    }
    uint32_t key[8];
    load_key8(row->key, key);
    const uint32_t aad_len = c.act ? (uint32_t)d.pn_offset + pn_len : 0u;
    const uint32_t P = c.act ? d.len - aad_len - 16 : 0u;
    const typename S::off_t pay = pkt + aad_len;
    const uint32_t n0 = row->iv[0], n1 = row->iv[1] ^ bswap32((uint32_t)(c.pn >> 32)),
                   n2 = row->iv[2] ^ bswap32((uint32_t)c.pn);
    const uint32_t nblk = 1 + (P + 63) / 64;
    const uint32_t C = (nblk + kLanesPerPkt - 1) / kLanesPerPkt;
    const uint32_t Cmax = wave_max_u32(c.act ? C : 0u);
    // first keystream block of every lane is computed before the MAC (lane 0: one-time key)
    const uint32_t ctr0 = (uint32_t)j;
    uint32_t ks0[16];
    chacha20_block(key, ctr0, n0, n1, n2, ks0);
    if (c.pre_hp) stg.complete();
    MQ_STAMP(c.tile, 2);
    const bool hdr_written = hp && write_unmasked_header(sp, pkt, c, j, b0, pn_len, trunc, orig_b0, orig_pn);
    MQ_STAMP(c.tile, 3);
    if (c.act && j == 0) store_otk(c.otk, ks0);
    wave_sync();
    uint32_t tag[4], got[4];
    poly_tag(sp, pkt, pay, aad_len, P, c.otk, j, c.act, tag);
    load_words<4>(sp, pay + P, got);
    const uint32_t diff = (tag[0] ^ got[0]) | (tag[1] ^ got[1]) | (tag[2] ^ got[2]) | (tag[3] ^ got[3]);
    if (c.act && diff != 0) {  // Error::Crypto, buffer left as received
      c.st = MQ_ERR_CRYPTO;
      c.act = false;
    }
    wave_sync();  // every lane's MAC reads precede any plaintext write
    MQ_STAMP(c.tile, 4);
    if (c.act && ctr0 >= 1 && ctr0 < nblk) {
      uint32_t w[17];
      load_block(sp, pay, ctr0, w);
      store_block(sp, pay, ctr0, P, ks0, w);
    }
    const uint32_t Cown = pool.on ? min(Cmax, kCcOwnIters) : Cmax;  // later slots: the workgroup's pool
    for (uint32_t it = 1; it < Cown; ++it) {
      const uint32_t ctr = (uint32_t)j + kLanesPerPkt * it;
      const bool a = c.act && ctr < nblk;
      uint32_t w[17];
      load_block(sp, pay, a ? ctr : 0u, w);
      uint32_t ks[16];
      chacha20_block(key, ctr, n0, n1, n2, ks);
      if (a) store_block(sp, pay, ctr, P, ks, w);
    }
    if (j == 0) {  // pool record: only verified packets are decrypted (no HP block on open)
      const uint32_t np = pool.on && c.act && nblk > kCcPoolSlot ? nblk - kCcPoolSlot : 0u;
      pool.rec[0] = np;
      if (np) {
        pool.rec[1] = (pool.base + (uint32_t)pay) | P << 17;
        pool.rec[3] = d.key_id;
        pool.rec[4] = n0; pool.rec[5] = n1; pool.rec[6] = n2;
      }
    }
    __syncthreads();  // every wave's MAC has read its ciphertext
    cc_pool_run<SINGLE, IMG, W>(pool);
    __syncthreads();
    MQ_STAMP(c.tile, 5);
    if (direct && hdr_written && !c.act) {  // direct path writes HBM in place: undo the unmask
      sp.st8(pkt, orig_b0);
      for (uint32_t b = 0; b < pn_len; ++b) sp.st8(pkt + d.pn_offset + b, (uint8_t)(orig_pn >> (8 * b)));
    }
  }
};

// ---- narrow tiles: G lanes per packet, 64 / G packets per wave (r05) ---------------------------
// The octet tile gives every packet 8 lanes whatever its length. A 64-B packet needs 2 ChaCha20
// blocks (one-time key, one keystream block) and 5 MAC blocks, so 3/4 of its octet's keystream
// slots idle and the per-packet work (powers of r, the final multiply, the octet reduction, the
// header-protection block, descriptor and placement) is paid per 8 packets: flat 64-B batches ran
// at 122 GiB/s against 1034 at 1200 B. A narrow tile packs Q = 64 / G packets into
// the wave with G in {1, 2, 4} (G = 8: the octet layout without the keystream pool): keystream
// block c of a packet on group lane c % G in iteration c / G, the header-protection block as the
// packet's next slot when it falls in a later iteration than keystream block 1 (whose ciphertext
// is its sample), the MAC a G-way interleaved Horner (multiplier r^G, final r^(G-j), group sum).
// No LDS scratch: the one-time key travels by DPP from group lane 0, the mask stays in the
// registers of the lane that made it, so the whole 10 KiB minus a 64-B read slack holds images.
// Staging maps image chunk c (lane-linear LDS destination, as LDS-DMA requires) to its packet by a
// binary search over the tile's slots; write-back runs per packet, chunk j, j + G, ... on group
// lane j. Used by flat ChaCha20 batches of short packets (mq_launch_chacha picks the narrow kernel
// by the arena's bytes per packet) and by the short length classes of a mixed batch's ChaCha20 list
// (mq_partition.hip regions).
constexpr uint32_t kNarrowSlack = 64;                              // load_raw overreach past an image
constexpr uint32_t kNarrowChunks = (kLdsBytes - kNarrowSlack) / 16;  // 636

template <int G>
struct NarrowStager {
  static constexpr int Q = kWave / G;
  uint8_t* smem;
  const uint8_t* arena;
  uint64_t arena_len;
  uint32_t total;  // image chunks of the tile
  uint32_t slot;   // this lane's packet: first chunk (group-uniform)
  uint64_t base;   // its image start in the arena (16-B aligned)
  int lane;
  uint32_t nch;    // its image chunks (a gap may follow them: narrow_tile)
  uint32_t tail_c = 0xFFFFFFFFu;  // a chunk that would read past the arena end: guarded load
  uint64_t tail_src = 0;

  // the packet of image chunk c < total: the last q with slot_q <= c (an empty packet shares the
  // next one's slot; the later one of equal slots is the one with chunks)
  __device__ __forceinline__ uint32_t owner(uint32_t c) const {
    uint32_t q = 0;
#pragma unroll
    for (int step = Q / 2; step >= 1; step >>= 1) {
      const uint32_t v = (uint32_t)__shfl((int)slot, G * (int)(q + step), kWave);
      if (v <= c) q += step;
    }
    return q;
  }
  __device__ __forceinline__ void issue() {
#if MQ_PROF_SKIP & 8
    return;
#endif
    for (uint32_t k = 0; k < total; k += kWave) {  // wave-uniform
      const uint32_t c = k + (uint32_t)lane;
      const uint32_t q = owner(c < total ? c : 0u);
      const uint32_t sq = (uint32_t)__shfl((int)slot, G * (int)q, kWave);
      const uint64_t bq = (uint64_t)(uint32_t)__shfl((int)(uint32_t)(base >> 32), G * (int)q, kWave) << 32 |
                          (uint32_t)__shfl((int)(uint32_t)base, G * (int)q, kWave);
      const uint64_t src = bq + 16ull * (c - sq);
      const uint32_t nq = (uint32_t)__shfl((int)nch, G * (int)q, kWave);
      if (c < total && c - sq < nq) {  // not a gap chunk
        if (src + 16 <= arena_len)
          __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(arena + src),
                                           (__attribute__((address_space(3))) void*)(smem + 16u * k), 16, 0, 0);
        else {
          tail_c = c;
          tail_src = src;
        }
      }
    }
  }
  __device__ __forceinline__ void complete() {
    wave_sync();  // s_waitcnt vmcnt(0) covers the LDS-DMA writes
    if (tail_c != 0xFFFFFFFFu) *(uint4*)(smem + 16u * tail_c) = load_chunk_guarded(arena, tail_src, arena_len);
    wave_sync();
  }
};

// LDS -> HBM of a narrow tile's packets with write = 1: group lane j stores chunks j, j + G, ... of
// its packet, whole chunks with 16-B stores, the partial first / last chunk byte-exact (bytes of
// neighbouring packets are never touched)
template <int G>
__device__ __forceinline__ void narrow_stage_out(const uint8_t* smem, uint8_t* arena, int j, bool write,
                                                 const Placement& pl) {
#if MQ_PROF_SKIP & 4
  return;
#endif
  const uint32_t nch = write ? pl.nch() : 0u, head = pl.head();
  const uint32_t tail_end = ((head + pl.len - 1u) & 15u) + 1u;
  const uint32_t nmax = wave_max_any(nch);
  uint8_t* dst = arena + pl.base();
  const uint8_t* src = smem + 16u * pl.slot;
  for (uint32_t c = (uint32_t)j; c < nmax + (uint32_t)j; c += G) {  // wave-uniform trip count (nmax / G)
    if (c < nch) {
      const uint32_t lo = c == 0 ? head : 0u, hi = c + 1 == nch ? tail_end : 16u;
      const uint4 v = *(const uint4*)(src + 16u * c);
      if (lo == 0 && hi == 16) {
        *(uint4*)(dst + 16u * c) = v;
      } else {
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
        for (uint32_t b = lo; b < hi; ++b) dst[16u * c + b] = (uint8_t)(w[b >> 2] >> (8 * (b & 3)));
      }
    }
  }
}

// Poly1305 tag of a narrow tile's packet (poly_tag with G lanes): lane j takes MAC blocks
// G k + j - z, Horner with r^G, final multiply by r^(G - j), group sum. r, s: the one-time key.
template <int G, class S>
__device__ __forceinline__ void poly_tag_g(const S& sp, typename S::off_t pkt, typename S::off_t pay, uint32_t aad_len,
                                           uint32_t ct_len, const uint32_t (&rk)[4], const uint32_t (&s)[4], int j,
                                           bool act, uint32_t (&tag)[4]) {
#if MQ_PROF_SKIP & 2
  for (int w = 0; w < 4; ++w) tag[w] = s[w] ^ rk[w] ^ aad_len ^ ct_len;
  return;
#endif
  typedef Grp<G> Gp;
  const P26 r = p26_from_words(rk[0] & 0x0fffffffu, rk[1] & 0x0ffffffcu, rk[2] & 0x0ffffffcu, rk[3] & 0x0ffffffcu, 0);
  // powers: v = r^(j + 1) on group lane j; rG = r^G, rj = r^(G - j)
  P26 v = r, rG = r, rj = r;
  if (G >= 2) {
    P26 t = r;
    p26_mul(t, p26_mult(r));  // r^2
#pragma unroll
    for (int l = 0; l < 5; ++l) v.l[l] = (j & 1) ? t.l[l] : v.l[l];
    if (G >= 4) {
      P26 u = v;
      p26_mul(u, p26_mult(t));
#pragma unroll
      for (int l = 0; l < 5; ++l) v.l[l] = (j & 2) ? u.l[l] : v.l[l];
    }
    if (G == 8) {
      P26 r4, u = v;
#pragma unroll
      for (int l = 0; l < 5; ++l) r4.l[l] = oct_lane3(v.l[l]);
      p26_mul(u, p26_mult(r4));
#pragma unroll
      for (int l = 0; l < 5; ++l) v.l[l] = (j & 4) ? u.l[l] : v.l[l];
    }
#pragma unroll
    for (int l = 0; l < 5; ++l) {
      rG.l[l] = Gp::last(v.l[l]);
      rj.l[l] = Gp::mirror(v.l[l]);
    }
  }
  const P26m mG = p26_mult(rG), mlast = p26_mult(rj);
  const uint32_t A = (aad_len + 15) >> 4, T = (ct_len + 15) >> 4, nb = A + T + 1;
  const uint32_t K = (nb + G - 1) / G;
  const uint32_t Kmax = wave_max_any(act ? K : 0u);
  const int z = (int)(G * Kmax) - (int)nb;  // prepended zero blocks: every packet runs Kmax steps
  P26 acc;
#pragma unroll
  for (int l = 0; l < 5; ++l) acc.l[l] = 0;
  struct Blk { typename S::off_t src; int rem; bool pre, lens; };
  auto where = [&](int i) {
    Blk b;
    const bool aad = i < (int)A;
    b.pre = i < 0;
    b.lens = i == (int)(A + T);
    b.src = aad ? pkt + 16 * (uint32_t)max(i, 0) : pay + 16 * (uint32_t)(i - (int)A);
    b.rem = aad ? (int)aad_len - 16 * i : (int)ct_len - 16 * (i - (int)A);
    if (b.pre || b.lens) b.src = pkt;
    return b;
  };
  auto absorb = [&](const Blk& b, uint32_t (&m)[4]) {
    if (wave_any(act && (b.pre || b.lens || b.rem < 16))) {
#pragma unroll
      for (int w = 0; w < 4; ++w) m[w] &= byte_mask(b.pre ? 0 : b.rem, w);
      if (b.lens) { m[0] = aad_len; m[1] = 0; m[2] = ct_len; m[3] = 0; }
    }
    const P26 x = p26_from_words(m[0], m[1], m[2], m[3], b.pre ? 0u : 1u);
#pragma unroll
    for (int l = 0; l < 5; ++l) acc.l[l] += x.l[l];
  };
  if (Kmax > 0) {
    int i = j - z;
    Blk b = where(i);
    uint32_t m[4];
    load_words<4>(sp, b.src, m);
    const uint32_t sel_pay = sel_load((uint32_t)(pay & 3));
    const int ct_full_end = (int)A + (int)(ct_len >> 4);
    const int zA = (int)A + z;
    const uint32_t k_lo = act ? (uint32_t)((zA + G - 1) / G) : 0u;
    const int hi = ct_full_end + z - 2 * G + 1;  // lean iff G k + 2G - 1 - z < ct_full_end
    const uint32_t k_hi = !act ? 0xFFFFFFFFu : (hi <= 0 ? 0u : (uint32_t)((hi + G - 1) / G));
    const uint32_t klo = wave_max_any(k_lo), khi = min(wave_min_any(k_hi), Kmax - 1);
    for (uint32_t k = 0; k + 1 < Kmax; ++k) {
      if (k == klo && k < khi) {  // the lean stretch: only the block address advances
        typename S::off_t a = b.src & ~(typename S::off_t)3;
        uint32_t sel = sel_pay;
        pin(sel);
        for (; k < khi; ++k) {
          const P26 x = p26_from_words(m[0], m[1], m[2], m[3], 1u);
#pragma unroll
          for (int l = 0; l < 5; ++l) acc.l[l] += x.l[l];
          a += 16 * G;
          load_words_sel<4>(sp, a, sel, m);
          p26_mul(acc, mG);
        }
        const uint32_t nl = khi - klo;
        i += (int)(G * nl);
        b.src += 16 * G * nl;
        b.rem -= (int)(16 * G * nl);
        if (k + 1 >= Kmax) break;
      }
      absorb(b, m);
      const bool steady = !act || (i >= (int)A && i + G < ct_full_end);
      i += G;
      if (!wave_any(!steady)) {
        b.src += 16 * G;
        b.rem -= 16 * G;
        load_words_sel<4>(sp, b.src & ~(typename S::off_t)3, sel_pay, m);
      } else {
        b = where(i);
        load_words<4>(sp, b.src, m);
      }
      p26_mul(acc, mG);
    }
    absorb(b, m);
    p26_mul(acc, mlast);
  }
#pragma unroll
  for (int l = 0; l < 5; ++l) acc.l[l] = Gp::sum(acc.l[l]);
  p26_finish(acc, s, tag);
}

template <int G, bool SINGLE>
struct NarrowPolicy {
  typedef Grp<G> Gp;

  // the one-time key (block 0, group lane 0's keystream words 0..7) on every lane of the group
  static __device__ __forceinline__ void otk_bcast(const uint32_t (&otk)[8], uint32_t (&r)[4], uint32_t (&s)[4]) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      r[k] = Gp::bcast0(otk[k]);
      s[k] = Gp::bcast0(otk[4 + k]);
    }
  }

  // send composite (transmit.rs:625-755) on a narrow tile. Slot order: keystream blocks 1 .. nblk-1
  // first, the one-time key (block 0) in slot nblk - 1 — made last, so its 8 words are not held
  // through the loop — then the header-protection block in slot nblk.
  template <class S, class St>
  static __device__ __forceinline__ void seal(const S& sp, typename S::off_t pkt, PktCtx& c, const KeyRow* row, int j,
                                              St& stg) {
    const mq_pkt_desc& d = c.d;
    uint32_t key[8];
    load_key8(row->key, key);
    const uint32_t aad_len = c.act ? (uint32_t)d.pn_offset + d.pn_len : 0u;
    const uint32_t P = c.act ? d.len - aad_len - 16 : 0u;
    const typename S::off_t pay = pkt + aad_len;
    uint32_t n0 = row->iv[0], n1 = row->iv[1] ^ bswap32((uint32_t)(c.pn >> 32)), n2 = row->iv[2] ^ bswap32((uint32_t)c.pn);
    // retire the key loads before the LDS-DMA is issued (else the first wait covers the DMA too);
    // a single-key tile keeps its key in SGPRs
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (SINGLE) key[k] = __builtin_amdgcn_readfirstlane(key[k]);
      else pin(key[k]);
    }
    pin(n0); pin(n1); pin(n2);
    stg.issue();
    const uint32_t nblk = 1 + (P + 63) / 64;
    const bool hp = c.act && !(d.flags & MQ_PKT_NO_HP);
    // the header-protection block in slot nblk: its sample (payload [4 - pn_len, 20 - pn_len)) is
    // ciphertext of keystream block 1 (slot 0, iteration 0), so slot nblk must fall in a later
    // iteration (nblk >= G), and must not reach into the tag (only the MAC produces it)
    const bool hp_in = hp && P + d.pn_len >= 20u && nblk >= (uint32_t)G;
    const uint32_t S_ = nblk + (hp_in ? 1u : 0u);
    const uint32_t Imax = wave_max_any(c.act ? (S_ + G - 1) / G : 0u);
    uint32_t otk[8] = {0, 0, 0, 0, 0, 0, 0, 0}, m0 = 0, m1 = 0;
    for (uint32_t it = 0; it < Imax; ++it) {
      const uint32_t slot = (uint32_t)j + G * it;
      const bool is_otk = c.act && slot + 1 == nblk;
      const uint32_t ctr = is_otk ? 0u : slot + 1;  // keystream block of the slot
      const bool a = c.act && ctr < nblk;            // a keystream block (or the one-time key)
      const bool is_hp = hp_in && slot == nblk;
      uint32_t ks[16];
      if (wave_any(is_hp)) {  // the HP lanes run the HP key on the sample (ciphertext by now)
        uint32_t smp[4], kh[8], kk[8];
        load_words<4>(sp, is_hp ? pay + 4u - d.pn_len : pay, smp);
        load_key8(row->hp, kh);
#pragma unroll
        for (int k = 0; k < 8; ++k) kk[k] = is_hp ? kh[k] : key[k];
        chacha20_block(kk, is_hp ? smp[0] : ctr, is_hp ? smp[1] : n0, is_hp ? smp[2] : n1, is_hp ? smp[3] : n2, ks);
      } else {
        chacha20_block(key, ctr, n0, n1, n2, ks);
      }
      if (it == 0) {
        stg.complete();
        const bool rec = c.act && is_record(d);
        if (wave_any(rec)) {  // TLS record: header (AAD) and inner content type before any use
          if (rec && j == 0) write_record_header(sp, pkt, d);
          wave_sync();
        }
      }
      // the block's raw LDS words after the rounds (not in flight during them: 17 VGPRs fewer)
      uint32_t w[17];
      ChaChaPolicy::load_block(sp, pay, a && !is_otk ? ctr : 0u, w);
      if (is_otk) {
#pragma unroll
        for (int k = 0; k < 8; ++k) otk[k] = ks[k];
      } else if (a) {
        ChaChaPolicy::store_block(sp, pay, ctr, P, ks, w);
      }
      if (is_hp) {
        m0 = ks[0];
        m1 = ks[1];
      }
      wave_sync();
    }
    if (Imax == 0) stg.complete();
    // the one-time key from its group lane (nblk - 1) % G to the whole group
    uint32_t r[4], s[4], tag[4];
    const int src = (int)(threadIdx.x & (kWave - 1)) - j + (int)((nblk + G - 1) % G);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      r[k] = G == 1 ? otk[k] : (uint32_t)__shfl((int)otk[k], src, kWave);
      s[k] = G == 1 ? otk[4 + k] : (uint32_t)__shfl((int)otk[4 + k], src, kWave);
    }
    poly_tag_g<G>(sp, pkt, pay, aad_len, P, r, s, j, c.act, tag);
    if (c.act && j == 0) store_words<4>(sp, pay + P, tag);
    // header protection (transmit.rs:713-738), once the MAC has read the unprotected header
    const bool late = hp && !hp_in;  // tiny payloads and G > nblk: one more block for the wave
    if (wave_any(late)) {
      wave_sync();  // ciphertext and tags are in place
      uint32_t a0, a1;
      ChaChaPolicy::hp_mask(sp, pkt + d.pn_offset + 4, row, a0, a1);
      if (late) {
        m0 = a0;
        m1 = a1;
      }
    }
    const int jh = hp_in ? (int)(nblk % G) : 0;  // the group lane holding the mask
    wave_sync();
    if (hp && j == jh) apply_hp(sp, pkt, d, m0, m1);
    wave_sync();
  }

  // receive composite (recv.rs:340-421 / 953-1025) on a narrow tile: HP removal, decode_pn, verify,
  // then decrypt
  template <class S, class St>
  static __device__ __forceinline__ void open(const S& sp, typename S::off_t pkt, PktCtx& c, const KeyRow* row, int j,
                                              bool direct, St& stg) {
    const mq_pkt_desc& d = c.d;
    stg.issue();
    uint32_t pn_len = d.pn_len, trunc = 0;
    uint8_t orig_b0 = 0, b0 = 0;
    uint32_t orig_pn = 0;
    const bool hp = c.act && !(d.flags & MQ_PKT_NO_HP);
    if (c.pre_hp) {
      if (hp) b0 = header_from_prepass(c, pn_len, trunc);
    } else {
      stg.complete();
      if (wave_any(hp)) {  // every lane of a group computes its packet's mask (one block for the wave)
        uint32_t m0, m1;
        ChaChaPolicy::hp_mask(sp, hp ? pkt + d.pn_offset + 4 : pkt, row, m0, m1);
        if (hp) b0 = header_from_mask(sp, pkt, c, m0, m1, pn_len, trunc);
      }
    }
    uint32_t key[8];
    load_key8(row->key, key);
    const uint32_t aad_len = c.act ? (uint32_t)d.pn_offset + pn_len : 0u;
    const uint32_t P = c.act ? d.len - aad_len - 16 : 0u;
    const typename S::off_t pay = pkt + aad_len;
    const uint32_t n0 = row->iv[0], n1 = row->iv[1] ^ bswap32((uint32_t)(c.pn >> 32)),
                   n2 = row->iv[2] ^ bswap32((uint32_t)c.pn);
    const uint32_t nblk = 1 + (P + 63) / 64;
    const uint32_t Imax = wave_max_any(c.act ? (nblk + G - 1) / G : 0u);
    const uint32_t ctr0 = (uint32_t)j;  // iteration 0 before the MAC (group lane 0: the one-time key)
    uint32_t ks0[16];
    chacha20_block(key, ctr0, n0, n1, n2, ks0);
    if (c.pre_hp) stg.complete();
    const bool hdr_written = hp && write_unmasked_header(sp, pkt, c, j, b0, pn_len, trunc, orig_b0, orig_pn);
    wave_sync();
    uint32_t otk[8], r[4], s[4], tag[4], got[4];
#pragma unroll
    for (int k = 0; k < 8; ++k) otk[k] = ks0[k];
    otk_bcast(otk, r, s);
    poly_tag_g<G>(sp, pkt, pay, aad_len, P, r, s, j, c.act, tag);
    load_words<4>(sp, pay + P, got);
    const uint32_t diff = (tag[0] ^ got[0]) | (tag[1] ^ got[1]) | (tag[2] ^ got[2]) | (tag[3] ^ got[3]);
    if (c.act && diff != 0) {  // Error::Crypto, buffer left as received
      c.st = MQ_ERR_CRYPTO;
      c.act = false;
    }
    wave_sync();  // every lane's MAC reads precede any plaintext write
    if (c.act && ctr0 >= 1 && ctr0 < nblk) {
      uint32_t w[17];
      ChaChaPolicy::load_block(sp, pay, ctr0, w);
      ChaChaPolicy::store_block(sp, pay, ctr0, P, ks0, w);
    }
    for (uint32_t it = 1; it < Imax; ++it) {
      const uint32_t ctr = (uint32_t)j + G * it;
      const bool a = c.act && ctr < nblk;
      uint32_t w[17];
      ChaChaPolicy::load_block(sp, pay, a ? ctr : 0u, w);
      uint32_t ks[16];
      chacha20_block(key, ctr, n0, n1, n2, ks);
      if (a) ChaChaPolicy::store_block(sp, pay, ctr, P, ks, w);
    }
    wave_sync();
    if (direct && hdr_written && !c.act) {  // direct path writes HBM in place: undo the unmask
      sp.st8(pkt, orig_b0);
      for (uint32_t b = 0; b < pn_len; ++b) sp.st8(pkt + d.pn_offset + b, (uint8_t)(orig_pn >> (8 * b)));
    }
  }
};

// One narrow tile: entries [e0, e0 + Q) of the batch (index != null: of the list `index`, holes
// skipped; else descriptor indices), count = the entries' end. Every lane of the wave calls it.
template <int G, bool OPEN, bool SINGLE>
__device__ __forceinline__ void narrow_tile(uint8_t* wsm, const KeyRow* __restrict__ kt, uint32_t n_rows,
                                            uint8_t* __restrict__ arena, uint64_t arena_len,
                                            const mq_pkt_desc* __restrict__ desc, uint32_t e0, uint32_t count,
                                            const uint32_t* __restrict__ index, uint8_t* __restrict__ status,
                                            uint64_t* __restrict__ pn_out, const uint2* __restrict__ hpm) {
  constexpr int Q = kWave / G;
  const int lane = threadIdx.x & (kWave - 1), p = lane / G, j = lane % G;
  PktCtx c;
  const uint32_t e = e0 + (uint32_t)p;
  c.tile = e0 / Q;
  c.valid = e < count;
  c.i = c.valid ? (index ? index[e] : e) : 0u;
  if (c.i == kListHole) { c.valid = false; c.i = 0; }
  if (c.valid) {
    c.d = desc[c.i];
  } else {
    c.d.offset = 0; c.d.len = 0; c.d.key_id = 0; c.d.pn = 0; c.d.pn_offset = 0; c.d.pn_len = 0;
    c.d.flags = 0; c.d.reserved = 0;
  }
  c.pre_hp = OPEN && hpm != nullptr;
  c.hm0 = c.hm1 = 0;
  if (OPEN && hpm && c.valid) {
    const uint2 m = hpm[c.i];
    c.hm0 = m.x;
    c.hm1 = m.y;
  }
  c.st = c.valid ? validate<MQ_SUITE_CHACHA20, OPEN, SINGLE>(c.d, kt, n_rows, arena_len) : (int)MQ_ERR_INVALID_ARG;
  c.act = c.valid && c.st == MQ_OK;
  c.pn = c.d.pn;
  c.otk = nullptr;
  const KeyRow* row = SINGLE ? kt : kt + (c.act ? c.d.key_id : 0u);
  Placement pl;
  pl.off = c.act ? c.d.offset : 0;
  pl.len = c.act ? c.d.len : 0u;
  const uint64_t nch64 = c.act ? ((pl.off & 15) + (uint64_t)c.d.len + 15) >> 4 : 0u;
  const uint32_t nch = (uint32_t)(nch64 < 0xFFFFu ? nch64 : 0xFFFFu);
  // equal even image sizes (e.g. 256-B packets: 16 chunks) would put every packet's blocks on the
  // same LDS banks: a one-chunk gap after each image when packet 0's size is even and the budget
  // has room (as chacha_tile)
#ifndef MQ_CC_NOPAD  // diagnostic A/B build only: no gaps
  const uint32_t t0 = lane_u32(wave_incl_scan(j == 0 ? nch : 0u), kWave - 1);
  const uint32_t pad = (lane_u32(nch, 0) & 1u) == 0 && t0 + (uint32_t)Q <= kNarrowChunks ? 1u : 0u;
#else
  const uint32_t pad = 0;
#endif
  const uint32_t incl = pad ? wave_incl_scan(j == 0 ? nch + 1u : 0u) : wave_incl_scan(j == 0 ? nch : 0u);
  const uint32_t total = lane_u32(incl, kWave - 1);
  if (total <= kNarrowChunks) {
    pl.slot = incl - nch - pad;
    NarrowStager<G> stg{wsm, arena, arena_len, total, pl.slot, pl.base(), lane, nch};
    LdsSpace sp{wsm};
    const uint32_t pkt = pl.slot * 16u + pl.head();
    if (OPEN) NarrowPolicy<G, SINGLE>::template open<LdsSpace>(sp, pkt, c, row, j, false, stg);
    else NarrowPolicy<G, SINGLE>::template seal<LdsSpace>(sp, pkt, c, row, j, stg);
    wave_sync();
    narrow_stage_out<G>(wsm, arena, j, c.act, pl);
  } else {
    GlobalSpace sp{arena, arena_len};
    NoStager stg;
    if (OPEN) NarrowPolicy<G, SINGLE>::template open<GlobalSpace>(sp, pl.off, c, row, j, true, stg);
    else NarrowPolicy<G, SINGLE>::template seal<GlobalSpace>(sp, pl.off, c, row, j, stg);
  }
  tile_status<OPEN>(c, j, status, pn_out);
}

}  // namespace mq

using namespace mq;

// Tile kernels: one tile per wave, each with its private 10 KiB LDS image, kCcWaves-wave
// workgroups sharing the keystream pool above between two barriers. Every wave of a workgroup
// runs both barriers: waves past the batch with an empty record, direct-path tiles (images over
// the budget) with nothing pooled. (A persistent grid walking
// tiles, as the AES kernels use, measured 10 % slower here: identical waves stay in phase, so
// their staging waits line up.) The "1" variants are launched when the key table has a single
// row (every valid packet on row 0): key material then lives in SGPRs.
// tb: the workgroup's block of W tiles (blockIdx.x, or the persistent kernels' current block)
// tid: threadIdx.x (the persistent list kernels pass an opaque copy per tile, so nothing derived
// from it is hoisted out of their loop and held across every tile — that pressure spilled)
// A partition list's narrow regions (mq_partition.hip: reg = tiles of G = 8, 4, 2, 1, then the first
// entries of the G = 4, 2, 1 regions): list tile u >= T8 is narrow tile u - T8 of the G = 4 region,
// and so on. Runs it, if there is one.
template <bool OPEN, bool SINGLE>
__device__ __forceinline__ void chacha_narrow_list(uint8_t* wsm, uint32_t u, const uint32_t* __restrict__ reg,
                                                   const KeyRow* __restrict__ kt, uint32_t n_rows,
                                                   uint8_t* __restrict__ arena, uint64_t arena_len,
                                                   const mq_pkt_desc* __restrict__ desc,
                                                   const uint32_t* __restrict__ index, uint8_t* __restrict__ status,
                                                   uint64_t* __restrict__ pn_out, const uint2* __restrict__ hpm) {
  const uint32_t T8 = reg[0], T4 = reg[1], T2 = reg[2], T1 = reg[3], R4 = reg[4], R2 = reg[5], R1 = reg[6];
  if (u < T8) return;
  uint32_t v = u - T8;
  if (v < T4) {
    narrow_tile<4, OPEN, SINGLE>(wsm, kt, n_rows, arena, arena_len, desc, R4 + 16 * v, R4 + 16 * T4, index, status,
                                 pn_out, hpm);
    return;
  }
  v -= T4;
  if (v < T2) {
    narrow_tile<2, OPEN, SINGLE>(wsm, kt, n_rows, arena, arena_len, desc, R2 + 32 * v, R2 + 32 * T2, index, status,
                                 pn_out, hpm);
    return;
  }
  v -= T2;
  if (v < T1)
    narrow_tile<1, OPEN, SINGLE>(wsm, kt, n_rows, arena, arena_len, desc, R1 + 64 * v, R1 + 64 * T1, index, status,
                                 pn_out, hpm);
}

// LIST: a partition list with narrow regions (reg): the octet tiles are the G = 8 region's (count =
// its entries), a workgroup with an octet tile runs the pool's barriers on every wave (its narrow
// waves run their tile first), one without any runs its narrow tiles with no barrier.
template <bool OPEN, bool SINGLE, bool LIST = false, uint32_t IMG = kLdsBytes, uint32_t W = kCcWaves>
__device__ __forceinline__ void chacha_tile(uint32_t tb, uint32_t tid, const KeyRow* __restrict__ kt, uint32_t n_rows,
                                            uint8_t* __restrict__ arena, uint64_t arena_len,
                                            const mq_pkt_desc* __restrict__ desc, uint32_t n,
                                            const uint32_t* __restrict__ index, const uint32_t* __restrict__ n_dev,
                                            uint8_t* __restrict__ status, uint64_t* __restrict__ pn_out,
                                            const uint2* __restrict__ hpm, const uint32_t* __restrict__ reg = nullptr) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t w = tid >> 6;
  uint8_t* wsm = smem + w * IMG;
  const int lane = tid & (kWave - 1), p = lane / kLanesPerPkt, j = lane % kLanesPerPkt;
  const uint32_t tile_id = tb * W + w;
  PktCtx c;
  const KeyRow* row;
  constexpr uint32_t kBudget = IMG - kScratchBytes;  // packet images (9728 B at 10 KiB)
  CcPool pool{false, smem, w * IMG, (uint32_t*)(wsm + kBudget + 32u * (uint32_t)p), kt};
  if (LIST) {  // the octet region's entries
    n = kPktsPerTile * __builtin_amdgcn_readfirstlane(reg[0]);
    n_dev = nullptr;
  }
  if (!tile_ctx<MQ_SUITE_CHACHA20, OPEN, SINGLE>(tile_id, kt, n_rows, arena_len, desc, n, index, n_dev, hpm,
                                                 TilePrefetch{false, 0u, 0u}, c, row, tid)) {
    // past the batch (list capacities exceed the count): a whole workgroup leaves at once, a
    // wave of a live workgroup only joins its barriers and pool
    if (tb * W * kPktsPerTile >= (n_dev ? *n_dev : n)) {  // workgroup-uniform
      if (LIST) chacha_narrow_list<OPEN, SINGLE>(wsm, tile_id, reg, kt, n_rows, arena, arena_len, desc, index, status,
                                                 pn_out, hpm);
      return;
    }
    if (LIST) {  // this wave's narrow tile, before the barriers (its records are reset after it)
      chacha_narrow_list<OPEN, SINGLE>(wsm, tile_id, reg, kt, n_rows, arena, arena_len, desc, index, status, pn_out,
                                       hpm);
      wave_sync();
    }
    if (j == 0) pool.rec[0] = 0;
    __syncthreads();
    cc_pool_run<SINGLE, IMG, W>(pool, tid);
    __syncthreads();
    return;
  }
  MQ_STAMP(tile_id, 0);
  c.otk = (uint32_t*)(wsm + IMG - 32u * kPktsPerTile + 32u * (uint32_t)p);
  const uint64_t off = c.act ? c.d.offset : 0;
  Placement pl;
  pl.off = off;
  pl.len = c.act ? c.d.len : 0u;
  const uint64_t nch64 = c.act ? ((off & 15) + (uint64_t)c.d.len + 15) >> 4 : 0u;
  const uint32_t nch = (uint32_t)(nch64 < 0xFFFFu ? nch64 : 0xFFFFu);
  const uint32_t incl = oct_incl_scan(nch);
  const uint32_t total = lane_u32(incl, kWave - 1);
  // Packets of one even image size (lengths a multiple of 32 B at one alignment: 1600, 2048 B...)
  // start their images an even number of chunks apart, so the same keystream dword of every packet
  // sits on one LDS bank: 8-way conflicts in the XOR passes at 2048 B. A 16-B gap after each image
  // staggers them when the budget has room (r05; odd sizes such as config B's 75 chunks get none).
#ifndef MQ_CC_NOPAD  // diagnostic A/B build only: no gaps
  const uint32_t pad = (lane_u32(nch, 0) & 1u) == 0 && (total + kPktsPerTile) * 16u <= kBudget ? 1u : 0u;
#else
  const uint32_t pad = 0;
#endif
  if (total * 16u <= kBudget) {
    pl.slot = incl - nch + (uint32_t)p * pad;
    pool.on = true;
    DmaStager stg{wsm, arena, arena_len, lane, j, pl};
    LdsSpace sp{wsm};
    MQ_STAMP(tile_id, 1);
    const uint32_t pkt = pl.slot * 16u + pl.head();
    if (OPEN) ChaChaPolicy::template open<SINGLE, LdsSpace, DmaStager, IMG, W>(sp, pkt, c, row, j, false, stg, pool);
    else ChaChaPolicy::template seal<SINGLE, LdsSpace, DmaStager, IMG, W>(sp, pkt, c, row, j, stg, pool);
    MQ_STAMP(tile_id, 6);
    wave_sync();
    stage_out(wsm, arena, lane, c.act, pl);
    MQ_STAMP(tile_id, 7);
  } else {
    GlobalSpace sp{arena, arena_len};
    NoStager stg;
    if (OPEN) ChaChaPolicy::template open<SINGLE, GlobalSpace, NoStager, IMG, W>(sp, off, c, row, j, true, stg, pool);
    else ChaChaPolicy::template seal<SINGLE, GlobalSpace, NoStager, IMG, W>(sp, off, c, row, j, stg, pool);
  }
  tile_status<OPEN>(c, j, status, pn_out);
}

#define MQ_CHACHA_KERNELS(NAME_SEAL, NAME_OPEN, SINGLE)                                                   \
  extern "C" __global__ __launch_bounds__(64 * kCcWaves) __attribute__((amdgpu_waves_per_eu(4))) void NAME_SEAL( \
      const KeyRow* __restrict__ kt, uint32_t n_rows, uint8_t* __restrict__ arena, uint64_t arena_len,    \
      const mq_pkt_desc* __restrict__ desc, uint32_t n, const uint32_t* __restrict__ index,               \
      const uint32_t* __restrict__ n_dev, uint8_t* __restrict__ status) {                                 \
    chacha_tile<false, SINGLE>(blockIdx.x, threadIdx.x, kt, n_rows, arena, arena_len, desc, n, index, n_dev, status, nullptr, \
                               nullptr);                                                                  \
  }                                                                                                       \
  extern "C" __global__ __launch_bounds__(64 * kCcWaves) __attribute__((amdgpu_waves_per_eu(4))) void NAME_OPEN( \
      const KeyRow* __restrict__ kt, uint32_t n_rows, uint8_t* __restrict__ arena, uint64_t arena_len,    \
      const mq_pkt_desc* __restrict__ desc, uint32_t n, const uint32_t* __restrict__ index,               \
      const uint32_t* __restrict__ n_dev, uint8_t* __restrict__ status, uint64_t* __restrict__ pn_out,    \
      const uint2* __restrict__ hpm) {                                                                    \
    chacha_tile<true, SINGLE>(blockIdx.x, threadIdx.x, kt, n_rows, arena, arena_len, desc, n, index, n_dev, status, pn_out, hpm); \
  }
MQ_CHACHA_KERNELS(mq_chacha_seal_kernel, mq_chacha_open_kernel, false)
MQ_CHACHA_KERNELS(mq_chacha_seal1_kernel, mq_chacha_open1_kernel, true)

// Flat batches of long packets (r05): the same octet tiles and keystream pool with
// larger LDS images, so eight packets over ~1216 B stay staged instead of running on HBM (direct:
// 358-409 GiB/s at 1232-2048 B, against 1034 at 1200): 13 KiB per wave (4-wave workgroups, 12
// waves per CU: eight images of up to 100 chunks, packets up to ~1570 B at any alignment) or 20 KiB
// (8 waves per CU: 156 chunks, ~2480 B). The waves-per-EU hint gives them the registers of that
// occupancy. (Measured and dropped: 16 KiB in 2-wave workgroups, 10 waves per CU — the pool shared
// by two waves lost more than the occupancy gained: 1800 B 833 vs 945 GiB/s, gpurun_out/r05p.)
constexpr uint32_t kLongImg = 13312, kLongerImg = 20480;
static_assert(kCcWaves * kLongImg * 3 <= kCuLdsBytes && kCcWaves * kLongerImg * 2 <= kCuLdsBytes, "long images per CU");
#define MQ_CHACHA_LONG_KERNELS(NAME_SEAL, NAME_OPEN, SINGLE, IMG, WPE, W)                                   \
  extern "C" __global__ __launch_bounds__(64 * W) __attribute__((amdgpu_waves_per_eu(WPE))) void NAME_SEAL( \
      const KeyRow* __restrict__ kt, uint32_t n_rows, uint8_t* __restrict__ arena, uint64_t arena_len,    \
      const mq_pkt_desc* __restrict__ desc, uint32_t n, uint8_t* __restrict__ status) {                   \
    chacha_tile<false, SINGLE, false, IMG, W>(blockIdx.x, threadIdx.x, kt, n_rows, arena, arena_len, desc, n, nullptr, \
                                              nullptr, status, nullptr, nullptr);                         \
  }                                                                                                       \
  extern "C" __global__ __launch_bounds__(64 * W) __attribute__((amdgpu_waves_per_eu(WPE))) void NAME_OPEN( \
      const KeyRow* __restrict__ kt, uint32_t n_rows, uint8_t* __restrict__ arena, uint64_t arena_len,    \
      const mq_pkt_desc* __restrict__ desc, uint32_t n, uint8_t* __restrict__ status, uint64_t* __restrict__ pn_out, \
      const uint2* __restrict__ hpm) {                                                                    \
    chacha_tile<true, SINGLE, false, IMG, W>(blockIdx.x, threadIdx.x, kt, n_rows, arena, arena_len, desc, n, nullptr, \
                                             nullptr, status, pn_out, hpm);                               \
  }
MQ_CHACHA_LONG_KERNELS(mq_chacha_seal_long_kernel, mq_chacha_open_long_kernel, false, kLongImg, 3, kCcWaves)
MQ_CHACHA_LONG_KERNELS(mq_chacha_seal_long1_kernel, mq_chacha_open_long1_kernel, true, kLongImg, 3, kCcWaves)
MQ_CHACHA_LONG_KERNELS(mq_chacha_seal_longer_kernel, mq_chacha_open_longer_kernel, false, kLongerImg, 2, kCcWaves)
MQ_CHACHA_LONG_KERNELS(mq_chacha_seal_longer1_kernel, mq_chacha_open_longer1_kernel, true, kLongerImg, 2, kCcWaves)

// One-shot grids over a partition list with narrow regions (reg, mq_partition.hip): tile
// tb * W + w is an octet tile of the G = 8 region or a narrow tile after it
#define MQ_CHACHA_LGRID_KERNELS(NAME_SEAL, NAME_OPEN, SINGLE)                                             \
  extern "C" __global__ __launch_bounds__(64 * kCcWaves) __attribute__((amdgpu_waves_per_eu(4))) void NAME_SEAL( \
      const KeyRow* __restrict__ kt, uint32_t n_rows, uint8_t* __restrict__ arena, uint64_t arena_len,    \
      const mq_pkt_desc* __restrict__ desc, uint32_t n, const uint32_t* __restrict__ index,               \
      const uint32_t* __restrict__ reg, uint8_t* __restrict__ status) {                                   \
    chacha_tile<false, SINGLE, true>(blockIdx.x, threadIdx.x, kt, n_rows, arena, arena_len, desc, n, index, nullptr, \
                                     status, nullptr, nullptr, reg);                                      \
  }                                                                                                       \
  extern "C" __global__ __launch_bounds__(64 * kCcWaves) __attribute__((amdgpu_waves_per_eu(4))) void NAME_OPEN( \
      const KeyRow* __restrict__ kt, uint32_t n_rows, uint8_t* __restrict__ arena, uint64_t arena_len,    \
      const mq_pkt_desc* __restrict__ desc, uint32_t n, const uint32_t* __restrict__ index,               \
      const uint32_t* __restrict__ reg, uint8_t* __restrict__ status, uint64_t* __restrict__ pn_out,      \
      const uint2* __restrict__ hpm) {                                                                    \
    chacha_tile<true, SINGLE, true>(blockIdx.x, threadIdx.x, kt, n_rows, arena, arena_len, desc, n, index, nullptr, \
                                    status, pn_out, hpm, reg);                                            \
  }
MQ_CHACHA_LGRID_KERNELS(mq_chacha_seal_lgrid_kernel, mq_chacha_open_lgrid_kernel, false)
MQ_CHACHA_LGRID_KERNELS(mq_chacha_seal_lgrid1_kernel, mq_chacha_open_lgrid1_kernel, true)

// Partition lists (index != null) run on PERSISTENT workgroups (r04): the list's length is a
// device count, so a grid covering the list capacity (1.6 x the batch in tiles of W) was mostly
// workgroups that read the count and left — config E's ChaCha list has ~15k blocks of work in a
// 52k-block grid, and an empty receive pass spent 350 us dispatching its 32k blocks
// (profiles/r04g_kernel_stats_recv.csv). Here cus x 4 workgroups (16 waves per CU, as the
// one-shot grid) take blocks of W tiles: block blockIdx.x first, then blocks claimed from the
// stream's schedule slot (head 0, one returning atomic per block; the claim for the block after
// next is issued when a block starts and read when it ends, so nobody waits on it), or, without a
// slot, by stride. (Flat batches keep the one-shot grid: a persistent grid measured 10 % slower on
// config B, r02 — identical waves stay in phase and their staging waits line up.)
// SINGLE: the list's packets share one key row (kt points at it)
template <bool OPEN, bool SINGLE>
__device__ __forceinline__ void chacha_list(const KeyRow* __restrict__ kt, uint32_t n_rows, uint8_t* __restrict__ arena,
                                            uint64_t arena_len, const mq_pkt_desc* __restrict__ desc, uint32_t n,
                                            const uint32_t* __restrict__ index, const uint32_t* __restrict__ n_dev,
                                            uint8_t* __restrict__ status, uint64_t* __restrict__ pn_out,
                                            const uint2* __restrict__ hpm, uint32_t* __restrict__ sched,
                                            const uint32_t* __restrict__ reg) {
  constexpr uint32_t W = kCcWaves;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  // the next block goes to every wave through word 7 of wave 0's first pool record, free between
  // tiles (the pool writes it only after the next tile's first barrier); the four 40-KiB
  // workgroups of a CU leave no LDS byte for a variable of its own
  uint32_t* next_slot = (uint32_t*)(smem + kDataBudget) + 7;
  uint32_t tb = blockIdx.x, pend = 0;
  if (threadIdx.x == 0 && sched) pend = __hip_atomic_fetch_add(sched, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  (void)reg;  // the receive passes' partitions have no narrow regions (mq_partition.hip, skip_unkeyed)
  for (;;) {
    const uint32_t count = n_dev ? *n_dev : n;
    if (tb * W * kPktsPerTile >= count) break;  // workgroup-uniform
    uint32_t tid = threadIdx.x;
    // open: an opaque copy per tile (chacha_tile) — 10 spilled VGPRs to 2; seal spills more with it
    // (9 to 24), so it keeps the plain index there
    if (OPEN) asm volatile("" : "+v"(tid));
    // single-key seal: the key table pointer opaque per tile too, so its key words are loaded per
    // tile rather than held in SGPRs across the loop (spilled 29 VGPRs)
    const KeyRow* ktt = kt;
    if (SINGLE && !OPEN) asm volatile("" : "+s"(ktt));
    chacha_tile<OPEN, SINGLE>(tb, tid, ktt, n_rows, arena, arena_len, desc, n, index, n_dev, status, pn_out, hpm);
    __syncthreads();  // every wave is done with the tile and its scratch
    if (threadIdx.x == 0) *next_slot = sched ? gridDim.x + pend : tb + gridDim.x;
    __syncthreads();
    tb = (uint32_t)__builtin_amdgcn_readfirstlane((int)*next_slot);  // uniform: keeps tile indexing scalar
    // the claim after this one: its result is used one block later (issued after the barrier, so
    // no barrier waits for it until the next tile's first one)
    if (threadIdx.x == 0 && sched) pend = __hip_atomic_fetch_add(sched, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // the last claim is never used, but it must have returned before sched_done can zero head 0
  // (ADVICE r04): consuming its value makes thread 0 wait for it whatever the barrier lowers to
  if (threadIdx.x == 0) asm volatile("" ::"v"(pend));
  __syncthreads();
  sched_done(sched);
}
// The "1" list kernels: every packet of the list is on one key row (the key table has a single
// non-AES row, mq_host.cpp), kt points at it, so key material is wave-uniform, in SGPRs, as in the
// flat single-key kernels.
#define MQ_CHACHA_LIST_KERNELS(NAME_SEAL, NAME_OPEN, SINGLE)                                                \
  extern "C" __global__ __launch_bounds__(64 * kCcWaves) __attribute__((amdgpu_waves_per_eu(4))) void NAME_SEAL( \
      const KeyRow* __restrict__ kt, uint32_t n_rows, uint8_t* __restrict__ arena, uint64_t arena_len,     \
      const mq_pkt_desc* __restrict__ desc, uint32_t n, const uint32_t* __restrict__ index,                \
      const uint32_t* __restrict__ n_dev, uint8_t* __restrict__ status, uint32_t* __restrict__ sched,      \
      const uint32_t* __restrict__ reg) {                                                                  \
    chacha_list<false, SINGLE>(kt, n_rows, arena, arena_len, desc, n, index, n_dev, status, nullptr, nullptr, sched, reg); \
  }                                                                                                        \
  extern "C" __global__ __launch_bounds__(64 * kCcWaves) __attribute__((amdgpu_waves_per_eu(4))) void NAME_OPEN( \
      const KeyRow* __restrict__ kt, uint32_t n_rows, uint8_t* __restrict__ arena, uint64_t arena_len,     \
      const mq_pkt_desc* __restrict__ desc, uint32_t n, const uint32_t* __restrict__ index,                \
      const uint32_t* __restrict__ n_dev, uint8_t* __restrict__ status, uint64_t* __restrict__ pn_out,     \
      const uint2* __restrict__ hpm, uint32_t* __restrict__ sched, const uint32_t* __restrict__ reg) {   \
    chacha_list<true, SINGLE>(kt, n_rows, arena, arena_len, desc, n, index, n_dev, status, pn_out, hpm, sched, reg); \
  }
MQ_CHACHA_LIST_KERNELS(mq_chacha_seal_list_kernel, mq_chacha_open_list_kernel, false)
MQ_CHACHA_LIST_KERNELS(mq_chacha_seal_list1_kernel, mq_chacha_open_list1_kernel, true)

// Flat batches of short packets (r05): one wave per 64 consecutive descriptors. The wave sizes
// its 64 images and takes the narrowest lane group whose rounds fit the LDS image: G = 1 (one
// round of 64 packets), 2 (two of 32), 4 (four of 16) or 8 (eight of 8, the octet layout without
// the pool); a round over the budget runs on HBM (direct). No barriers: every wave is independent.
template <bool OPEN, bool SINGLE>
__device__ __forceinline__ void chacha_narrow_flat(const KeyRow* __restrict__ kt, uint32_t n_rows,
                                                   uint8_t* __restrict__ arena, uint64_t arena_len,
                                                   const mq_pkt_desc* __restrict__ desc, uint32_t n,
                                                   uint8_t* __restrict__ status, uint64_t* __restrict__ pn_out,
                                                   const uint2* __restrict__ hpm) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t w = wave_id();
  uint8_t* wsm = smem + w * kLdsBytes;
  const uint32_t e0 = (blockIdx.x * kCcWaves + w) * (uint32_t)kWave;
  if (e0 >= n) return;
  const uint32_t lane = threadIdx.x & (kWave - 1), e = e0 + lane;
  uint32_t nch = 0;
  if (e < n) {  // offset and length only; validity is the tile's business (an over-count is harmless)
    const uint32_t* dw = reinterpret_cast<const uint32_t*>(desc + e);
    const uint64_t x = ((dw[0] & 15u) + (uint64_t)dw[2] + 15u) >> 4;
    nch = (uint32_t)(x < 0xFFFFu ? x : 0xFFFFu);
  }
  const uint32_t incl = wave_incl_scan(nch);
  auto fits = [&](uint32_t Q) -> bool {  // every round of Q packets within the budget (uniform)
    for (uint32_t r = 0; r < (uint32_t)kWave / Q; ++r) {
      const uint32_t hi = lane_u32(incl, (int)(r * Q + Q - 1)), lo = r ? lane_u32(incl, (int)(r * Q - 1)) : 0u;
      if (hi - lo > kNarrowChunks) return false;
    }
    return true;
  };
#ifdef MQ_NARROW_ONLY  // register-pressure diagnostic: one lane group only
  (void)fits;
  for (uint32_t r = 0; r < MQ_NARROW_ONLY; ++r)
    narrow_tile<MQ_NARROW_ONLY, OPEN, SINGLE>(wsm, kt, n_rows, arena, arena_len, desc, e0 + 64 / MQ_NARROW_ONLY * r, n,
                                              nullptr, status, pn_out, hpm);
  return;
#endif
  if (fits(64)) {
    narrow_tile<1, OPEN, SINGLE>(wsm, kt, n_rows, arena, arena_len, desc, e0, n, nullptr, status, pn_out, hpm);
  } else if (fits(32)) {
    for (uint32_t r = 0; r < 2; ++r)
      narrow_tile<2, OPEN, SINGLE>(wsm, kt, n_rows, arena, arena_len, desc, e0 + 32 * r, n, nullptr, status, pn_out, hpm);
  } else if (fits(16)) {
    for (uint32_t r = 0; r < 4; ++r)
      narrow_tile<4, OPEN, SINGLE>(wsm, kt, n_rows, arena, arena_len, desc, e0 + 16 * r, n, nullptr, status, pn_out, hpm);
  } else {
    for (uint32_t r = 0; r < 8; ++r)
      narrow_tile<8, OPEN, SINGLE>(wsm, kt, n_rows, arena, arena_len, desc, e0 + 8 * r, n, nullptr, status, pn_out, hpm);
  }
}
#define MQ_CHACHA_NARROW_KERNELS(NAME_SEAL, NAME_OPEN, SINGLE)                                                \
  extern "C" __global__ __launch_bounds__(64 * kCcWaves) __attribute__((amdgpu_waves_per_eu(4))) void NAME_SEAL( \
      const KeyRow* __restrict__ kt, uint32_t n_rows, uint8_t* __restrict__ arena, uint64_t arena_len,        \
      const mq_pkt_desc* __restrict__ desc, uint32_t n, uint8_t* __restrict__ status) {                       \
    chacha_narrow_flat<false, SINGLE>(kt, n_rows, arena, arena_len, desc, n, status, nullptr, nullptr);       \
  }                                                                                                           \
  extern "C" __global__ __launch_bounds__(64 * kCcWaves) __attribute__((amdgpu_waves_per_eu(4))) void NAME_OPEN( \
      const KeyRow* __restrict__ kt, uint32_t n_rows, uint8_t* __restrict__ arena, uint64_t arena_len,        \
      const mq_pkt_desc* __restrict__ desc, uint32_t n, uint8_t* __restrict__ status, uint64_t* __restrict__ pn_out, \
      const uint2* __restrict__ hpm) {                                                                        \
    chacha_narrow_flat<true, SINGLE>(kt, n_rows, arena, arena_len, desc, n, status, pn_out, hpm);             \
  }
MQ_CHACHA_NARROW_KERNELS(mq_chacha_seal_narrow_kernel, mq_chacha_open_narrow_kernel, false)
MQ_CHACHA_NARROW_KERNELS(mq_chacha_seal_narrow1_kernel, mq_chacha_open_narrow1_kernel, true)

// ---- fused send composite (mq_batch_protect with the ChaCha20 suite hint, r04) -----------------
// build + seal + header protection in one pass: the tile's eight packets are BUILT from their
// requests straight into the wave's LDS image (layout from mq_build.h, the frames at any alignment
// with unaligned 16-B loads, header / PN / PADDING / tag-room chunks byte-wise), sealed there by the
// same ChaChaPolicy::seal as a staged batch, and written to `out` once. The two-kernel composite
// (mq_build_kernel, then the seal kernel over its descriptors) moved every packet through HBM twice:
// written by the build, read back and rewritten by the seal — 4.9 GB per 2^20 x 1200 B against the
// 2.4 GB of frames in and packets out here. Tiles whose images exceed the LDS budget build in HBM
// (the build kernel's stores) and seal there (direct path). Statuses and lengths as the composite:
// the build's status when it fails (pkt_len = `needed` or 0), else the seal's.
#ifndef MQ_PROTECT_BATCH
#define MQ_PROTECT_BATCH 5
#endif
constexpr uint32_t kProtectBatch = MQ_PROTECT_BATCH;  // image chunks per lane whose loads fly together (5:
                                                      // no spills beside the seal state; 8 or 10 spill)

template <bool SINGLE>
__device__ __forceinline__ void chacha_protect_tile(uint32_t tb, const KeyRow* __restrict__ kt, uint32_t n_rows,
                                                    const mq_conn_send* __restrict__ conns, uint32_t n_conns,
                                                    const uint8_t* __restrict__ frames, uint64_t frames_len,
                                                    uint8_t* __restrict__ out, uint64_t out_len,
                                                    const mq_send_req* __restrict__ req, uint32_t n,
                                                    uint32_t suite_hint, uint8_t* __restrict__ status,
                                                    uint32_t* __restrict__ pkt_len) {
  constexpr uint32_t W = kCcWaves;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t w = threadIdx.x >> 6;
  uint8_t* wsm = smem + w * kLdsBytes;
  const int lane = threadIdx.x & (kWave - 1), p = lane / kLanesPerPkt, j = lane % kLanesPerPkt;
  const uint32_t tile_id = tb * W + w;
  CcPool pool{false, smem, w * kLdsBytes, (uint32_t*)(wsm + kDataBudget + 32u * (uint32_t)p), kt};
  const uint32_t tile0 = tile_id * kPktsPerTile;
  if (tile0 >= n) {  // a wave past the batch in a live workgroup joins the barriers and the pool
    if (j == 0) pool.rec[0] = 0;
    __syncthreads();
    cc_pool_run<SINGLE>(pool);
    __syncthreads();
    return;
  }
  PktCtx c;
  c.tile = tile_id;
  c.i = tile0 + (uint32_t)p;
  c.valid = c.i < n;
  c.pre_hp = false;
  c.hm0 = c.hm1 = 0;
  const BuildLayout b = build_layout(c.i, c.valid, kt, n_rows, conns, n_conns, frames_len, out_len, req, suite_hint);
  c.d = b.d;
  c.pn = b.pn;
  if (!c.valid || b.st != MQ_OK) c.st = c.valid ? b.st : (int)MQ_ERR_INVALID_ARG;
  else c.st = validate<MQ_SUITE_CHACHA20, false, SINGLE>(c.d, kt, n_rows, out_len);
  c.act = c.valid && c.st == MQ_OK;
  const KeyRow* row = SINGLE ? kt : kt + (c.act ? c.d.key_id : 0u);
  c.otk = (uint32_t*)(wsm + kLdsBytes - 32u * kPktsPerTile + 32u * (uint32_t)p);
  Placement pl;
  pl.off = c.act ? c.d.offset : 0;
  pl.len = c.act ? c.d.len : 0u;
  const uint64_t nch64 = c.act ? ((pl.off & 15) + (uint64_t)c.d.len + 15) >> 4 : 0u;
  const uint32_t nch = (uint32_t)(nch64 < 0xFFFFu ? nch64 : 0xFFFFu);
  const uint32_t incl = oct_incl_scan(nch);
  const uint32_t total = lane_u32(incl, kWave - 1);
  const uint8_t* fr = frames + b.frames_offset;
  if (total * 16u <= kDataBudget) {
    pl.slot = incl - nch;
    pool.on = true;
    // the image: chunk k holds packet bytes [16k - head, 16k - head + 16); lane j builds k = j,
    // j + 8, ... (kProtectBatch chunks' loads issued before any of their LDS stores)
    uint8_t* img = wsm + 16u * pl.slot;
    const int head = (int)pl.head();
    for (uint32_t k0 = (uint32_t)j; k0 < nch; k0 += kLanesPerPkt * kProtectBatch) {
      uint4 v[kProtectBatch];
#pragma unroll
      for (uint32_t t = 0; t < kProtectBatch; ++t) {
        const uint32_t k = k0 + kLanesPerPkt * t;
        const int x0 = 16 * (int)k - head;
        const bool whole = k < nch && x0 >= (int)b.hp && (uint32_t)x0 + 16u <= b.hp + b.m;
#if MQ_PROF_SKIP & 512  // phase-cost diagnostic: no frames loads
        v[t] = make_uint4(x0, 0, 0, 0);
#else
        v[t] = whole ? ld16(fr + ((uint32_t)x0 - b.hp)) : make_uint4(0, 0, 0, 0);
#endif
      }
#pragma unroll
      for (uint32_t t = 0; t < kProtectBatch; ++t) {
        const uint32_t k = k0 + kLanesPerPkt * t;
        const int x0 = 16 * (int)k - head;
        const bool whole = x0 >= (int)b.hp && (uint32_t)x0 + 16u <= b.hp + b.m;
        const bool zero = x0 >= (int)(b.hp + b.m);  // PADDING / tag room (and bytes past the packet)
        if (k < nch && (whole || zero)) *(uint4*)(img + 16u * k) = v[t];
      }
    }
    // edge chunks, byte-wise, outside the unrolled batch: those holding header / PN bytes, and the
    // one where the frames end mid-chunk
    const uint32_t kh = (uint32_t)(head + (int)b.hp + 15) >> 4, fe = (uint32_t)head + b.hp + b.m;
#if !(MQ_PROF_SKIP & 256)  // phase-cost diagnostic: no edge chunks
    // their frames bytes first (one guarded 16-B load each, zeros elsewhere), then the header and PN
    // bytes on top, eight per lane from the connection row's words: r04's first version built
    // each edge chunk byte by byte on one lane, a dependent load per byte (0.12 of its 1.40 ms,
    // profiles/r04n_protect_phases.txt)
    for (uint32_t k = (uint32_t)j; k < kh && k < nch; k += kLanesPerPkt)
      *(uint4*)(img + 16u * k) = edge_frames(b, fr, 16 * (int)k - head, b.frames_offset, frames_len);
    if ((fe & 15u) && (fe >> 4) >= kh && (fe >> 4) < nch && ((fe >> 4) & (kLanesPerPkt - 1)) == (uint32_t)j)
      *(uint4*)(img + 16u * (fe >> 4)) = edge_frames(b, fr, 16 * (int)(fe >> 4) - head, b.frames_offset, frames_len);
    if (c.act && 8u * (uint32_t)j < b.hp) {
      HeaderLane hl;
      hl.load(b.cp, b.level, j);
      uint8_t* hd = img + head;
#pragma unroll
      for (uint32_t u = 0; u < 8; ++u) {
        const uint32_t x = 8u * (uint32_t)j + u;
        if (x < b.hp)
          hd[x] = x < b.hdr ? hl.byte(b.level, b.pn_len, b.payload_length, x, u)
                            : (uint8_t)(b.pn >> (8 * (b.pn_len - 1 - (x - b.hdr))));
      }
    }
#endif
    LdsSpace sp{wsm};
    NoStager stg;  // complete(): the wave's image stores are done before any lane reads the image
    ChaChaPolicy::template seal<SINGLE, LdsSpace>(sp, pl.slot * 16u + pl.head(), c, row, j, stg, pool);
    wave_sync();
    stage_out(wsm, out, lane, c.act, pl);
  } else {
    if (c.act) build_store<kProtectBatch>(b, j, frames, out);
    wave_sync();  // the packets are in HBM before the seal reads them
    GlobalSpace sp{out, out_len};
    NoStager stg;
    ChaChaPolicy::template seal<SINGLE, GlobalSpace>(sp, c.act ? c.d.offset : 0, c, row, j, stg, pool);
  }
  if (c.valid && j == 0) {
    status[c.i] = (uint8_t)c.st;
    pkt_len[c.i] = (b.st != MQ_OK || c.st == MQ_OK) ? b.len_out : 0u;
  }
}

#define MQ_CHACHA_PROTECT_KERNEL(NAME, SINGLE)                                                             \
  extern "C" __global__ __launch_bounds__(64 * kCcWaves) __attribute__((amdgpu_waves_per_eu(4))) void NAME( \
      const KeyRow* __restrict__ kt, uint32_t n_rows, const mq_conn_send* __restrict__ conns, uint32_t n_conns, \
      const uint8_t* __restrict__ frames, uint64_t frames_len, uint8_t* __restrict__ out, uint64_t out_len,   \
      const mq_send_req* __restrict__ req, uint32_t n, uint32_t suite_hint, uint8_t* __restrict__ status,     \
      uint32_t* __restrict__ pkt_len) {                                                                       \
    chacha_protect_tile<SINGLE>(blockIdx.x, kt, n_rows, conns, n_conns, frames, frames_len, out, out_len, req, n, \
                                suite_hint, status, pkt_len);                                                 \
  }
MQ_CHACHA_PROTECT_KERNEL(mq_chacha_protect_kernel, false)
MQ_CHACHA_PROTECT_KERNEL(mq_chacha_protect1_kernel, true)

extern "C" __global__ __launch_bounds__(256) void mq_chacha_hp_kernel(
    const KeyRow* __restrict__ kt, uint32_t n_rows, const uint32_t* __restrict__ key_ids,
    const uint8_t* __restrict__ samples, uint8_t* __restrict__ masks, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t kid = key_ids[i];
  if (kid >= n_rows || kt[kid].suite != MQ_SUITE_CHACHA20) {
    // rows of neither suite (bad key id, empty row): all-zero mask (include/mq_aead.h); AES
    // rows are the AES kernel's
    if (kid >= n_rows || kt[kid].suite != MQ_SUITE_AES128GCM)
      for (int b = 0; b < 5; ++b) masks[5 * (size_t)i + b] = 0;
    return;
  }
  GlobalSpace sp{const_cast<uint8_t*>(samples), (uint64_t)n * 16};
  uint32_t m0, m1;
  ChaChaPolicy::hp_mask(sp, (uint64_t)i * 16, kt + kid, m0, m1);
  for (int b = 0; b < 4; ++b) masks[5 * (size_t)i + b] = (uint8_t)(m0 >> (8 * b));
  masks[5 * (size_t)i + 4] = (uint8_t)m1;
}

// Open pre-pass: ChaChaHeaderProtection::mask of every packet's sample, one packet per lane, so
// the tile kernel spends no keystream slot of its octet on it. DECODE (the batch open path):
// store the unmasked first byte and truncated PN (prepass_decode) instead of the raw mask
// (which mq_recv.hip's planner consumes).
template <bool DECODE>
__global__ __launch_bounds__(256) void mq_chacha_open_hp_kernel(
    const KeyRow* __restrict__ kt, uint32_t n_rows, const uint8_t* __restrict__ arena, uint64_t arena_len,
    const mq_pkt_desc* __restrict__ desc, uint32_t n, const uint32_t* __restrict__ index,
    const uint32_t* __restrict__ n_dev, uint2* __restrict__ hpm) {
  uint32_t i;
  const KeyRow* row;
  uint64_t at;
  mq_pkt_desc d;
  if (!prepass_pick(blockIdx.x * blockDim.x + threadIdx.x, MQ_SUITE_CHACHA20, kt, n_rows, arena_len, desc, n,
                    index, n_dev, i, row, at, d))
    return;
  GlobalSpace sp{const_cast<uint8_t*>(arena), arena_len};
  uint32_t m0, m1;
  if (DECODE) {  // PN bytes and sample (contiguous) and the first byte in one round of loads
    uint32_t w[5];
    uint8_t b0;
    prepass_header(arena, d, b0, w);
    const uint32_t smp[4] = {w[1], w[2], w[3], w[4]};
    ChaChaPolicy::hp_mask_words(smp, row, m0, m1);
    hpm[i] = prepass_decode_words(b0, w[0], d, m0, m1);
  } else {
    ChaChaPolicy::hp_mask(sp, at, row, m0, m1);
    hpm[i] = make_uint2(m0, m1);
  }
}

// ---- host-side launchers (called from mq_host.cpp) -------------------------------------------
// index != null (a partition list, length on the device): the persistent list kernels, cus x 4
// workgroups, sched = the stream's schedule slot (null: static stride)
// Flat batches (no partition list): the kernel family from the batch's bytes per packet `bpp` —
// the caller's length hint (MQ_BATCH_LEN_HINT), else arena_len / n. 0: narrow tiles (a batch
// averaging at most 640 B per packet: short packets, G = 8 / 4 / 2 / 1 lanes chosen per wave;
// configs B and E never), 1: octet tiles over 10-KiB images (config B: 1200), 2: 13-KiB images (eight
// images over 1216 B), 3: 20-KiB images (over 1584 B). Tiles whose images overflow the kernel's LDS
// image take the direct HBM path: right, only slower.
int mq_chacha_flat_kind(uint64_t bpp) {
  constexpr uint64_t kNarrowAvg = 640, kLongAvg0 = 1216, kLongAvg1 = 1584;
  return bpp <= kNarrowAvg ? 0 : bpp <= kLongAvg0 ? 1 : bpp <= kLongAvg1 ? 2 : 3;
}

hipError_t mq_launch_chacha(bool open, const KeyRow* kt, uint32_t n_rows, uint8_t* arena,
                            uint64_t arena_len, const mq_pkt_desc* desc, uint32_t n,
                            const uint32_t* index, const uint32_t* n_dev, uint8_t* status,
                            uint64_t* pn_out, uint2* hpm, bool own_hp, hipStream_t s, int cus, uint32_t* sched,
                            int64_t single_row, bool persistent, const uint32_t* reg, uint64_t bpp) {
  const uint32_t tiles = (n + kPktsPerTile - 1) / kPktsPerTile;
  if (tiles == 0) return hipSuccess;
  if (open && hpm && own_hp) {  // !own_hp: mq_launch_mixed_hp covers both suites' lists
    hipLaunchKernelGGL(mq_chacha_open_hp_kernel<true>, dim3((n + 255) / 256), dim3(256), 0, s, kt, n_rows, arena,
                       arena_len, desc, n, index, n_dev, hpm);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  const uint32_t blocks = (tiles + kCcWaves - 1) / kCcWaves;
  // Lists run on the persistent grid when asked for (the receive composite's passes: an empty
  // list then costs 1024 workgroups, not a grid over the list capacity), else on the one-shot grid,
  // which measured 1.1 % faster on config E (r04q: 557.9 vs 551.6 GiB/s, three alternating runs).
  // MQ_CC_LIST=0 / 1 (diagnostic, mq_opts.h: tests run both grids on one batch) forces either.
  const long forced = mq::opt(mq::Opt::CcList);
  if (forced >= 0) persistent = forced != 0;
  // single_row >= 0: every packet of the list is on that row (the single-key kernels)
  const bool one = index && single_row >= 0 && (uint64_t)single_row < n_rows;
  const KeyRow* kl = one ? kt + single_row : kt;
  if (index && persistent) {
    const uint32_t per = (uint32_t)(cus > 0 ? cus : 256) * 4u, grid = blocks < per ? blocks : per;
    if (open)
      hipLaunchKernelGGL(one ? mq_chacha_open_list1_kernel : mq_chacha_open_list_kernel, dim3(grid),
                         dim3(kWave * kCcWaves), kLdsBytes * kCcWaves, s, kl, n_rows, arena, arena_len, desc, n, index,
                         n_dev, status, pn_out, hpm, sched, reg);
    else
      hipLaunchKernelGGL(one ? mq_chacha_seal_list1_kernel : mq_chacha_seal_list_kernel, dim3(grid),
                         dim3(kWave * kCcWaves), kLdsBytes * kCcWaves, s, kl, n_rows, arena, arena_len, desc, n, index,
                         n_dev, status, sched, reg);
    return hipGetLastError();
  }
  if (index) {  // one-shot grid over the list capacity (every region's tiles fit: a tile holds >= 8 entries)
    if (open)
      hipLaunchKernelGGL(one ? mq_chacha_open_lgrid1_kernel : mq_chacha_open_lgrid_kernel, dim3(blocks),
                         dim3(kWave * kCcWaves), kLdsBytes * kCcWaves, s, kl, n_rows, arena, arena_len, desc, n, index,
                         reg, status, pn_out, hpm);
    else
      hipLaunchKernelGGL(one ? mq_chacha_seal_lgrid1_kernel : mq_chacha_seal_lgrid_kernel, dim3(blocks),
                         dim3(kWave * kCcWaves), kLdsBytes * kCcWaves, s, kl, n_rows, arena, arena_len, desc, n, index,
                         reg, status);
    return hipGetLastError();
  }
  // Flat batches: the kernel family from the bytes per packet (mq_chacha_flat_kind). MQ_CC_NARROW=0 / 1
  // and MQ_CC_LONG=0 / 1 / 2 (diagnostic, mq_opts.h: tests run several kernels on one batch) force
  // the wide / narrow kernels and the 10-, 13- or 20-KiB images.
  if (!index) {
    const int kind = mq_chacha_flat_kind(bpp);
    bool narrow = kind == 0;
    const long fn = mq::opt(mq::Opt::CcNarrow);
    if (fn >= 0) narrow = fn == 1;
    if (narrow) {
      const uint32_t nb = (uint32_t)(((uint64_t)n + kWave * kCcWaves - 1) / (kWave * kCcWaves));
      if (open)
        hipLaunchKernelGGL(n_rows == 1 ? mq_chacha_open_narrow1_kernel : mq_chacha_open_narrow_kernel, dim3(nb),
                           dim3(kWave * kCcWaves), kLdsBytes * kCcWaves, s, kt, n_rows, arena, arena_len, desc, n,
                           status, pn_out, hpm);
      else
        hipLaunchKernelGGL(n_rows == 1 ? mq_chacha_seal_narrow1_kernel : mq_chacha_seal_narrow_kernel, dim3(nb),
                           dim3(kWave * kCcWaves), kLdsBytes * kCcWaves, s, kt, n_rows, arena, arena_len, desc, n,
                           status);
      return hipGetLastError();
    }
    int img = kind >= 2 ? kind - 1 : 0;  // 0: 10 KiB, 1: 13 KiB, 2: 20 KiB
    const long fl = mq::opt(mq::Opt::CcLong);
    if (fl >= 0) img = fl >= 2 ? 2 : (int)fl;
    const bool o1 = n_rows == 1;
    if (img) {
      const uint32_t lds = (img == 2 ? kLongerImg : kLongImg) * kCcWaves;
      if (open)
        hipLaunchKernelGGL(img == 2 ? (o1 ? mq_chacha_open_longer1_kernel : mq_chacha_open_longer_kernel)
                                    : (o1 ? mq_chacha_open_long1_kernel : mq_chacha_open_long_kernel),
                           dim3(blocks), dim3(kWave * kCcWaves), lds, s, kt, n_rows, arena, arena_len, desc, n, status,
                           pn_out, hpm);
      else
        hipLaunchKernelGGL(img == 2 ? (o1 ? mq_chacha_seal_longer1_kernel : mq_chacha_seal_longer_kernel)
                                    : (o1 ? mq_chacha_seal_long1_kernel : mq_chacha_seal_long_kernel),
                           dim3(blocks), dim3(kWave * kCcWaves), lds, s, kt, n_rows, arena, arena_len, desc, n, status);
      return hipGetLastError();
    }
  }
  if (open)
    hipLaunchKernelGGL(n_rows == 1 || one ? mq_chacha_open1_kernel : mq_chacha_open_kernel, dim3(blocks),
                       dim3(kWave * kCcWaves), kLdsBytes * kCcWaves, s, kl, n_rows, arena, arena_len, desc, n, index,
                       n_dev, status, pn_out, hpm);
  if (open) return hipGetLastError();
  // seal: header protection runs inside the tile kernel (the pool's HP blocks, cc_pool_run)
  hipLaunchKernelGGL(n_rows == 1 || one ? mq_chacha_seal1_kernel : mq_chacha_seal_kernel, dim3(blocks),
                     dim3(kWave * kCcWaves), kLdsBytes * kCcWaves, s, kl, n_rows, arena, arena_len, desc, n, index,
                     n_dev, status);
  return hipGetLastError();
}

hipError_t mq_launch_chacha_protect(const KeyRow* kt, uint32_t n_rows, const mq_conn_send* conns, uint32_t n_conns,
                                    const uint8_t* frames, uint64_t frames_len, uint8_t* out, uint64_t out_len,
                                    const mq_send_req* req, uint32_t n, uint32_t suite_hint, uint8_t* status,
                                    uint32_t* pkt_len, hipStream_t s) {
  const uint32_t tiles = (n + kPktsPerTile - 1) / kPktsPerTile;
  if (tiles == 0) return hipSuccess;
  const uint32_t blocks = (tiles + kCcWaves - 1) / kCcWaves;
  hipLaunchKernelGGL(n_rows == 1 ? mq_chacha_protect1_kernel : mq_chacha_protect_kernel, dim3(blocks),
                     dim3(kWave * kCcWaves), kLdsBytes * kCcWaves, s, kt, n_rows, conns, n_conns, frames, frames_len,
                     out, out_len, req, n, suite_hint, status, pkt_len);
  return hipGetLastError();
}

// header-protection masks of the ChaCha20 rows of `desc` only (mq_recv.hip plans with them)
hipError_t mq_launch_chacha_prepass(const KeyRow* kt, uint32_t n_rows, const uint8_t* arena, uint64_t arena_len,
                                    const mq_pkt_desc* desc, uint32_t n, uint2* hpm, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(mq_chacha_open_hp_kernel<false>, dim3((n + 255) / 256), dim3(256), 0, s, kt, n_rows, arena, arena_len,
                     desc, n, (const uint32_t*)nullptr, (const uint32_t*)nullptr, hpm);
  return hipGetLastError();
}

hipError_t mq_launch_chacha_hp(const KeyRow* kt, uint32_t n_rows, const uint32_t* key_ids,
                               const uint8_t* samples, uint8_t* masks, uint32_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(mq_chacha_hp_kernel, dim3((n + 255) / 256), dim3(256), 0, s, kt, n_rows, key_ids,
                     samples, masks, n);
  return hipGetLastError();
}

#ifdef MQ_STAMPS
void mq_stamps_set_chacha(uint64_t* p) { (void)hipMemcpyToSymbol(HIP_SYMBOL(mq_stamp_buf), &p, sizeof p); }
#endif
