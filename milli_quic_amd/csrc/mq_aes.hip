// mq_aes.hip — AEAD_AES_128_GCM packet protection (SP 800-38D, RFC 9001 §5) on gfx950.
//
// Replaces, per packet of a batch, the reference's Aes128GcmAead::seal_in_place /
// open_in_place (src/crypto/rustcrypto.rs:38-94) and AesHeaderProtection::mask (:175-186),
// composed as in src/connection/transmit.rs:499-755 and src/connection/recv.rs:340-421,953-1025.
//
// gfx950 has no AES or carry-less-multiply instructions, so:
//   * AES-128 rounds use the wide T-table (T0 and T2, 32 replicas each, 64 KiB per workgroup,
//     mq_aes.h): one v_perm_b32 per lookup address, conflict-free ds_read_b32, one rotation per
//     round column; round keys in SGPRs (single-key kernels) or VGPRs;
//   * GHASH: in the single-key kernels every Horner step's multiply by H^8 is 32 table reads
//     (mq_aes.h gh_mul_tab, built per workgroup from H^8); the final multiply by H^(8-j) and all
//     multiplies of the multi-key kernels use the bit-holed integer product (gf_mul).
// Workgroups of kAesWaves waves are persistent (one per CU, LDS-bound), so the 72 KiB of tables
// are built once per CU and each wave walks tiles w, w + stride, ...
// Work split per tile (mq_tile.h): keystream block b of a packet (b = 0: E_K(J0), b >= 1:
// counter b+1) on lane b % 8; GHASH interleaved over the octet with H^8 (precomputed on the
// host per key) and a final multiply by H^(8-j).
#include "mq_aes.h"
#include "mq_tile.h"

#include <cstdlib>

namespace mq {

// Interleaved GHASH over AAD||pad||CT||pad||[len(A)]64||[len(C)]64 (bit lengths): lane j takes
// blocks 8k + j with multiplier H^8, then one final multiply by H^(8-j) (row->H[7-j], computed on
// the host per key), then the octet XOR. Every lane of the octet returns the same value
// (reflected basis). The H^8 multiplies go through the LDS table in the single-key kernels (TAB)
// and, in the multi-key kernels, in waves whose active packets all use the table's row
// (g_aes_hot_row); otherwise through the bit-holed integer product.
template <bool TAB, class S>
__device__ __forceinline__ void ghash_impl(const S& sp, typename S::off_t pkt, typename S::off_t pay,
                                           uint32_t aad_len, uint32_t ct_len, const KeyRow* row, int j,
                                           bool act, uint32_t (&y)[4]) {
#if MQ_PROF_SKIP & 2
  for (int w = 0; w < 4; ++w) y[w] = row->H[0][w] ^ aad_len ^ ct_len;
  return;
#endif
  uint32_t hp[4];
  GfOp m8, mlast;
  {
    if (!TAB) {
#pragma unroll
      for (int w = 0; w < 4; ++w) hp[w] = brev(row->H[7][w]);
      m8 = gf_prepare(hp);
    }
    const int e = 7 - j;  // H^(8-j)
#pragma unroll
    for (int w = 0; w < 4; ++w) hp[w] = brev(row->H[e][w]);
    mlast = gf_prepare(hp);
  }
  const uint32_t A = (aad_len + 15) >> 4, T = (ct_len + 15) >> 4, nb = A + T + 1;
  const uint32_t K = (nb + kLanesPerPkt - 1) / kLanesPerPkt;
  const uint32_t Kmax = wave_max_u32(act ? K : 0u);
  const int z = (int)(kLanesPerPkt * Kmax) - (int)nb;
  uint32_t acc[4] = {0, 0, 0, 0};
  struct Blk { typename S::off_t src; int rem; bool lens; };
  auto where = [&](uint32_t k) {
    const int i = (int)(kLanesPerPkt * k) + j - z;
    Blk b{pkt, 0, false};
    if (act && i >= 0) {
      if ((uint32_t)i < A) {
        b.src = pkt + 16 * (uint32_t)i; b.rem = (int)aad_len - 16 * i;
      } else if ((uint32_t)i < A + T) {
        b.src = pay + 16 * ((uint32_t)i - A); b.rem = (int)ct_len - 16 * (i - (int)A);
      } else {
        b.lens = true;
      }
    }
    return b;
  };
  auto absorb = [&](const Blk& b, uint32_t (&m)[4]) {
#pragma unroll
    for (int w = 0; w < 4; ++w) m[w] = refl(m[w] & byte_mask(b.rem, w));
    if (b.lens) {
      const uint64_t ab = (uint64_t)aad_len * 8, cb = (uint64_t)ct_len * 8;
      m[0] = brev((uint32_t)(ab >> 32)); m[1] = brev((uint32_t)ab);
      m[2] = brev((uint32_t)(cb >> 32)); m[3] = brev((uint32_t)cb);
    }
#pragma unroll
    for (int w = 0; w < 4; ++w) acc[w] ^= m[w];
  };
  if (Kmax > 0) {
    Blk b = where(0);
    uint32_t m[4];
    load_words<4>(sp, b.src, m);
    for (uint32_t k = 0; k + 1 < Kmax; ++k) {
      absorb(b, m);
      b = where(k + 1);
      load_words<4>(sp, b.src, m);
      if (TAB) gh_mul_tab(acc);
      else gf_mul(acc, m8);
    }
    absorb(b, m);
    gf_mul(acc, mlast);
  }
#pragma unroll
  for (int w = 0; w < 4; ++w) y[w] = oct_xor(acc[w]);
}

// Two instantiations, so that a wave holds the registers of one multiply method only.
template <bool TAB, class S>
__device__ __forceinline__ void ghash(const S& sp, typename S::off_t pkt, typename S::off_t pay,
                                      uint32_t aad_len, uint32_t ct_len, const KeyRow* row, int j,
                                      bool act, uint32_t (&y)[4]) {
  if (TAB || (g_aes_hot_row != nullptr && !wave_any(act && row != g_aes_hot_row)))
    ghash_impl<true>(sp, pkt, pay, aad_len, ct_len, row, j, act, y);
  else
    ghash_impl<false>(sp, pkt, pay, aad_len, ct_len, row, j, act, y);
}

// TAB: single-key kernel with the GHASH table of H^8 in LDS
template <bool TAB>
struct AesPolicyT {
  static constexpr uint32_t kSuite = MQ_SUITE_AES128GCM;

  // keystream of block index b (0: E(J0), b >= 1: counter b + 1) as little-endian data words
  static __device__ __forceinline__ void ctr_block(const AesRk& rk, const TwLane& rb, const uint32_t (&nb)[3],
                                                   uint32_t b, uint32_t (&ks)[4]) {
    uint32_t s0 = nb[0], s1 = nb[1], s2 = nb[2], s3 = b == 0 ? 1u : b + 1;
    aes128_block(rk, rb, s0, s1, s2, s3);
    ks[0] = bswap32(s0); ks[1] = bswap32(s1); ks[2] = bswap32(s2); ks[3] = bswap32(s3);
  }

  // blocks b and b + 8 (the lane's next iteration) at once
  static __device__ __forceinline__ void ctr_block2(const AesRk& rk, const TwLane& rb, const uint32_t (&nb)[3],
                                                    uint32_t b, uint32_t (&ks)[4], uint32_t (&ks2)[4]) {
    uint32_t x[4] = {nb[0], nb[1], nb[2], b == 0 ? 1u : b + 1};
    uint32_t y[4] = {nb[0], nb[1], nb[2], b + kLanesPerPkt + 1};
    aes128_block2(rk, rb, x, y);
#pragma unroll
    for (int q = 0; q < 4; ++q) { ks[q] = bswap32(x[q]); ks2[q] = bswap32(y[q]); }
  }

  // the same from the packet's CTR cache (every counter of the wave's packets < 256)
  static __device__ __forceinline__ void ctr_block2c(const AesRk& rk, const TwLane& rb, const AesCtrCache& cc,
                                                     uint32_t b, uint32_t (&ks)[4], uint32_t (&ks2)[4]) {
    uint32_t x[4], y[4];
    aes128_ctr2(rk, rb, cc, b == 0 ? 1u : b + 1, b + kLanesPerPkt + 1, x, y);
#pragma unroll
    for (int q = 0; q < 4; ++q) { ks[q] = bswap32(x[q]); ks2[q] = bswap32(y[q]); }
  }
  static __device__ __forceinline__ void ctr_blockc(const AesRk& rk, const TwLane& rb, const AesCtrCache& cc,
                                                    uint32_t b, uint32_t (&ks)[4]) {
    uint32_t x[4];
    aes128_ctr1(rk, rb, cc, b == 0 ? 1u : b + 1, x);
#pragma unroll
    for (int q = 0; q < 4; ++q) ks[q] = bswap32(x[q]);
  }

  template <class S>
  static __device__ __forceinline__ void xor_block(const S& sp, typename S::off_t pay, uint32_t b,
                                                   uint32_t P, const uint32_t (&ks)[4]) {
    const uint32_t o = 16 * (b - 1);
    const int ln = (int)min(16u, P - o);
    uint32_t raw[5];
    load_raw<4>(sp, pay + o, raw);
    xor_words<4>(sp, pay + o, ks, ln, raw);
  }

  // AesHeaderProtection::mask (rustcrypto.rs:175-186): AES-ECB(hp, sample)[0..5]
  // (rb: TwLane in the tile kernels, the small table's replica offset in the per-lane kernels)
  template <class T>
  static __device__ __forceinline__ void hp_mask_words(const uint32_t (&smp)[4], const KeyRow* row, const T& rb,
                                                       uint32_t& m0, uint32_t& m1) {
    AesRk hk;
    load_rk(row->hp_rk, hk);
    uint32_t s0 = bswap32(smp[0]), s1 = bswap32(smp[1]), s2 = bswap32(smp[2]), s3 = bswap32(smp[3]);
    aes128_block(hk, rb, s0, s1, s2, s3);
    m0 = bswap32(s0);
    m1 = s1 >> 24;
  }
  template <class S, class T>
  static __device__ __forceinline__ void hp_mask(const S& sp, typename S::off_t sample_at,
                                                 const KeyRow* row, const T& rb, uint32_t& m0, uint32_t& m1) {
    uint32_t smp[4];
    load_words<4>(sp, sample_at, smp);
    AesRk hk;
    load_rk(row->hp_rk, hk);
    uint32_t s0 = bswap32(smp[0]), s1 = bswap32(smp[1]), s2 = bswap32(smp[2]), s3 = bswap32(smp[3]);
    aes128_block(hk, rb, s0, s1, s2, s3);
    m0 = bswap32(s0);
    m1 = s1 >> 24;
  }

  static __device__ __forceinline__ void nonce_be(const KeyRow* row, uint64_t pn, uint32_t (&nb)[3]) {
    // DirectionalKeys::nonce (src/crypto/mod.rs:66-74), as big-endian AES input words
    nb[0] = bswap32(row->iv[0]);
    nb[1] = bswap32(row->iv[1]) ^ (uint32_t)(pn >> 32);
    nb[2] = bswap32(row->iv[2]) ^ (uint32_t)pn;
  }

  static __device__ __forceinline__ void tag_words(const uint32_t (&y)[4], const uint32_t (&ej0)[4],
                                                   uint32_t (&tag)[4]) {
#pragma unroll
    for (int w = 0; w < 4; ++w) tag[w] = bswap32(brev(y[w])) ^ ej0[w];
  }

  template <class S>
  static __device__ __forceinline__ void apply_hp(const S& sp, typename S::off_t pkt, const mq_pkt_desc& d,
                                                  uint32_t m0, uint32_t m1) {
    const uint8_t fb = (d.flags & MQ_PKT_LONG_HEADER) ? 0x0f : 0x1f;
    sp.st8(pkt, sp.ld8(pkt) ^ ((uint8_t)m0 & fb));
    const uint32_t mk = (m0 >> 8) | (m1 << 24);
    for (uint32_t b = 0; b < d.pn_len; ++b)
      sp.st8(pkt + d.pn_offset + b, sp.ld8(pkt + d.pn_offset + b) ^ (uint8_t)(mk >> (8 * b)));
  }

  // send composite: CTR block b (0 = E_K(J0)) on lane b % 8 in iteration b / 8; the HP block runs
  // in the first free slot after the blocks holding the sample (b = 1, 2), or in a separate phase
  // when the sample reaches into the tag.
  template <class S, class G>
  static __device__ __forceinline__ void seal(const S& sp, typename S::off_t pkt, PktCtx& c, const KeyRow* row, int j, G& stg) {
    const mq_pkt_desc& d = c.d;
    const TwLane rb = tw_lane();
    const uint32_t aad_len = c.act ? (uint32_t)d.pn_offset + d.pn_len : 0u;
    const uint32_t P = c.act ? d.len - aad_len - 16 : 0u;
    const typename S::off_t pay = pkt + aad_len;
    uint32_t nb[3];
    nonce_be(row, c.pn, nb);
    const uint32_t nblk = 1 + (P + 15) / 16;
    const bool hp_on = c.act && !(d.flags & MQ_PKT_NO_HP);
    const bool hp_post = hp_on && 20 > P + d.pn_len;
    uint32_t hp_it = nblk / kLanesPerPkt, hp_lane = nblk % kLanesPerPkt;
    if (hp_it == 0) { hp_it = 1; hp_lane = 0; }
    const uint32_t iters = max((nblk + kLanesPerPkt - 1) / kLanesPerPkt, (hp_on && !hp_post) ? hp_it + 1 : 0u);
    const uint32_t Imax = wave_max_u32(c.act ? iters : 0u);
    uint32_t ej0[4] = {0, 0, 0, 0};
    uint32_t m0 = 0, m1 = 0;
    bool have_mask = false;
    {
      AesRk rk;
      load_rk(row->aes_rk, rk);
#pragma unroll
      for (int k = 0; k < 44; ++k) pin(rk.w[k]);
      pin(nb[0]); pin(nb[1]); pin(nb[2]);
      stg.issue();
      // CTR cache while the packets land in LDS (counters of every active packet < 256)
      const bool cached = !wave_any(c.act && nblk > 255u);
      AesCtrCache cc{};
      if (cached) cc = ctr_cache(rk, rb, nb);
      auto first_iter = [&]() {  // before any packet byte is touched
        stg.complete();
        MQ_STAMP(c.tile, 2);
        const bool rec = c.act && is_record(d);
        if (wave_any(rec)) {  // TLS record: header (AAD) and inner content type before any use
          if (rec && j == 0) write_record_header(sp, pkt, d);
          wave_sync();
        }
      };
      auto use_block = [&](uint32_t b, const uint32_t (&ks)[4]) {
        if (c.act && b < nblk) {
          if (b == 0) {
#pragma unroll
            for (int k = 0; k < 4; ++k) ej0[k] = ks[k];
          } else {
            xor_block(sp, pay, b, P, ks);
          }
        }
      };
      uint32_t it = 0;
      while (it < Imax) {
        const uint32_t b = (uint32_t)j + kLanesPerPkt * it;
        const bool is_hp = hp_on && !hp_post && it == hp_it && (uint32_t)j == hp_lane;
        const bool hp_next = hp_on && !hp_post && it + 1 == hp_it && (uint32_t)j == hp_lane;
        // iterations it and it + 1 together unless either carries an HP block (its sample is
        // ciphertext of iteration 0, and its lane needs the HP key)
        if (it + 1 < Imax && !wave_any(is_hp || hp_next)) {
          uint32_t ks[4], ks2[4];
          if (cached) ctr_block2c(rk, rb, cc, b, ks, ks2);
          else ctr_block2(rk, rb, nb, b, ks, ks2);
          if (it == 0) first_iter();
          use_block(b, ks);
          use_block(b + kLanesPerPkt, ks2);
          wave_sync();
          it += 2;
          continue;
        }
        uint32_t ks[4];
        if (wave_any(is_hp)) {  // iteration carrying HP blocks: per-lane key/input
          AesRk hk;
          load_rk(row->hp_rk, hk);
          uint32_t smp[4];
          load_words<4>(sp, pkt + (c.act ? d.pn_offset + 4u : 0u), smp);
#pragma unroll
          for (int k = 0; k < 44; ++k) hk.w[k] = is_hp ? hk.w[k] : rk.w[k];
          uint32_t s0 = nb[0], s1 = nb[1], s2 = nb[2], s3 = b == 0 ? 1u : b + 1;
          if (is_hp) { s0 = bswap32(smp[0]); s1 = bswap32(smp[1]); s2 = bswap32(smp[2]); s3 = bswap32(smp[3]); }
          aes128_block(hk, rb, s0, s1, s2, s3);
          ks[0] = bswap32(s0); ks[1] = bswap32(s1); ks[2] = bswap32(s2); ks[3] = bswap32(s3);
          if (is_hp) { m0 = ks[0]; m1 = s1 >> 24; have_mask = true; }
        } else if (cached) {
          ctr_blockc(rk, rb, cc, b, ks);
        } else {
          ctr_block(rk, rb, nb, b, ks);
        }
        if (it == 0) first_iter();
        if (!is_hp) use_block(b, ks);
        wave_sync();  // this iteration's ciphertext (the HP sample) is visible to the next
        it += 1;
      }
      if (Imax == 0) stg.complete();
    }
    MQ_STAMP(c.tile, 3);
#pragma unroll
    for (int k = 0; k < 4; ++k) ej0[k] = oct_bcast0(ej0[k]);
    uint32_t y[4], tag[4];
    ghash<TAB>(sp, pkt, pay, aad_len, P, row, j, c.act, y);
    tag_words(y, ej0, tag);
    if (c.act && j == 0) store_words<4>(sp, pay + P, tag);
    wave_sync();
    MQ_STAMP(c.tile, 4);
    if (wave_any(hp_post)) {
      uint32_t t0, t1;
      hp_mask(sp, pkt + (c.act ? d.pn_offset + 4u : 0u), row, rb, t0, t1);
      if (hp_post && j == 0) { m0 = t0; m1 = t1; have_mask = true; }
    }
    if (have_mask) apply_hp(sp, pkt, d, m0, m1);
    MQ_STAMP(c.tile, 5);
  }

  template <class S, class G>
  static __device__ __forceinline__ void open(const S& sp, typename S::off_t pkt, PktCtx& c, const KeyRow* row, int j,
                              bool direct, G& stg) {
    const mq_pkt_desc& d = c.d;
    stg.issue();
    const TwLane rb = tw_lane();
    uint32_t pn_len = d.pn_len, trunc = 0;
    uint8_t orig_b0 = 0, b0 = 0;
    uint32_t orig_pn = 0;
    const bool hp = c.act && !(d.flags & MQ_PKT_NO_HP);
    // header (recv.rs:363-395): from the pre-pass values when present (wave-uniform), so that
    // in the single-key kernels the nonce and the first CTR block are computed while the packet
    // is still landing in LDS
    if (c.pre_hp) {
      if (hp) b0 = header_from_prepass(c, pn_len, trunc);
    } else {
      stg.complete();
      if (hp) {
        uint32_t m0, m1;
        hp_mask(sp, pkt + d.pn_offset + 4, row, rb, m0, m1);
        b0 = header_from_mask(sp, pkt, c, m0, m1, pn_len, trunc);
      }
    }
    const uint32_t aad_len = c.act ? (uint32_t)d.pn_offset + pn_len : 0u;
    const uint32_t P = c.act ? d.len - aad_len - 16 : 0u;
    const typename S::off_t pay = pkt + aad_len;
    uint32_t nb[3];
    nonce_be(row, c.pn, nb);
    const uint32_t nblk = 1 + (P + 15) / 16;
    const uint32_t C = (nblk + kLanesPerPkt - 1) / kLanesPerPkt;
    const uint32_t Cmax = wave_max_u32(c.act ? C : 0u);
    AesRk rk;
    uint32_t ks0[4];  // block j: E(J0) on lane 0, keystream elsewhere
    const bool cached = !wave_any(c.act && nblk > 255u);
    AesCtrCache cc{};
    if (TAB) {  // round keys in SGPRs: cheap to keep across the GHASH
      load_rk(row->aes_rk, rk);
      if (cached) {
        cc = ctr_cache(rk, rb, nb);
        ctr_blockc(rk, rb, cc, (uint32_t)j, ks0);
      } else {
        ctr_block(rk, rb, nb, (uint32_t)j, ks0);
      }
    }
    if (c.pre_hp) stg.complete();
    MQ_STAMP(c.tile, 2);
    const bool hdr_written = hp && write_unmasked_header(sp, pkt, c, j, b0, pn_len, trunc, orig_b0, orig_pn);
    wave_sync();
    uint32_t y[4];
    MQ_STAMP(c.tile, 3);
    ghash<TAB>(sp, pkt, pay, aad_len, P, row, j, c.act, y);
    MQ_STAMP(c.tile, 4);
    if (!TAB) {
      load_rk(row->aes_rk, rk);
      if (cached) {
        cc = ctr_cache(rk, rb, nb);
        ctr_blockc(rk, rb, cc, (uint32_t)j, ks0);
      } else {
        ctr_block(rk, rb, nb, (uint32_t)j, ks0);
      }
    }
    uint32_t ej0[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) ej0[k] = oct_bcast0(ks0[k]);
    uint32_t tag[4], got[4];
    tag_words(y, ej0, tag);
    load_words<4>(sp, pay + P, got);
    const uint32_t diff = (tag[0] ^ got[0]) | (tag[1] ^ got[1]) | (tag[2] ^ got[2]) | (tag[3] ^ got[3]);
    if (c.act && diff != 0) {
      c.st = MQ_ERR_CRYPTO;
      c.act = false;
    }
    wave_sync();
    MQ_STAMP(c.tile, 5);
    if (c.act && j >= 1 && (uint32_t)j < nblk) xor_block(sp, pay, (uint32_t)j, P, ks0);
    uint32_t it = 1;
    for (; it + 1 < Cmax; it += 2) {  // two iterations per pass (interleaved AES rounds)
      const uint32_t b = (uint32_t)j + kLanesPerPkt * it;
      uint32_t ks[4], ks2[4];
      if (cached) ctr_block2c(rk, rb, cc, b, ks, ks2);
      else ctr_block2(rk, rb, nb, b, ks, ks2);
      if (c.act && b < nblk) xor_block(sp, pay, b, P, ks);
      if (c.act && b + kLanesPerPkt < nblk) xor_block(sp, pay, b + kLanesPerPkt, P, ks2);
    }
    if (it < Cmax) {
      const uint32_t b = (uint32_t)j + kLanesPerPkt * it;
      uint32_t ks[4];
      if (cached) ctr_blockc(rk, rb, cc, b, ks);
      else ctr_block(rk, rb, nb, b, ks);
      if (c.act && b < nblk) xor_block(sp, pay, b, P, ks);
    }
    if (direct && hdr_written && !c.act) {
      sp.st8(pkt, orig_b0);
      for (uint32_t b = 0; b < pn_len; ++b) sp.st8(pkt + d.pn_offset + b, (uint8_t)(orig_pn >> (8 * b)));
    }
  }
};

}  // namespace mq

using namespace mq;

// Tile kernels: persistent workgroups of kAesWaves waves share the LDS tables (built once per
// workgroup); wave w walks tiles blockIdx.x * kAesWaves + w + k * gridDim.x * kAesWaves. The "1"
// variants run when the key table has a single row: round keys and H powers in SGPRs, and the
// GHASH table of that row's H^8.
template <bool SINGLE>
__device__ __forceinline__ void aes_tables(const KeyRow* __restrict__ kt, uint32_t n_rows,
                                           const uint32_t* __restrict__ hot) {
  build_tw(threadIdx.x, blockDim.x);
  // multi-key kernels: a GHASH table for the hot row when the partition found one (`hot` points
  // at its index in the workspace; an out-of-range index means none)
  const uint32_t r = SINGLE ? 0u : (hot ? *hot : 0xFFFFFFFFu);
  if (SINGLE || r < n_rows) {
    if (!SINGLE && threadIdx.x == 0) g_aes_hot_row = kt + r;
    uint32_t h8[4];
#pragma unroll
    for (int w = 0; w < 4; ++w) h8[w] = brev(kt[r].H[7][w]);
    build_gh(h8, threadIdx.x, blockDim.x);  // ends with a barrier
  } else {
    if (threadIdx.x == 0) g_aes_hot_row = nullptr;
    __syncthreads();
  }
}

#define MQ_AES_KERNELS(NAME_SEAL, NAME_OPEN, SINGLE)                                                      \
  extern "C" __global__ __launch_bounds__(64 * kAesWaves) void NAME_SEAL(                                 \
      const KeyRow* __restrict__ kt, uint32_t n_rows, uint8_t* __restrict__ arena, uint64_t arena_len,    \
      const mq_pkt_desc* __restrict__ desc, uint32_t n, const uint32_t* __restrict__ index,               \
      const uint32_t* __restrict__ n_dev, uint8_t* __restrict__ status, const uint32_t* __restrict__ hot) { \
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];                                        \
    aes_tables<SINGLE>(kt, n_rows, hot);                                                                  \
    const uint32_t w = threadIdx.x >> 6;                                                                  \
    run_tiles<AesPolicyT<SINGLE>, false, SINGLE>(smem + w * kLdsBytes, blockIdx.x * kAesWaves + w,        \
                                                 gridDim.x * kAesWaves, kt, n_rows, arena, arena_len, desc,\
                                                 n, index, n_dev, status, nullptr, nullptr);              \
  }                                                                                                       \
  extern "C" __global__ __launch_bounds__(64 * kAesWaves) void NAME_OPEN(                                 \
      const KeyRow* __restrict__ kt, uint32_t n_rows, uint8_t* __restrict__ arena, uint64_t arena_len,    \
      const mq_pkt_desc* __restrict__ desc, uint32_t n, const uint32_t* __restrict__ index,               \
      const uint32_t* __restrict__ n_dev, uint8_t* __restrict__ status, uint64_t* __restrict__ pn_out,    \
      const uint2* __restrict__ hpm, const uint32_t* __restrict__ hot) {                                  \
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];                                        \
    aes_tables<SINGLE>(kt, n_rows, hot);                                                                  \
    const uint32_t w = threadIdx.x >> 6;                                                                  \
    run_tiles<AesPolicyT<SINGLE>, true, SINGLE>(smem + w * kLdsBytes, blockIdx.x * kAesWaves + w,         \
                                                gridDim.x * kAesWaves, kt, n_rows, arena, arena_len, desc, \
                                                n, index, n_dev, status, pn_out, hpm);                    \
  }
MQ_AES_KERNELS(mq_aes_seal_kernel, mq_aes_open_kernel, false)
MQ_AES_KERNELS(mq_aes_seal1_kernel, mq_aes_open1_kernel, true)

extern "C" __global__ __launch_bounds__(256) void mq_aes_hp_kernel(
    const KeyRow* __restrict__ kt, uint32_t n_rows, const uint32_t* __restrict__ key_ids,
    const uint8_t* __restrict__ samples, uint8_t* __restrict__ masks, uint32_t n) {
  build_t0(threadIdx.x, blockDim.x);
  __syncthreads();
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t kid = key_ids[i];
  if (kid >= n_rows || kt[kid].suite != MQ_SUITE_AES128GCM) return;
  GlobalSpace sp{const_cast<uint8_t*>(samples), (uint64_t)n * 16};
  uint32_t m0, m1;
  AesPolicyT<false>::hp_mask(sp, (uint64_t)i * 16, kt + kid, (threadIdx.x & (kTReplicas - 1)) * 4, m0, m1);
  for (int b = 0; b < 4; ++b) masks[5 * (size_t)i + b] = (uint8_t)(m0 >> (8 * b));
  masks[5 * (size_t)i + 4] = (uint8_t)m1;
}

// Open pre-pass: AesHeaderProtection::mask of every packet's sample, one packet per lane.
// DECODE (the batch open path): store the unmasked first byte and truncated PN (prepass_decode)
// instead of the raw mask (which mq_recv.hip's planner consumes).
template <bool DECODE>
__global__ __launch_bounds__(256) void mq_aes_open_hp_kernel(
    const KeyRow* __restrict__ kt, uint32_t n_rows, const uint8_t* __restrict__ arena, uint64_t arena_len,
    const mq_pkt_desc* __restrict__ desc, uint32_t n, const uint32_t* __restrict__ index,
    const uint32_t* __restrict__ n_dev, uint2* __restrict__ hpm) {
  build_t0(threadIdx.x, blockDim.x);
  __syncthreads();
  uint32_t i;
  const KeyRow* row;
  uint64_t at;
  mq_pkt_desc d;
  if (!prepass_pick(blockIdx.x * blockDim.x + threadIdx.x, MQ_SUITE_AES128GCM, kt, n_rows, arena_len, desc, n,
                    index, n_dev, i, row, at, d))
    return;
  GlobalSpace sp{const_cast<uint8_t*>(arena), arena_len};
  uint32_t m0, m1;
  const uint32_t rb = (threadIdx.x & (kTReplicas - 1)) * 4;
  if (DECODE) {  // PN bytes and sample (contiguous) and the first byte in one round of loads
    uint32_t w[5];
    load_words<5>(sp, at - 4, w);
    const uint8_t b0 = arena[d.offset];
    const uint32_t smp[4] = {w[1], w[2], w[3], w[4]};
    AesPolicyT<false>::hp_mask_words(smp, row, rb, m0, m1);
    hpm[i] = prepass_decode_words(b0, w[0], d, m0, m1);
  } else {
    AesPolicyT<false>::hp_mask(sp, at, row, rb, m0, m1);
    hpm[i] = make_uint2(m0, m1);
  }
}

// Persistent grid: one workgroup per CU (152 KiB of LDS each), capped by the tile count.
static uint32_t aes_grid(uint32_t tiles) {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0, v = 0;
    (void)hipGetDevice(&dev);
    cus = hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0 ? v : 256;
  }
  static int per_cu = -1;
  if (per_cu < 0) {  // diagnostic override: workgroups per CU of the grid (0 = one tile per wave)
    const char* e = getenv("MQ_AES_WGS_PER_CU");
    per_cu = e ? max(atoi(e), 0) : 1;
  }
  const uint32_t wgs = (tiles + kAesWaves - 1) / kAesWaves;
  if (per_cu == 0) return wgs;
  return wgs < (uint32_t)(cus * per_cu) ? wgs : (uint32_t)(cus * per_cu);
}

hipError_t mq_launch_aes(bool open, const KeyRow* kt, uint32_t n_rows, uint8_t* arena, uint64_t arena_len,
                         const mq_pkt_desc* desc, uint32_t n, const uint32_t* index, const uint32_t* n_dev,
                         uint8_t* status, uint64_t* pn_out, uint2* hpm, hipStream_t s, const uint32_t* hot) {
  const uint32_t tiles = (n + kPktsPerTile - 1) / kPktsPerTile;
  if (tiles == 0) return hipSuccess;
  const uint32_t blocks = aes_grid(tiles);
  const size_t dyn = (size_t)kLdsBytes * kAesWaves;
  if (open && hpm) {
    hipLaunchKernelGGL(mq_aes_open_hp_kernel<true>, dim3((n + 255) / 256), dim3(256), 0, s, kt, n_rows, arena,
                       arena_len, desc, n, index, n_dev, hpm);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  if (open)
    hipLaunchKernelGGL(n_rows == 1 ? mq_aes_open1_kernel : mq_aes_open_kernel, dim3(blocks), dim3(64 * kAesWaves),
                       dyn, s, kt, n_rows, arena, arena_len, desc, n, index, n_dev, status, pn_out, hpm, hot);
  else
    hipLaunchKernelGGL(n_rows == 1 ? mq_aes_seal1_kernel : mq_aes_seal_kernel, dim3(blocks), dim3(64 * kAesWaves),
                       dyn, s, kt, n_rows, arena, arena_len, desc, n, index, n_dev, status, hot);
  return hipGetLastError();
}

// header-protection masks of the AES-128-GCM rows of `desc` only (mq_recv.hip plans with them)
hipError_t mq_launch_aes_prepass(const KeyRow* kt, uint32_t n_rows, const uint8_t* arena, uint64_t arena_len,
                                 const mq_pkt_desc* desc, uint32_t n, uint2* hpm, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(mq_aes_open_hp_kernel<false>, dim3((n + 255) / 256), dim3(256), 0, s, kt, n_rows, arena, arena_len,
                     desc, n, (const uint32_t*)nullptr, (const uint32_t*)nullptr, hpm);
  return hipGetLastError();
}

hipError_t mq_launch_aes_hp(const KeyRow* kt, uint32_t n_rows, const uint32_t* key_ids, const uint8_t* samples,
                            uint8_t* masks, uint32_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(mq_aes_hp_kernel, dim3((n + 255) / 256), dim3(256), 0, s, kt, n_rows, key_ids, samples,
                     masks, n);
  return hipGetLastError();
}

#ifdef MQ_STAMPS
void mq_stamps_set_aes(uint64_t* p) { (void)hipMemcpyToSymbol(HIP_SYMBOL(mq_stamp_buf), &p, sizeof p); }
#endif
