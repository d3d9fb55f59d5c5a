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
//   * GHASH: every Horner step's multiply by H^8 reads an LDS table of H^8: the workgroup's
//     byte-position table in the single-key kernels (16 reads, mq_aes.h gh_mul_tab8), and in the
//     multi-key kernels a nibble half table per wave, built for the tile's key whenever all its
//     packets share one (32 reads, gh_mul_half; the mixed-batch partition lays AES packets out key
//     by key so they do); otherwise, and for the multi-key final multiply by H^e, the bit-holed
//     integer product (gf_mul).
//
// STREAMING tiles (r02): a wave = 8 packets x 8 lanes (mq_tile.h), slot b of a packet on lane
// b % 8 in iteration b / 8. Slot b >= 1 is CTR block b (counter b + 1) over payload bytes
// [16(b-1), 16b); slot 0 is E_K(J0); slots 1-A .. 0 carry the A AAD blocks and slot nblk the
// GHASH length block; slot nblk (or 8) the header-protection block of seal. GHASH block i sits in
// slot i - A + 1, so lane j's GHASH blocks are exactly its own CTR blocks: each lane loads its
// 16 B of packet straight from HBM into VGPRs (one iteration ahead), XORs the keystream, stores,
// and absorbs the ciphertext into its Horner accumulator (multiplier H^8) in the same iteration;
// a final multiply by H^e (e = blocks after the lane's last one, 1..8) and an octet XOR give the
// tag. No LDS packet image: the workgroup's LDS is its tables (72 KiB in r02; 156 KiB with the r03
// byte-position GHASH table), so 12-16 waves per CU
// (3-4 per SIMD; 12 since r04, see aes_waves) fit where the staged design (10-KiB images, r01) ran
// 8 — measured 1.41 vs 2.23 ms for a config-C seal (tools/ubench/ubench6.hip). Open decrypts in the same single pass,
// storing plaintext speculatively; a packet whose tag fails is restored by XORing the same
// keystream again, so every failed packet ends byte-identical to its input (recv.rs:416-421).
#include "mq_aes.h"
#include "mq_tile.h"
#include "mq_opts.h"

#include <cstdlib>

namespace mq {

// Packet data streams of the AES kernels. MQ_AES_NT (diagnostic build): non-temporal loads / stores,
// so the streamed packet bytes do not displace the kernel's spill slots from the L2.
#if MQ_AES_NT
typedef unsigned int aes_v4u __attribute__((ext_vector_type(4)));
typedef aes_v4u __attribute__((aligned(1))) aes_v4u_u;
__device__ __forceinline__ uint4 ald16(const uint8_t* p) {
  const aes_v4u v = __builtin_nontemporal_load((const aes_v4u_u*)p);
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void ast16(uint8_t* p, const uint32_t (&w)[4]) {
  aes_v4u v = {w[0], w[1], w[2], w[3]};
  __builtin_nontemporal_store(v, (aes_v4u_u*)p);
}
#else
__device__ __forceinline__ uint4 ald16(const uint8_t* p) { return ld16(p); }
__device__ __forceinline__ void ast16(uint8_t* p, const uint32_t (&w)[4]) { st16(p, w); }
#endif
__device__ __forceinline__ void ast_block(uint8_t* p, const uint32_t (&w)[4], uint32_t rem) {
  if (rem >= 16) ast16(p, w);
  else st_bytes(p, w, rem);
}
// bytes [lo, hi) of a 16-B block at p
__device__ __forceinline__ void st_range(uint8_t* p, const uint32_t (&w)[4], uint32_t lo, uint32_t hi) {
  if (lo == 0 && hi >= 16) {
    st16(p, w);
    return;
  }
  for (uint32_t b = lo; b < hi; ++b) p[b] = (uint8_t)(w[b >> 2] >> (8 * (b & 3)));
}

// DirectionalKeys::nonce (src/crypto/mod.rs:66-74), as big-endian AES input words
__device__ __forceinline__ void nonce_be(const KeyRow* row, uint64_t pn, uint32_t (&nb)[3]) {
  nb[0] = bswap32(row->iv[0]);
  nb[1] = bswap32(row->iv[1]) ^ (uint32_t)(pn >> 32);
  nb[2] = bswap32(row->iv[2]) ^ (uint32_t)pn;
}

// AesHeaderProtection::mask (rustcrypto.rs:175-186): AES-ECB(hp, sample)[0..5], sample as
// little-endian words. rb: TwLane in the tile kernels, the small table's replica offset in the
// one-packet-per-lane kernels.
template <class T>
__device__ __forceinline__ void aes_hp_mask_words(const uint32_t (&smp)[4], const KeyRow* row, const T& rb,
                                                  uint32_t& m0, uint32_t& m1) {
  AesRk hk;
  load_rk(row->hp_rk, hk);
  uint32_t s0 = bswap32(smp[0]), s1 = bswap32(smp[1]), s2 = bswap32(smp[2]), s3 = bswap32(smp[3]);
  aes128_block(hk, rb, s0, s1, s2, s3);
  m0 = bswap32(s0);
  m1 = s1 >> 24;
}

// GHASH length block: [len(A)]64 || [len(C)]64 in bits, reflected words
__device__ __forceinline__ void len_block(uint32_t aad_len, uint32_t ct_len, uint32_t (&x)[4]) {
  const uint64_t ab = (uint64_t)aad_len * 8, cb = (uint64_t)ct_len * 8;
  x[0] = brev((uint32_t)(ab >> 32)); x[1] = brev((uint32_t)ab);
  x[2] = brev((uint32_t)(cb >> 32)); x[3] = brev((uint32_t)cb);
}

// GHASH data block from little-endian memory words, the first `rem` bytes kept
__device__ __forceinline__ void gh_block(const uint32_t (&m)[4], uint32_t rem, uint32_t (&x)[4]) {
#pragma unroll
  for (int w = 0; w < 4; ++w) x[w] = refl(m[w] & byte_mask((int)rem, w));
}

// End of the iterations in which every active packet's lanes all hold a whole payload block that
// is not their last GHASH block (slots G it .. G it + G - 1 with G it + 2G - 2 <= full blocks), the
// range [1, lean_end) that the tile loops run without the edge cases (AAD, length block, partial
// block, HP slot, last-block multiplier). G: lanes per packet.
template <int G>
__device__ __forceinline__ int lean_end(bool act, uint32_t P) {
  const uint32_t F = P >> 4, E = 2u * G - 2u;
  return (int)Grp<G>::wave_min(!act ? 0xFFFFFFFFu : (F >= E ? (F - E) / G + 1 : 0u));
}

// Per-packet, per-lane state of a streaming tile (octet-uniform fields are equal on the 8 lanes)
struct AesPkt {
  bool act, rec, hp;
  uint32_t aad_len, P, A, nblk;
  uint64_t pkt, pay;
  uint32_t nb[3];
};

// Byte x of the unmasked header (open): byte 0 -> b0, PN bytes -> the truncated PN (big-endian)
__device__ __forceinline__ void patch_header(uint32_t (&m)[4], uint32_t at, uint8_t b0, uint32_t pn_off,
                                             uint32_t pn_len, uint32_t trunc) {
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const uint32_t x = at + (uint32_t)k;
    const uint32_t sh = 8u * (k & 3);
    uint32_t v = 0x100;  // none
    if (x == 0) v = b0;
    else if (x >= pn_off && x < pn_off + pn_len) v = (trunc >> (8u * (pn_len - 1u - (x - pn_off)))) & 0xffu;
    if (v != 0x100) m[k >> 2] = (m[k >> 2] & ~(0xffu << sh)) | (v << sh);
  }
}

// Seal: the original values of the header bytes that header protection masks — byte 0 (bits 0-7
// of hv, present: bit 8) and PN byte q (byte q of pn, present: bit 9 + q) — from the AAD block at
// packet offset `at` that this lane absorbs,
// so that the masked bytes are stored at the end without reading the header back from HBM (r05:
// that dependent read-modify-write cost the C seal 3-6 %, E's 4.6 %, profiles/r05n_phase_aes_hdr.txt)
__device__ __forceinline__ void save_header(const uint32_t (&m)[4], uint32_t at, uint32_t pn_off, uint32_t pn_len,
                                            uint32_t& hv, uint32_t& pn) {
  if (at == 0) hv |= (m[0] & 0xffu) | 0x100u;
#pragma unroll
  for (uint32_t q = 0; q < 4; ++q) {
    const uint32_t x = pn_off + q - at;  // the PN byte's offset in this block (wraps when before it)
    if (q < pn_len && x < 16u) {
      const uint32_t w = x < 4 ? m[0] : x < 8 ? m[1] : x < 12 ? m[2] : m[3];
      pn |= ((w >> (8 * (x & 3))) & 0xffu) << (8 * q);
      hv |= 0x200u << q;
    }
  }
}

// How a streaming tile multiplies by H^8: the workgroup's full table (single-key kernels), the
// wave's half table (multi-key kernels, key-uniform tile) or the bit-holed product (mixed keys)
enum GhMode { kGhWorkgroup, kGhWave, kGhProduct };

// The streaming tile of one wave: 8 packets on 8 lanes each (G = 8), or 16 on 4 (G = 4, the narrow
// single-key kernels, r06): lane j of a packet holds slots j, j + G, j + 2G, ... and the Horner
// multiplier is H^G (the workgroup's byte-position table holds H^G: aes_key_tables<G>).
template <bool SINGLE, int GH, int G = kLanesPerPkt>
struct AesStream {
  static_assert(G == 8 || ((G == 4 || G == 2) && GH == kGhWorkgroup), "narrow tiles: single-key kernels only");
  // seal: the HP sample (slots 1 and 2) is complete after iteration kSmpIt; the HP block can take
  // slot nblk when that slot lies in a later iteration
  static constexpr int kSmpIt = G >= 4 ? 0 : 1;
  static constexpr uint32_t kHpSlotMin = G >= 4 ? (uint32_t)G : 4u;
  using Gp = Grp<G>;
  // AES of slot b (b >= 0) from the CTR cache or full rounds; keystream as little-endian words
  template <bool CACHED, class K>
  static __device__ __forceinline__ void ctr(const K& key, const TwLane& L, const AesPkt& k,
                                             const AesCtrCache& cc, uint32_t b, uint32_t (&ks)[4]) {
    const uint32_t cnt = b == 0 ? 1u : b + 1;
    uint32_t s[4];
    if (CACHED) {
      aes128_ctr1(key, L, cc, cnt, s);
    } else {
      s[0] = k.nb[0]; s[1] = k.nb[1]; s[2] = k.nb[2]; s[3] = cnt;
      aes128_enc(key, L, s);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) ks[q] = bswap32(s[q]);
  }

  // Horner step acc = (acc ^ x) * H^8 for a lane holding GHASH block x; the lane's last block is
  // only added (its multiplier H^e comes in finish)
  static __device__ __forceinline__ void gh_step(uint32_t (&acc)[4], const GfOp& m8, bool has, bool last,
                                                 const uint32_t (&x)[4]) {
#pragma unroll
    for (int w = 0; w < 4; ++w) acc[w] ^= has ? x[w] : 0u;
#if MQ_PROF_SKIP & 2
    for (int w = 0; w < 4; ++w) acc[w] += m8.y[0][w & 3];
    return;
#endif
    uint32_t t[4] = {acc[0], acc[1], acc[2], acc[3]};
#if MQ_AES_NIBBLE
    if (GH == kGhWorkgroup) gh_mul_half(t, (const uint8_t*)g_aes_gh8);
#else
    if (GH == kGhWorkgroup) gh_mul_tab8(t);  // the workgroup's byte-position table of H^G
#endif
    else if (GH == kGhWave) gh_mul_half(t, (const uint8_t*)g_aes_wtab + kGhHalfBytes * wave_id());
    else gf_mul(t, m8);
#pragma unroll
    for (int w = 0; w < 4; ++w) acc[w] = (has && !last) ? t[w] : acc[w];
  }

  // tag = GHASH (final multiply by H^e, group XOR) ^ E_K(J0) (lane 0's, broadcast)
  static __device__ __forceinline__ void finish(uint32_t (&acc)[4], const KeyRow* row, int j, const AesPkt& k,
                                                const uint32_t (&ej0)[4], uint32_t (&tag)[4]) {
    uint32_t e1 = (k.nblk + (uint32_t)G - (uint32_t)j) & (uint32_t)(G - 1);  // H^(e1 + 1): blocks after the lane's last
    pin(e1);  // keeps the H^e load and its preparation (36 VGPRs) after the tile loop
#if MQ_PROF_SKIP & 64  // phase-cost diagnostic build only: no final multiply by H^e
    acc[0] ^= e1; acc[1] ^= row->H[0][1];
#else
    if (GH == kGhWorkgroup) {  // single key: the workgroup's table of H^(e1 + 1), per lane
      // e1 = G - 1 (H^G): the lane multiplied its last block in the Horner loop (fin_in_loop)
      uint32_t t[4] = {acc[0], acc[1], acc[2], acc[3]};
      gh_mul_half(t, fin_table(min(e1, (uint32_t)G - 2u)));
#pragma unroll
      for (int w = 0; w < 4; ++w) acc[w] = e1 == (uint32_t)G - 1u ? acc[w] : t[w];
    } else {
      uint32_t hp[4];
#pragma unroll
      for (int w = 0; w < 4; ++w) hp[w] = brev(row->H[e1][w]);
      const GfOp ml = gf_prepare(hp);
      gf_mul(acc, ml);
    }
#endif
#pragma unroll
    for (int w = 0; w < 4; ++w) tag[w] = bswap32(brev(Gp::xr(acc[w]))) ^ Gp::bcast0(ej0[w]);
  }

  // single-key kernels: the lane whose final multiplier would be H^G (e1 = G - 1) takes it in its
  // last Horner step instead, through the loop's table (finish skips it)
  static __device__ __forceinline__ bool fin_in_loop(const AesPkt& k, int j) {
    return GH == kGhWorkgroup && ((k.nblk + (uint32_t)G - (uint32_t)j) & (uint32_t)(G - 1)) == (uint32_t)G - 1u;
  }

  static __device__ __forceinline__ GfOp prep_m8(const KeyRow* row) {
    GfOp m8;
    if (GH == kGhProduct) {
      uint32_t h[4];
#pragma unroll
      for (int w = 0; w < 4; ++w) h[w] = brev(row->H[G - 1][w]);
      m8 = gf_prepare(h);
    }
    return m8;
  }

  // send composite (transmit.rs:625-755): seal, then header protection from the sample. For
  // packets of at least 7 CTR blocks (nblk >= 8) the HP block runs in slot nblk — a free slot of
  // the last iteration, after iteration 0 produced the sample — with the HP key through its LDS
  // pointer; shorter packets get theirs from one extra AES block of the wave after the tag (r03:
  // it replaced a post-pass over the whole batch). key: the AEAD key source (SGPRs in single-key
  // kernels, LDS otherwise); kl: this packet's LDS key schedules. CACHED: every counter of the wave's
  // packets < 256 (aes128_ctr1).
  template <bool CACHED, class K>
  static __device__ __forceinline__ void seal(uint8_t* __restrict__ arena, PktCtx& c, const KeyRow* row, int j, const K& key,
                              const uint32_t* kl) {
    const mq_pkt_desc& d = c.d;
    const TwLane L = tw_lane();
    AesPkt k;
    k.act = c.act;
    k.rec = k.act && is_record(d);
    k.aad_len = k.act ? (uint32_t)d.pn_offset + d.pn_len : 0u;
    k.P = k.act ? d.len - k.aad_len - 16 : 0u;
    k.pkt = k.act ? d.offset : 0;
    k.pay = k.pkt + k.aad_len;
    k.A = (k.aad_len + 15) >> 4;
    k.nblk = 1 + ((k.P + 15) >> 4);
    k.hp = k.act && !(d.flags & MQ_PKT_NO_HP);
    const bool hp_slot = k.hp && k.nblk >= kHpSlotMin;  // else after the tag
    const int it_lo = -(int)Gp::wave_max(k.act ? (k.A + G - 2) / G : 0u);
    const int it_hi = (int)Gp::wave_max(k.act ? k.nblk / G + 1 : 0u);
    nonce_be(row, c.pn, k.nb);
    AesCtrCache cc{};
    if (CACHED) cc = ctr_cache(key, L, k.nb);
    const GfOp m8 = prep_m8(row);
    // TLS record (seal_record, record.rs:88-113): header = ApplicationData, 0x0303, len - 5 (the
    // AAD, built in registers), the inner content type at payload byte P - 1 (patched into the
    // plaintext before encryption)
    const uint32_t rlen = d.len - 5u;
    if (k.rec && j == 0) {
      uint8_t* h = arena + k.pkt;
      h[0] = 23; h[1] = 3; h[2] = 3; h[3] = (uint8_t)(rlen >> 8); h[4] = (uint8_t)rlen;
    }
    auto data = [&](int b) -> uint4 {
      if (k.act && b >= 1 && (uint32_t)b < k.nblk) return ald16(arena + k.pay + 16ull * (uint32_t)(b - 1));
      if (k.act && !k.rec && b <= 0 && b >= 1 - (int)k.A)
        return ald16(arena + k.pkt + 16ull * (uint32_t)((int)k.A + b - 1));
      return make_uint4(0, 0, 0, 0);
    };
    uint32_t acc[4] = {0, 0, 0, 0}, ej0[4] = {0, 0, 0, 0}, smp[4] = {0, 0, 0, 0}, s1[4] = {0, 0, 0, 0};
    uint32_t m0 = 0, m1 = 0;
    bool have_mask = false;
    uint4 cur = data(j + G * it_lo);
    const int it_lean = lean_end<G>(k.act, k.P);
    const bool fin8 = fin_in_loop(k, j);
#if MQ_AES_DEFER
    // First-line deferral (r04, build option, off in the product): the payload bytes in the rest of
    // the packet's first 128-B line (after the header; at most blocks 1-7, iteration 0) are stored
    // at the end, with the tag and the header-protection bytes, so that line — shared with the
    // previous packet's tail, which is written last — goes to HBM once instead of as an early and a
    // late partial write. Measured (profiles/r04v_ab_aes_defer.txt): C seal writes 1.38 -> 1.31 GB
    // (1.10 -> 1.045 x algorithmic) but the seal 3-5 % slower (C, C/1024 keys: one more spilled
    // VGPR in the tile loop and the split block's byte stores), so the product keeps the writes.
    // Single-key kernels only: the multi-key ones have no registers to spare (15 -> 41 spills).
    const uint32_t line_rest = 128u - (uint32_t)(k.pkt & 127u);
    const uint32_t dl = (GH != kGhWorkgroup || G != 8 || !k.act || k.rec || line_rest <= k.aad_len)
                            ? 0u
                            : min(min(line_rest - k.aad_len, 112u), k.P);
#else
    const uint32_t dl = 0;
#endif
    uint32_t dct[4] = {0, 0, 0, 0}, dn = 0, doff = 0;  // this lane's deferred bytes (one block at most)
    uint32_t hs_v = 0, hs_pn = 0;                      // this lane's header bytes to mask (save_header)
    MQ_STAMP(c.tile, 1);
#pragma nounroll
    for (int it = it_lo; it < it_hi; ++it) {
      const int b = j + G * it;
      const uint32_t ub = (uint32_t)b;
      const uint4 nxt = data(b + G);  // next iteration's block, in flight during this one
      if (it > kSmpIt && it < it_lean) {  // interior iteration (wave-uniform)
        uint32_t ks[4], ct[4], x[4];
        ctr<CACHED>(key, L, k, cc, ub, ks);
        ct[0] = cur.x ^ ks[0]; ct[1] = cur.y ^ ks[1]; ct[2] = cur.z ^ ks[2]; ct[3] = cur.w ^ ks[3];
        if (k.act) ast16(arena + k.pay + 16ull * (ub - 1), ct);
#pragma unroll
        for (int q = 0; q < 4; ++q) x[q] = refl(ct[q]);
        gh_step(acc, m8, true, false, x);
        cur = nxt;
        continue;
      }
      uint32_t ks[4] = {0, 0, 0, 0};
      if (it >= 0) {  // wave-uniform: slots >= 0 run AES
        const bool is_hp = hp_slot && ub == k.nblk;
        if (wave_any(is_hp)) {  // full rounds, the HP lanes with the HP key and the sample
          uint32_t s[4] = {k.nb[0], k.nb[1], k.nb[2], ub + 1};
          if (is_hp) { s[0] = bswap32(smp[0]); s[1] = bswap32(smp[1]); s[2] = bswap32(smp[2]); s[3] = bswap32(smp[3]); }
          aes128_enc(RkLds{is_hp ? kl + 44 : kl}, L, s);
#pragma unroll
          for (int q = 0; q < 4; ++q) ks[q] = bswap32(s[q]);
          if (is_hp) { m0 = ks[0]; m1 = s[1] >> 24; have_mask = true; }
        } else {
          ctr<CACHED>(key, L, k, cc, ub, ks);
        }
      }
      uint32_t x[4] = {0, 0, 0, 0}, ct[4] = {0, 0, 0, 0};
      bool has = false;
      if (k.act && b >= 1 && ub < k.nblk) {  // payload block b - 1
        uint32_t pt[4];
        u4w(cur, pt);
        const uint32_t off = 16u * (ub - 1), rem = min(16u, k.P - off);
        if (k.rec && k.P - 1 - off < 16u) {  // inner content type
          const uint32_t at = k.P - 1 - off, sh = 8u * (at & 3);
          pt[at >> 2] = (pt[at >> 2] & ~(0xffu << sh)) | ((d.reserved & 0xffu) << sh);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) ct[q] = pt[q] ^ ks[q];
        if (off < dl) {  // its first bytes are in the packet's first line: kept for the end
#pragma unroll
          for (int q = 0; q < 4; ++q) dct[q] = ct[q];
          doff = off;
          dn = min(rem, dl - off);
          if (dn < rem) st_range(arena + k.pay + off, ct, dn, rem);
        } else {
          ast_block(arena + k.pay + off, ct, rem);
        }
        gh_block(ct, rem, x);
        has = true;
      } else if (k.act && b <= 0 && b >= 1 - (int)k.A) {  // AAD block A + b - 1
        uint32_t m[4];
        u4w(cur, m);
        if (k.rec) { m[0] = 23u | 3u << 8 | 3u << 16 | (rlen >> 8 & 0xffu) << 24; m[1] = rlen & 0xffu; }
        if (k.hp) save_header(m, 16u * (uint32_t)((int)k.A + b - 1), d.pn_offset, d.pn_len, hs_v, hs_pn);
        gh_block(m, k.aad_len - 16u * (uint32_t)((int)k.A + b - 1), x);
        has = true;
      } else if (k.act && ub == k.nblk) {  // length block
        len_block(k.aad_len, k.P, x);
        has = true;
      }
      if (b == 0) {
#pragma unroll
        for (int q = 0; q < 4; ++q) ej0[q] = ks[q];
      }
      if (G == 2 && it == 0) {  // slot 1 (lane 1); slot 2 comes in iteration 1
#pragma unroll
        for (int q = 0; q < 4; ++q) s1[q] = Gp::template lane<G - 1>(ct[q]);
      }
      if (it == kSmpIt) {  // the HP sample: payload bytes [4 - pn_len, 20 - pn_len) from slots 1 and 2
        uint32_t src[8];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          src[q] = G == 2 ? s1[q] : Gp::template lane<1 % G>(ct[q]);
          src[4 + q] = Gp::template lane<2 % G>(ct[q]);
        }
        const uint32_t o = 4u - (k.hp ? d.pn_len : 4u);
#pragma unroll
        for (int q = 0; q < 4; ++q) smp[q] = __builtin_amdgcn_alignbyte(src[q + 1], src[q], o);
      }
      gh_step(acc, m8, has, b + G > (int)k.nblk && !fin8, x);
      cur = nxt;
      if (it == 0) MQ_STAMP(c.tile, 2);
    }
    MQ_STAMP(c.tile, 3);
    uint32_t tag[4];
    finish(acc, row, j, k, ej0, tag);
    if (k.act && j == 0) st16(arena + k.pay + k.P, tag);
    MQ_STAMP(c.tile, 4);
    if (dn) st_range(arena + k.pay + doff, dct, 0, dn);  // the first line's deferred bytes
    // packets of fewer than 7 CTR blocks (no free slot for the HP block; a sample that may reach
    // into the tag): one more AES block for the wave once ciphertext and tag are stored — length-
    // sorted batches put such packets in a few tiles of their own
    const bool late = k.hp && !hp_slot;
    if (wave_any(late)) {
      wave_sync();  // this wave's ciphertext and tag stores before its sample loads
      uint32_t s[4] = {0, 0, 0, 0};
      if (late) {
        u4w(ld16(arena + k.pkt + d.pn_offset + 4), s);  // inside the packet (pn_offset + 20 <= len)
#pragma unroll
        for (int q = 0; q < 4; ++q) s[q] = bswap32(s[q]);
      }
      aes128_enc(RkLds{kl + 44}, L, s);
      if (late && j == 0) { m0 = bswap32(s[0]); m1 = s[1] >> 24; have_mask = true; }
    }
    // the masked header (RFC 9001 §5.4.1; the MAC read it unprotected): the mask from its one lane
    // to the octet, then each lane stores the header bytes it saved from its AAD blocks
    const uint32_t mk0 = Gp::xr(have_mask ? m0 : 0u), mk1 = Gp::xr(have_mask ? m1 : 0u);
#if MQ_PROF_SKIP & 128  // phase-cost diagnostic build only: no header mask writes
    hs_v = 0;
#endif
    if (hs_v) {
      uint8_t* h = arena + k.pkt;
      if (hs_v & 0x100u) h[0] = (uint8_t)(hs_v ^ (mk0 & ((d.flags & MQ_PKT_LONG_HEADER) ? 0x0fu : 0x1fu)));
      const uint32_t mk = (mk0 >> 8) | (mk1 << 24);
#pragma unroll
      for (uint32_t q = 0; q < 4; ++q)
        if (hs_v & (0x200u << q)) h[d.pn_offset + q] = (uint8_t)((hs_pn ^ mk) >> (8 * q));
    }
    MQ_STAMP(c.tile, 5);
  }

  // receive composite (recv.rs:340-421 / 953-1025): HP removal, decode_pn, open. Plaintext is
  // stored as it is produced; a packet whose tag then fails gets its ciphertext back (the same
  // keystream XORed again) and its header untouched, as the reference leaves a failed packet.
  template <bool CACHED, class K>
  static __device__ __forceinline__ void open(uint8_t* __restrict__ arena, PktCtx& c, const KeyRow* row, int j, const K& key,
                              const uint32_t* kl) {
    const mq_pkt_desc& d = c.d;
    const TwLane L = tw_lane();
    AesPkt k;
    k.hp = c.act && !(d.flags & MQ_PKT_NO_HP);
    uint32_t pn_len = d.pn_len, trunc = 0;
    uint8_t b0 = 0;
    // recv.rs:363-395 / :968-997: mask, unmask byte 0, pn_len, unmask PN, decode_pn — from the
    // pre-pass values (batch path) or computed here (one AES block per lane)
    if (c.pre_hp) {
      if (k.hp) b0 = header_from_prepass(c, pn_len, trunc);
    } else if (wave_any(k.hp)) {
      uint32_t smp[4] = {0, 0, 0, 0};
      if (k.hp) u4w(ld16(arena + d.offset + d.pn_offset + 4), smp);
      uint32_t t[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) t[q] = bswap32(smp[q]);
      aes128_enc(RkLds{kl + 44}, L, t);
      const uint32_t m0 = bswap32(t[0]), m1 = t[1] >> 24;
      if (k.hp) {
        GlobalSpace sp{arena, d.offset + d.len};
        b0 = header_from_mask(sp, d.offset, c, m0, m1, pn_len, trunc);
      }
    }
    k.act = c.act;  // PN > 2^62 - 1 fails the packet here
    k.rec = k.act && is_record(d);
    k.aad_len = k.act ? (uint32_t)d.pn_offset + pn_len : 0u;
    k.P = k.act ? d.len - k.aad_len - 16 : 0u;
    k.pkt = k.act ? d.offset : 0;
    k.pay = k.pkt + k.aad_len;
    k.A = (k.aad_len + 15) >> 4;
    k.nblk = 1 + ((k.P + 15) >> 4);
    const int it_lo = -(int)Gp::wave_max(k.act ? (k.A + G - 2) / G : 0u);
    const int it_hi = (int)Gp::wave_max(k.act ? k.nblk / G + 1 : 0u);
    uint32_t got[4] = {0, 0, 0, 0};
    if (k.act) u4w(ld16(arena + k.pay + k.P), got);
    nonce_be(row, c.pn, k.nb);
    AesCtrCache cc{};
    if (CACHED) cc = ctr_cache(key, L, k.nb);
    const GfOp m8 = prep_m8(row);
    auto data = [&](int b) -> uint4 {
      if (k.act && b >= 1 && (uint32_t)b < k.nblk) return ald16(arena + k.pay + 16ull * (uint32_t)(b - 1));
      if (k.act && b <= 0 && b >= 1 - (int)k.A) return ald16(arena + k.pkt + 16ull * (uint32_t)((int)k.A + b - 1));
      return make_uint4(0, 0, 0, 0);
    };
    uint32_t acc[4] = {0, 0, 0, 0}, ej0[4] = {0, 0, 0, 0};
    uint4 cur = data(j + G * it_lo);
    const int it_lean = lean_end<G>(k.act, k.P);
    const bool fin8 = fin_in_loop(k, j);
    MQ_STAMP(c.tile, 1);
#pragma nounroll
    for (int it = it_lo; it < it_hi; ++it) {
      const int b = j + G * it;
      const uint32_t ub = (uint32_t)b;
      const uint4 nxt = data(b + G);
      if (it >= 1 && it < it_lean) {  // interior iteration (wave-uniform)
        uint32_t ks[4], pt[4], x[4];
        ctr<CACHED>(key, L, k, cc, ub, ks);
        x[0] = refl(cur.x); x[1] = refl(cur.y); x[2] = refl(cur.z); x[3] = refl(cur.w);
        pt[0] = cur.x ^ ks[0]; pt[1] = cur.y ^ ks[1]; pt[2] = cur.z ^ ks[2]; pt[3] = cur.w ^ ks[3];
        if (k.act) ast16(arena + k.pay + 16ull * (ub - 1), pt);
        gh_step(acc, m8, true, false, x);
        cur = nxt;
        continue;
      }
      uint32_t ks[4] = {0, 0, 0, 0};
      if (it >= 0) ctr<CACHED>(key, L, k, cc, ub, ks);
      uint32_t x[4] = {0, 0, 0, 0};
      bool has = false;
      if (k.act && b >= 1 && ub < k.nblk) {  // ciphertext block b - 1
        uint32_t m[4], pt[4];
        u4w(cur, m);
        const uint32_t off = 16u * (ub - 1), rem = min(16u, k.P - off);
        gh_block(m, rem, x);
        has = true;
#pragma unroll
        for (int q = 0; q < 4; ++q) pt[q] = m[q] ^ ks[q];
        ast_block(arena + k.pay + off, pt, rem);
      } else if (k.act && b <= 0 && b >= 1 - (int)k.A) {  // AAD block: the unprotected header
        uint32_t m[4];
        u4w(cur, m);
        const uint32_t at = 16u * (uint32_t)((int)k.A + b - 1);
        if (k.hp) patch_header(m, at, b0, d.pn_offset, pn_len, trunc);
        gh_block(m, k.aad_len - at, x);
        has = true;
      } else if (k.act && ub == k.nblk) {
        len_block(k.aad_len, k.P, x);
        has = true;
      }
      if (b == 0) {
#pragma unroll
        for (int q = 0; q < 4; ++q) ej0[q] = ks[q];
      }
      gh_step(acc, m8, has, b + G > (int)k.nblk && !fin8, x);
      cur = nxt;
      if (it == 0) MQ_STAMP(c.tile, 2);
    }
    MQ_STAMP(c.tile, 3);
    uint32_t tag[4];
    finish(acc, row, j, k, ej0, tag);
    MQ_STAMP(c.tile, 4);
    const bool bad = k.act && ((tag[0] ^ got[0]) | (tag[1] ^ got[1]) | (tag[2] ^ got[2]) | (tag[3] ^ got[3])) != 0;
    if (bad) {  // Error::Crypto (rustcrypto.rs:60-94)
      c.st = MQ_ERR_CRYPTO;
      c.act = false;
    }
    if (wave_any(bad)) {  // restore the ciphertext of failed packets
#pragma nounroll
      for (int it = 0; it < it_hi; ++it) {
        const uint32_t b = (uint32_t)j + (uint32_t)G * (uint32_t)it;
        uint32_t ks[4];
        ctr<CACHED>(key, L, k, cc, b, ks);
        if (bad && b >= 1 && b < k.nblk) {
          const uint32_t off = 16u * (b - 1), rem = min(16u, k.P - off);
          uint32_t m[4];
          u4w(ld16(arena + k.pay + off), m);
#pragma unroll
          for (int q = 0; q < 4; ++q) m[q] ^= ks[q];
          st_block(arena + k.pay + off, m, rem);
        }
      }
    }
    if (c.act && k.hp && j == 0) {  // the unprotected header of an opened packet
      uint8_t* h = arena + k.pkt;
      h[0] = b0;
      for (uint32_t q = 0; q < pn_len; ++q) h[d.pn_offset + q] = (uint8_t)(trunc >> (8 * (pn_len - 1 - q)));
    }
  }
};

}  // namespace mq

using namespace mq;

// Tile kernels: persistent workgroups of aes_waves(SINGLE) waves share the LDS tables (built once
// per workgroup); wave w walks tiles blockIdx.x * W + w + k * gridDim.x * W. Every AES kernel runs
// 12 waves per CU in 168 VGPRs (r04; the multi-key ones always did: more state per packet — LDS key
// pointers, the bit-holed GHASH operand). The single-key kernels ran 16 waves in 128 VGPRs until
// r04 and spilled ~36 VGPRs per lane inside the tile loop: 116 B of scratch per lane, 3.8 MB per
// XCD, which the streamed packets kept evicting from the L2 — C's seal moved 3.92 GB per launch
// (1.56x algorithmic, writes 1.49x); at 12 waves it moves 2.83 GB (1.12x, writes 1.10x) in the same
// time (profiles/r04r_ab_aes_waves.txt). The "1" variants run when the key table has a single row:
// round keys in SGPRs and the GHASH table of that row's H^8.
#ifndef MQ_AES_SINGLE_WAVES
#define MQ_AES_SINGLE_WAVES 12
#endif
constexpr int aes_waves(bool single) { return single ? MQ_AES_SINGLE_WAVES : (int)kAesMultiWaves; }
// the key-segmented single-key kernels (mq_aes_seals / opens_kernel)
#ifndef MQ_AES_SEG_WAVES
#define MQ_AES_SEG_WAVES MQ_AES_SINGLE_WAVES
#endif
constexpr int aes_seg_waves() { return MQ_AES_SEG_WAVES; }
// Work distribution (r04): every wave runs its first tile by grid position, then claims chunks of
// the rest dynamically (mq_tile.h for_tiles, TileSched; guided chunk sizes, one head per XCD),
// when the launch has a schedule slot. That replaced (a) the static stride, under which a workgroup
// placed late — its CU held by the resident per-packet server or by the hot-key kernel forked
// beside this one — ended the launch a whole share late, and (b) the multi-key
// kernels' fixed chunks of 8 tiles (r03: a wave meets a key's consecutive tiles, E -0.8..-1.3 %),
// which left most workgroups idle on small lists: guided chunks are up to kMaxChunk
// tiles while much is left and single tiles at the end.
// key schedules in LDS: multi-key kernels, per wave and packet (copied per tile; a key-uniform
// tile uses its wave's first slot); single-key kernels, row 0's in slot 0 (copied once per
// workgroup)
__shared__ __attribute__((aligned(16))) uint32_t g_aes_keys[kAesMultiWaves * kPktsPerTile * kRkSlotBytes / 4];
__shared__ __attribute__((aligned(16))) uint32_t g_aes_keys1[kRkSlotBytes / 4];

// the key-dependent tables of a single-key workgroup (row kt[0]); ends with a barrier. G: lanes per
// packet of its tiles — the byte-position table holds the Horner multiplier H^G (H^8, or H^4 for the
// narrow kernels)
template <int G = kLanesPerPkt>
__device__ __forceinline__ void aes_key_tables(const KeyRow* __restrict__ kt) {
    if (threadIdx.x < kRkSlotBytes / 4) g_aes_keys1[threadIdx.x] = kt[0].aes_rk[threadIdx.x];  // aes_rk || hp_rk
    const uint32_t w = wave_id();
    if (w < 7) {  // waves 0..6: the half table of H^(w + 1) for the tags' final multiplies
      uint32_t hw[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) hw[q] = brev(kt[0].H[w][q]);
      build_gh_half(const_cast<uint8_t*>(fin_table(w)), hw, (int)(threadIdx.x & (kWave - 1)));
    }
    uint32_t h8[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) h8[q] = brev(kt[0].H[G - 1][q]);
#if MQ_AES_NIBBLE  // diagnostic A/B build only: the Horner multiply by H^8 through a nibble half table
    if (w == 7) build_gh_half((uint8_t*)g_aes_gh8, h8, (int)(threadIdx.x & (kWave - 1)));
    __syncthreads();
#else
    build_gh8(h8, threadIdx.x, blockDim.x);  // ends with a barrier
#endif
}

template <bool SINGLE, int G = kLanesPerPkt>
__device__ __forceinline__ void aes_tables(const KeyRow* __restrict__ kt) {
  build_tw(threadIdx.x, blockDim.x);
  if (SINGLE) aes_key_tables<G>(kt);
  else __syncthreads();
}

template <bool SINGLE, bool OPEN, int GH, bool CACHED, int G, class K>
__device__ __forceinline__ void aes_run(uint8_t* __restrict__ arena, PktCtx& c, const KeyRow* row, int j, const K& key,
                                        const uint32_t* kl) {
  if (OPEN) AesStream<SINGLE, GH, G>::template open<CACHED>(arena, c, row, j, key, kl);
  else AesStream<SINGLE, GH, G>::template seal<CACHED>(arena, c, row, j, key, kl);
}

// G: lanes per packet — 8 (tiles of 8 packets), or 4 (16 packets, single-key kernels only)
template <bool SINGLE, bool OPEN, int G = kLanesPerPkt>
__device__ __forceinline__ void aes_stream_tiles(const KeyRow* __restrict__ kt, uint32_t n_rows,
                                                 uint8_t* __restrict__ arena, uint64_t arena_len,
                                                 const mq_pkt_desc* __restrict__ desc, uint32_t n,
                                                 const uint32_t* __restrict__ index,
                                                 const uint32_t* __restrict__ n_dev, uint8_t* __restrict__ status,
                                                 uint64_t* __restrict__ pn_out, const uint2* __restrict__ hpm,
                                                 uint32_t skip, const TileSched& ts, uint32_t e0 = 0) {
  const uint32_t w = wave_id();
  static_assert(SINGLE || G == kLanesPerPkt, "narrow tiles: single-key kernels only");
  const int lane = (int)(threadIdx.x & (kWave - 1)), j = lane & (G - 1);
  uint32_t wt_kid = 0xFFFFFFFFu;  // multi-key: the row whose half table and key schedules the wave holds
  for_tiles<OPEN, G>(ts, desc, n, index, n_dev, hpm,
                     [&](uint32_t t, const TilePrefetch& pf) __attribute__((always_inline)) {
    PktCtx c;
    const KeyRow* row;
    if (!tile_ctx<MQ_SUITE_AES128GCM, OPEN, SINGLE, G>(t, kt, n_rows, arena_len, desc, n, index, n_dev, hpm, pf, c,
                                                       row, threadIdx.x, e0))
      return;
    MQ_STAMP(t, 0);
    // CTR caching needs every counter < 256: packets of at most 4080 bytes
    const bool cached = !wave_any(c.act && c.d.len > 4080u);
    if constexpr (SINGLE) {
      AesRk rk;
      load_rk(kt[0].aes_rk, rk);  // wave-uniform: SGPRs
      if (cached) aes_run<SINGLE, OPEN, kGhWorkgroup, true, G>(arena, c, row, j, RkRegs{rk}, g_aes_keys1);
      else aes_run<SINGLE, OPEN, kGhWorkgroup, false, G>(arena, c, row, j, RkRegs{rk}, g_aes_keys1);
    } else {
      // a tile whose active packets share one row: round keys in SGPRs, that row's H^8 half table
      // (and key schedules for the HP block) in the wave's LDS, rebuilt only when the row changes
      const uint32_t kid = __builtin_amdgcn_readfirstlane(wave_min_u32(c.act ? c.d.key_id : 0xFFFFFFFFu));
      if (kid != 0xFFFFFFFFu && !wave_any(c.act && c.d.key_id != kid)) {
        const KeyRow* urow = kt + kid;
        uint32_t* kl = g_aes_keys + w * kPktsPerTile * (kRkSlotBytes / 4);
        if (kid != wt_kid) {
          uint32_t h8[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) h8[q] = brev(urow->H[7][q]);
          build_gh_half((uint8_t*)g_aes_wtab + kGhHalfBytes * w, h8, lane);  // ends with wave_sync
          for (int q = lane; q < (int)(kRkSlotBytes / 4); q += kWave) kl[q] = urow->aes_rk[q];  // aes_rk || hp_rk
          wave_sync();
          wt_kid = kid;
        }
        AesRk rk;
        load_rk(urow->aes_rk, rk);
        if (cached) aes_run<SINGLE, OPEN, kGhWave, true, G>(arena, c, urow, j, RkRegs{rk}, kl);
        else aes_run<SINGLE, OPEN, kGhWave, false, G>(arena, c, urow, j, RkRegs{rk}, kl);
      } else {
        // mixed keys: each packet's key schedules into its own LDS slot (lane j copies words
        // 11j .. 11j + 10 of aes_rk || hp_rk, contiguous in the row)
        const uint32_t p = (uint32_t)lane / kLanesPerPkt;
        uint32_t* kl = g_aes_keys + (w * kPktsPerTile + p) * (kRkSlotBytes / 4);
        const uint32_t* src = row->aes_rk + 11 * j;
        uint32_t v[11];
#pragma unroll
        for (int q = 0; q < 11; ++q) v[q] = src[q];
#pragma unroll
        for (int q = 0; q < 11; ++q) kl[11 * j + q] = v[q];
        wave_sync();
        wt_kid = 0xFFFFFFFFu;  // slot 0 no longer holds a key-uniform tile's schedules
        if (cached) aes_run<SINGLE, OPEN, kGhProduct, true, G>(arena, c, row, j, RkLds{kl}, kl);
        else aes_run<SINGLE, OPEN, kGhProduct, false, G>(arena, c, row, j, RkLds{kl}, kl);
      }
    }
    MQ_STAMP(t, 7);
    tile_status<OPEN>(c, j, status, pn_out);
  }, skip, e0);
}

// hot (partition lists only, else null): hot[0] = the hot key's row, hot[1] = the entries of its
// segment at the front of the list (whole tiles). A single-key kernel then runs that segment with
// the hot row as its one-row table; the multi-key kernel starts after it.
template <bool SINGLE, int G = kLanesPerPkt>
__device__ __forceinline__ bool aes_hot_split(const uint32_t* __restrict__ hot, const KeyRow* __restrict__& kt,
                                              const uint32_t* __restrict__& n_dev, uint32_t& skip) {
  skip = 0;
  if (!hot) return true;
  const uint32_t entries = hot[1];
  if (SINGLE) {
    // workgroup-uniform, before any barrier: no segment (hot[0] may be no row), or no tile for
    // this workgroup (a small segment: skip the table builds)
    if (blockIdx.x * (aes_waves(true) * (kWave / G)) >= entries) return false;
    kt += hot[0];
    n_dev = hot + 1;
  } else {
    skip = entries / kPktsPerTile;
  }
  return true;
}

// workgroup-uniform, before any table is built: whether this workgroup of a persistent grid has
// a tile (a partition list's device count may be small or zero — an AES batch's leftover list is
// usually empty, and 256 workgroups building their tables for nothing cost ~35 us). Its waves' first
// tiles are skip + blockIdx.x * W + w; every later tile lies beyond all first tiles, so a
// workgroup without a first tile has none at all.
template <bool SINGLE, int G = kLanesPerPkt>
__device__ __forceinline__ bool aes_wg_has_work(uint32_t n, const uint32_t* __restrict__ n_dev, uint32_t skip) {
  const uint32_t count = n_dev ? *n_dev : n;
  const uint32_t tiles = (count + kWave / G - 1) / (kWave / G);
  return skip + blockIdx.x * aes_waves(SINGLE) < tiles;
}

__device__ __forceinline__ TileSched aes_sched(uint32_t* sched, bool single) {
  const uint32_t W = (uint32_t)aes_waves(single);
  return TileSched{sched, blockIdx.x * W + wave_id(), gridDim.x * W, blockIdx.x % kSchedHeads};
}

// sched: the launch's schedule slot (dynamic tiles), null for the static stride. Every workgroup
// reaches sched_done once: without work at its only exit, else after a barrier behind its tiles.
#define MQ_AES_KERNELS(NAME_SEAL, NAME_OPEN, SINGLE, G)                                                   \
  extern "C" __global__ __launch_bounds__(64 * aes_waves(SINGLE)) void NAME_SEAL(                           \
      const KeyRow* __restrict__ kt, uint32_t n_rows, uint8_t* __restrict__ arena, uint64_t arena_len,    \
      const mq_pkt_desc* __restrict__ desc, uint32_t n, const uint32_t* __restrict__ index,               \
      const uint32_t* __restrict__ n_dev, const uint32_t* __restrict__ hot, uint8_t* __restrict__ status, \
      uint32_t* __restrict__ sched) {                                                                     \
    uint32_t skip;                                                                                        \
    if (!aes_hot_split<SINGLE, G>(hot, kt, n_dev, skip) || !aes_wg_has_work<SINGLE, G>(n, n_dev, skip)) { \
      sched_done(sched);                                                                                  \
      return;                                                                                             \
    }                                                                                                     \
    aes_tables<SINGLE, G>(kt);                                                                            \
    aes_stream_tiles<SINGLE, false, G>(kt, n_rows, arena, arena_len, desc, n, index, n_dev, status, nullptr, \
                                    nullptr, skip, aes_sched(sched, SINGLE));                             \
    __syncthreads();                                                                                      \
    sched_done(sched);                                                                                    \
  }                                                                                                       \
  extern "C" __global__ __launch_bounds__(64 * aes_waves(SINGLE)) void NAME_OPEN(                           \
      const KeyRow* __restrict__ kt, uint32_t n_rows, uint8_t* __restrict__ arena, uint64_t arena_len,    \
      const mq_pkt_desc* __restrict__ desc, uint32_t n, const uint32_t* __restrict__ index,               \
      const uint32_t* __restrict__ n_dev, const uint32_t* __restrict__ hot, uint8_t* __restrict__ status, \
      uint64_t* __restrict__ pn_out, const uint2* __restrict__ hpm, uint32_t* __restrict__ sched) {       \
    uint32_t skip;                                                                                        \
    if (!aes_hot_split<SINGLE, G>(hot, kt, n_dev, skip) || !aes_wg_has_work<SINGLE, G>(n, n_dev, skip)) { \
      sched_done(sched);                                                                                  \
      return;                                                                                             \
    }                                                                                                     \
    aes_tables<SINGLE, G>(kt);                                                                            \
    aes_stream_tiles<SINGLE, true, G>(kt, n_rows, arena, arena_len, desc, n, index, n_dev, status, pn_out, hpm, \
                                   skip, aes_sched(sched, SINGLE));                                       \
    __syncthreads();                                                                                      \
    sched_done(sched);                                                                                    \
  }
MQ_AES_KERNELS(mq_aes_seal_kernel, mq_aes_open_kernel, false, 8)
MQ_AES_KERNELS(mq_aes_seal1_kernel, mq_aes_open1_kernel, true, 8)
// narrow single-key kernels (r06): tiles of 16 short packets on 4 lanes each (AesStream G = 4)
MQ_AES_KERNELS(mq_aes_seal1n_kernel, mq_aes_open1n_kernel, true, 4)
MQ_AES_KERNELS(mq_aes_seal1n2_kernel, mq_aes_open1n2_kernel, true, 2)

// Key-segmented single-key kernels (r03): for a partition list in the keyed layout whose keys carry
// many packets each (config C with 1024 keys: 128 tiles per key), every key's segment runs at
// single-key speed — one persistent workgroup per CU walks segments (the hot key's classes at the
// list's front, then row r's segment, hot[] and rowseg[] from the partition), rebuilding only the
// key-dependent tables (round keys, the byte-position GHASH table of H^8, the half tables of
// H^1..H^7: a few us)
// between them, its waves striding the segment's tiles. The multi-key kernel pays for
// key changes per tile instead (per-lane key set-up, the bit-holed final multiply: 1024-key C 21 %
// slower than one key on the same packets, profiles/r03p_scatter_probe.json).
// Work goes to workgroups in SLICES of the list (r04): list 0 is the hot key's segment followed by
// the rows' segments, back to back in whole tiles, and slice u is its tiles [uP, uP + P), P =
// list tiles / (4 x workgroups) clamped to [16, 128] (config C with 1024 keys: 128, one row's
// segment per slice). A workgroup claims slices from head 0 of the launch's schedule slot (or by
// stride without one) and runs the part of each segment inside its slice, rebuilding the tables
// only when the row changes. Until r04 the unit was a whole segment: with two keys of 2^19 packets
// each, each segment ran on ONE workgroup, 6.3 GiB/s (gpurun_out/r04za).
constexpr uint32_t kSegMinSlice = 16, kSegMaxSlice = 128;  // tiles

// the row whose segment holds list entry e >= rowseg[0] (the first row's start): the last row r
// with rowseg[2r] <= e (a row without packets starts where the next one does, so the last of
// equal starts is the one with packets). 64-ary search, every wave computing the same answer.
__device__ __forceinline__ uint32_t seg_row_of(const uint32_t* __restrict__ rowseg, uint32_t n_rows, uint32_t e) {
  const int lane = (int)(threadIdx.x & (kWave - 1));
  uint32_t lo = 0, span = n_rows;  // the answer lies in [lo, lo + span)
  while (span > 1) {               // uniform
    const uint32_t step = (span + kWave - 1) / kWave, idx = lo + (uint32_t)lane * step;
    const bool ok = idx < lo + span && rowseg[2 * (size_t)idx] <= e;  // a prefix of the lanes (lane 0 holds)
    const uint64_t m = __ballot(ok);
    const uint32_t k = 63u - (uint32_t)__builtin_clzll(m | 1ull);
    const uint32_t nlo = lo + k * step;
    span = min(step, lo + span - nlo);
    lo = nlo;
  }
  return lo;
}

template <bool OPEN, int G>
__device__ __forceinline__ void aes_seg_tiles(const KeyRow* __restrict__ kt, uint32_t n_rows, uint8_t* __restrict__ arena,
                                              uint64_t arena_len, const mq_pkt_desc* __restrict__ desc,
                                              const uint32_t* __restrict__ list, const uint32_t* __restrict__ n_dev,
                                              const uint32_t* __restrict__ hot, const uint32_t* __restrict__ rowseg,
                                              uint8_t* __restrict__ status, uint64_t* __restrict__ pn_out,
                                              const uint2* __restrict__ hpm, uint32_t* __restrict__ sched) {
  constexpr uint32_t W = aes_seg_waves();
  __shared__ uint32_t s_seg;
  build_tw(threadIdx.x, blockDim.x);  // key-independent: once
  const uint32_t w = wave_id();
  const uint32_t entries = __builtin_amdgcn_readfirstlane(*n_dev), tiles = entries / kPktsPerTile;
  const uint32_t hot_row = __builtin_amdgcn_readfirstlane(hot[0]), hot_e = __builtin_amdgcn_readfirstlane(hot[1]);
  const uint32_t P = min(max((tiles + 4 * gridDim.x - 1) / (4 * gridDim.x), kSegMinSlice), kSegMaxSlice);
  uint32_t sg = blockIdx.x, built = 0xFFFFFFFFu;  // built: the row whose tables are in LDS
  for (;;) {
    __syncthreads();  // every wave is done with the previous slice (its tiles, s_seg)
    if (sched) {
      if (threadIdx.x == 0)
        s_seg = __hip_atomic_fetch_add(sched, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __syncthreads();
      sg = s_seg;
    }
    if ((uint64_t)sg * P >= tiles) break;  // workgroup-uniform
    const uint32_t e1 = kPktsPerTile * min(sg * P + P, tiles);
    uint32_t e = kPktsPerTile * sg * P;
    if (!sched) sg += gridDim.x;
    while (e < e1) {  // the segments overlapping the slice, workgroup-uniform
      uint32_t row, end;
      if (e < hot_e) {
        row = hot_row;
        end = hot_e;
      } else {
        const uint32_t r = __builtin_amdgcn_readfirstlane(seg_row_of(rowseg, n_rows, e));
        row = r;
        end = __builtin_amdgcn_readfirstlane(rowseg[2 * (size_t)r] + rowseg[2 * (size_t)r + 1]);
      }
      end = min(end, e1);
      if (end <= e) break;  // no segment holds e (a broken layout: leave the slice)
      if (row < n_rows) {
        const KeyRow* ks = kt + row;  // the segment's row as a one-row table (validation uses n_rows)
        if (row != built) {
          __syncthreads();  // the previous segment's tiles are done with the tables
          aes_key_tables<G>(ks);  // ends with a barrier
          built = row;
        }
        aes_stream_tiles<true, OPEN, G>(ks, n_rows, arena, arena_len, desc, end, list, nullptr, status, pn_out, hpm,
                                        0, TileSched{nullptr, w, W, 0}, e);
      }
      e = end;
    }
  }
  sched_done(sched);  // after the loop's last barrier
}
#define MQ_AES_SEG_KERNELS(NAME_SEAL, NAME_OPEN, G)                                                                 \
  extern "C" __global__ __launch_bounds__(64 * aes_seg_waves()) void NAME_SEAL(                                     \
      const KeyRow* __restrict__ kt, uint32_t n_rows, uint8_t* __restrict__ arena, uint64_t arena_len,             \
      const mq_pkt_desc* __restrict__ desc, const uint32_t* __restrict__ list, const uint32_t* __restrict__ n_dev, \
      const uint32_t* __restrict__ hot, const uint32_t* __restrict__ rowseg, uint8_t* __restrict__ status,         \
      uint32_t* __restrict__ sched) {                                                                              \
    aes_seg_tiles<false, G>(kt, n_rows, arena, arena_len, desc, list, n_dev, hot, rowseg, status, nullptr, nullptr, \
                            sched);                                                                                \
  }                                                                                                                \
  extern "C" __global__ __launch_bounds__(64 * aes_seg_waves()) void NAME_OPEN(                                     \
      const KeyRow* __restrict__ kt, uint32_t n_rows, uint8_t* __restrict__ arena, uint64_t arena_len,             \
      const mq_pkt_desc* __restrict__ desc, const uint32_t* __restrict__ list, const uint32_t* __restrict__ n_dev, \
      const uint32_t* __restrict__ hot, const uint32_t* __restrict__ rowseg, uint8_t* __restrict__ status,         \
      uint64_t* __restrict__ pn_out, const uint2* __restrict__ hpm, uint32_t* __restrict__ sched) {                \
    aes_seg_tiles<true, G>(kt, n_rows, arena, arena_len, desc, list, n_dev, hot, rowseg, status, pn_out, hpm, sched); \
  }
MQ_AES_SEG_KERNELS(mq_aes_seals_kernel, mq_aes_opens_kernel, 8)
// narrow tiles (16 packets on 4 lanes each) within every key's segment (r06)
MQ_AES_SEG_KERNELS(mq_aes_sealsn_kernel, mq_aes_opensn_kernel, 4)
MQ_AES_SEG_KERNELS(mq_aes_sealsn2_kernel, mq_aes_opensn2_kernel, 2)

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
  uint32_t smp[4], m0, m1;
  load_words<4>(sp, (uint64_t)i * 16, smp);
  aes_hp_mask_words(smp, kt + kid, (uint32_t)(threadIdx.x & (kTReplicas - 1)) * 4, m0, m1);
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
  if (blockIdx.x * blockDim.x >= (n_dev ? *n_dev : n)) return;  // list mode: grids cover the list capacity
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
    uint8_t b0;
    prepass_header(arena, d, b0, w);
    const uint32_t smp[4] = {w[1], w[2], w[3], w[4]};
    aes_hp_mask_words(smp, row, rb, m0, m1);
    hpm[i] = prepass_decode_words(b0, w[0], d, m0, m1);
  } else {
    uint32_t smp[4];
    load_words<4>(sp, at, smp);
    aes_hp_mask_words(smp, row, rb, m0, m1);
    hpm[i] = make_uint2(m0, m1);
  }
}

// Persistent grid: one workgroup per CU (152 KiB of LDS each), capped by the tile count.
static uint32_t aes_grid(uint32_t tiles, uint32_t waves, int cus) {
  static const int per_cu = [] {  // diagnostic override: workgroups per CU of the grid (0 = one tile per wave)
    const char* e = getenv("MQ_AES_WGS_PER_CU");
    return e ? max(atoi(e), 0) : 1;
  }();
  if (cus <= 0) cus = 256;
  const uint32_t wgs = (tiles + waves - 1) / waves;
  if (per_cu == 0) return wgs;
  return wgs < (uint32_t)(cus * per_cu) ? wgs : (uint32_t)(cus * per_cu);
}

// hs: the stream of the hot segment's kernel — a side stream forked from s by the caller
// (mq_host.cpp, one per device and caller stream), so each CU moves from one tile kernel to the
// other as its own workgroup ends, not after the other kernel's last one; s when not forked.
// cus: the device's compute units (the persistent grid).
// rowseg (a keyed partition list, mq_partition_rowseg): the key-segmented kernels run the whole
// list (hot key included) instead of the hot split + multi-key kernel.
// sched_s / sched_hs: the schedule slots of streams s / hs (mq_runtime.h SchedSlots), null for the
// static stride.
// Flat single-key batches (bytes per packet bpp, 0 = unknown) up to MQ_AES_NARROW_MAX run the
// narrow kernels: 16 packets per tile on 4 lanes each, so the per-tile fixed work (set-up, J0, the
// final multiply, the header-protection block) is shared by twice the packets, the HP block of a
// packet with at least 4 CTR blocks takes a free slot instead of a late extra round, and a packet's
// slots fill whole iterations of 4 instead of 8 (1200 B: 76 slots in 19 iterations, not 80 in 10).
// Measured (profiles/r06i_*): seal + open 64 B 150 -> 244 GiB/s, 256 B 421 -> 555, 700 B 651 -> 739,
// 1200 B 732 -> 768 (config C: 3.18 -> 3.02 ms), 1500 B 758 -> 768; 1600 B 771 -> 759, 2048 B 796 -> 768
// (r06j), so the octet kernels keep packets over 1536 B.
// Flat batches up to MQ_AES_NARROW2_MAX bytes per packet take tiles of 32 packets on 2 lanes each
// (r06l: 64 B 248 -> 339 GiB/s, 128 B 393 -> 505, 256 B 569 -> 619, 448 B equal, 700 B 757 -> 653:
// a packet's 2 lanes walk 22+ iterations each).
#ifndef MQ_AES_NARROW_MAX
#define MQ_AES_NARROW_MAX 1536
#endif
#ifndef MQ_AES_NARROW2_MAX
#define MQ_AES_NARROW2_MAX 400
#endif
constexpr uint64_t kAesNarrowMaxBpp = MQ_AES_NARROW_MAX, kAesNarrow2MaxBpp = MQ_AES_NARROW2_MAX;
// lanes per packet of the single-key tiles: MQ_AES_NARROW 0 -> 8, 1 -> 4, 2 -> 2; unset: flat
// batches by their bytes per packet, partition segments (mixed lengths: config E 2.42 ms with 4,
// 2.47 with 2, r06l) 4
static int aes_lanes(bool flat, uint64_t bpp) {
  const long f = opt(Opt::AesNarrow);
  if (f >= 0) return f == 0 ? 8 : f == 2 ? 2 : 4;
  if (!flat) return 4;
  if (bpp == 0 || bpp > kAesNarrowMaxBpp) return 8;
  return bpp <= kAesNarrow2MaxBpp ? 2 : 4;
}
int mq_aes_flat_lanes(uint64_t bpp) { return aes_lanes(true, bpp); }
using AesSealK = void (*)(const KeyRow*, uint32_t, uint8_t*, uint64_t, const mq_pkt_desc*, uint32_t, const uint32_t*,
                          const uint32_t*, const uint32_t*, uint8_t*, uint32_t*);
using AesOpenK = void (*)(const KeyRow*, uint32_t, uint8_t*, uint64_t, const mq_pkt_desc*, uint32_t, const uint32_t*,
                          const uint32_t*, const uint32_t*, uint8_t*, uint64_t*, const uint2*, uint32_t*);
using AesSegSealK = void (*)(const KeyRow*, uint32_t, uint8_t*, uint64_t, const mq_pkt_desc*, const uint32_t*,
                             const uint32_t*, const uint32_t*, const uint32_t*, uint8_t*, uint32_t*);
using AesSegOpenK = void (*)(const KeyRow*, uint32_t, uint8_t*, uint64_t, const mq_pkt_desc*, const uint32_t*,
                             const uint32_t*, const uint32_t*, const uint32_t*, uint8_t*, uint64_t*, const uint2*,
                             uint32_t*);
static AesSealK seal1_of(int g) { return g == 2 ? mq_aes_seal1n2_kernel : g == 4 ? mq_aes_seal1n_kernel : mq_aes_seal1_kernel; }
static AesOpenK open1_of(int g) { return g == 2 ? mq_aes_open1n2_kernel : g == 4 ? mq_aes_open1n_kernel : mq_aes_open1_kernel; }
static AesSegSealK seals_of(int g) { return g == 2 ? mq_aes_sealsn2_kernel : g == 4 ? mq_aes_sealsn_kernel : mq_aes_seals_kernel; }
static AesSegOpenK opens_of(int g) { return g == 2 ? mq_aes_opensn2_kernel : g == 4 ? mq_aes_opensn_kernel : mq_aes_opens_kernel; }

hipError_t mq_launch_aes(bool open, const KeyRow* kt, uint32_t n_rows, uint8_t* arena, uint64_t arena_len,
                         const mq_pkt_desc* desc, uint32_t n, const uint32_t* index, const uint32_t* n_dev,
                         const uint32_t* hot, uint8_t* status, uint64_t* pn_out, uint2* hpm, bool own_hp,
                         hipStream_t s, hipStream_t hs, int cus, const uint32_t* rowseg, uint32_t* sched_s,
                         uint32_t* sched_hs, uint64_t bpp) {
  const uint32_t tiles = (n + kPktsPerTile - 1) / kPktsPerTile;
  if (tiles == 0) return hipSuccess;
  const int gflat = aes_lanes(true, bpp);
  if (n_rows == 1 && !index && !n_dev && !hot && gflat != 8) {
    const uint32_t waves = aes_waves(true), ppt = 64u / (uint32_t)gflat, blocks = aes_grid((n + ppt - 1) / ppt, waves, cus);
    if (open && hpm && own_hp) {
      hipLaunchKernelGGL(mq_aes_open_hp_kernel<true>, dim3((n + 255) / 256), dim3(256), 0, s, kt, n_rows, arena,
                         arena_len, desc, n, index, n_dev, hpm);
      const hipError_t e = hipGetLastError();
      if (e != hipSuccess) return e;
    }
    if (open)
      hipLaunchKernelGGL(open1_of(gflat), dim3(blocks), dim3(64 * waves), 0, s, kt, n_rows, arena, arena_len, desc,
                         n, index, n_dev, hot, status, pn_out, hpm, sched_s);
    else
      hipLaunchKernelGGL(seal1_of(gflat), dim3(blocks), dim3(64 * waves), 0, s, kt, n_rows, arena, arena_len, desc,
                         n, index, n_dev, hot, status, sched_s);
    return hipGetLastError();
  }
  // the hot key's segment of a partition list, and the key-segmented kernels' segments, run narrow
  // tiles too, unless MQ_AES_NARROW=0
  const int ghot = aes_lanes(false, bpp);
  if (rowseg && index && hot && n_rows > 1 && !own_hp) {
    const uint32_t blocks = (uint32_t)(cus > 0 ? cus : 256);
    if (open)
      hipLaunchKernelGGL(opens_of(ghot), dim3(blocks),
                         dim3(64 * aes_seg_waves()), 0, s, kt, n_rows, arena, arena_len, desc, index, n_dev, hot,
                         rowseg, status, pn_out, hpm, sched_s);
    else
      hipLaunchKernelGGL(seals_of(ghot), dim3(blocks),
                         dim3(64 * aes_seg_waves()), 0, s, kt, n_rows, arena, arena_len, desc, index, n_dev, hot,
                         rowseg, status, sched_s);
    return hipGetLastError();
  }
  const uint32_t waves = aes_waves(n_rows == 1), blocks = aes_grid(tiles, waves, cus);
  // a partition list over several rows: the hot key's segment on a single-key kernel first
  hot = (hot && index && n_rows > 1) ? hot : nullptr;
  const uint32_t hot_blocks = hot ? aes_grid(tiles, aes_waves(true), cus) : 0u;
  if (open && hpm && own_hp) {  // !own_hp: mq_launch_mixed_hp covers both suites' lists
    hipLaunchKernelGGL(mq_aes_open_hp_kernel<true>, dim3((n + 255) / 256), dim3(256), 0, s, kt, n_rows, arena,
                       arena_len, desc, n, index, n_dev, hpm);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  if (!hot) hs = s;
  // the launch's own HP passes run on s: a forked hot kernel would race them
  if (own_hp && hs != s) return hipErrorInvalidValue;
  // two kernels at once on one stream's slot would share its heads
  if (hot && hs == s) sched_hs = nullptr;
  // the hot segment on the key-segmented (slice) kernel: one workgroup per CU walks contiguous slices
  // of the length-sorted segment (count = the segment's entries, so no row segment is ever reached).
  // E's hot AES key alone 2.94 -> 2.54 ns per packet, hot + Initial keys 3.03 -> 2.76; the whole
  // config-E batch unchanged (its ChaCha20 list after the multi-key kernel on s is the longer chain;
  // profiles/r06q_*). MQ_AES_HOT_SEG=0: the tile kernel.
  const bool hot_seg = hot && opt(Opt::AesHotSeg) != 0;
  const uint32_t seg_blocks = (uint32_t)(cus > 0 ? cus : 256);
  if (hot_seg) {
    if (open)
      hipLaunchKernelGGL(opens_of(ghot), dim3(seg_blocks), dim3(64 * aes_seg_waves()), 0, hs, kt, n_rows, arena,
                         arena_len, desc, index, hot + 1, hot, (const uint32_t*)nullptr, status, pn_out, hpm, sched_hs);
    else
      hipLaunchKernelGGL(seals_of(ghot), dim3(seg_blocks), dim3(64 * aes_seg_waves()), 0, hs, kt, n_rows, arena,
                         arena_len, desc, index, hot + 1, hot, (const uint32_t*)nullptr, status, sched_hs);
  }
  if (open) {
    if (hot && !hot_seg)
      hipLaunchKernelGGL(open1_of(ghot), dim3(hot_blocks),
                         dim3(64 * aes_waves(true)), 0, hs, kt, n_rows, arena, arena_len, desc, n, index, n_dev, hot,
                         status, pn_out, hpm, sched_hs);
    hipLaunchKernelGGL(n_rows == 1 ? mq_aes_open1_kernel : mq_aes_open_kernel, dim3(blocks), dim3(64 * waves),
                       0, s, kt, n_rows, arena, arena_len, desc, n, index, n_dev, hot, status, pn_out, hpm, sched_s);
  } else {
    if (hot && !hot_seg)
      hipLaunchKernelGGL(seal1_of(ghot), dim3(hot_blocks),
                         dim3(64 * aes_waves(true)), 0, hs, kt, n_rows, arena, arena_len, desc, n, index, n_dev, hot,
                         status, sched_hs);
    hipLaunchKernelGGL(n_rows == 1 ? mq_aes_seal1_kernel : mq_aes_seal_kernel, dim3(blocks), dim3(64 * waves),
                       0, s, kt, n_rows, arena, arena_len, desc, n, index, n_dev, hot, status, sched_s);
  }
  return hipGetLastError();
}

// Mixed batches: the open pre-pass over every descriptor of the batch in DESCRIPTOR order, one
// packet per lane, either suite per lane. (r02 walked the two partition lists: their order
// scatters the descriptor and header reads over the arena, 0.34 GB per 2^20-packet config-E
// launch where the descriptors alone are 34 MB, r03b PMC.) Seal needs no pass: both suites' tiles
// mask their own packets (r03). The block's AES packets go to its first threads and its ChaCha20
// packets to the next ones, so only the wave on the boundary runs both suites' code (in
// descriptor order a mixed batch puts both suites in nearly every wave, and a wave paid for the
// AES block and the ChaCha20 block).
__device__ __forceinline__ bool mixed_hp_pick(const KeyRow* __restrict__ kt, uint32_t n_rows, uint64_t arena_len,
                                              const mq_pkt_desc* __restrict__ desc, uint32_t n, uint32_t i,
                                              mq_pkt_desc& d, bool& aes) {
  aes = false;
  if (i >= n) return false;
  d = desc[i];  // prepass_pick's checks; the tile kernels report the rest
  if (!(d.key_id < n_rows && d.offset + (uint64_t)d.len <= arena_len && !(d.flags & MQ_PKT_NO_HP) &&
        (uint64_t)d.pn_offset + 20 <= d.len))
    return false;
  const uint32_t su = kt[d.key_id].suite;
  aes = su == MQ_SUITE_AES128GCM;
  return aes || su == MQ_SUITE_CHACHA20;
}

__global__ __launch_bounds__(256) void mq_mixed_hp_kernel(
    const KeyRow* __restrict__ kt, uint32_t n_rows, const uint8_t* __restrict__ arena, uint64_t arena_len,
    const mq_pkt_desc* __restrict__ desc, uint32_t n, uint2* __restrict__ hpm) {
  __shared__ uint32_t s_item[256];
  __shared__ uint32_t s_wcnt[2][4];
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x >> 6;
  mq_pkt_desc d{};
  bool aes;
  const bool act = mixed_hp_pick(kt, n_rows, arena_len, desc, n, i, d, aes);
  // compaction: AES packets to threads [0, nA), ChaCha20 packets to [nA, nA + nC)
  const uint64_t ba = __ballot(act && aes), bc = __ballot(act && !aes);
  const uint64_t below = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  if (lane == 0) { s_wcnt[0][w] = (uint32_t)__popcll(ba); s_wcnt[1][w] = (uint32_t)__popcll(bc); }
  __syncthreads();
  uint32_t nA = 0, nC = 0, preA = 0, preC = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (q < w) { preA += s_wcnt[0][q]; preC += s_wcnt[1][q]; }
    nA += s_wcnt[0][q];
    nC += s_wcnt[1][q];
  }
  if (nA + nC == 0) return;  // block-uniform
  if (act) s_item[aes ? preA + (uint32_t)__popcll(ba & below) : nA + preC + (uint32_t)__popcll(bc & below)] = i;
  if (nA) build_t0(threadIdx.x, blockDim.x);  // the S-box table only where AES lanes have work
  __syncthreads();
  const uint32_t t = threadIdx.x;
  if (t >= nA + nC) return;
  const uint32_t item = s_item[t];
  const bool a = t < nA;
  if (item != i) d = desc[item];  // the moved packets' descriptors (cached: this block just read them)
  const KeyRow* row = kt + d.key_id;
  uint32_t wd[5], m0, m1;
  uint8_t b0;
  prepass_header(arena, d, b0, wd);
  const uint32_t smp[4] = {wd[1], wd[2], wd[3], wd[4]};
  if (a) {
    aes_hp_mask_words(smp, row, (uint32_t)(threadIdx.x & (kTReplicas - 1)) * 4, m0, m1);
  } else {  // ChaChaHeaderProtection::mask (rustcrypto.rs:197-220)
    uint32_t hk[8], blk[16];
#pragma unroll
    for (int q = 0; q < 8; ++q) hk[q] = row->hp[q];
    chacha20_block(hk, smp[0], smp[1], smp[2], smp[3], blk);
    m0 = blk[0];
    m1 = blk[1];
  }
  hpm[item] = prepass_decode_words(b0, wd[0], d, m0, m1);
}

hipError_t mq_launch_mixed_open_hp(const KeyRow* kt, uint32_t n_rows, const uint8_t* arena, uint64_t arena_len,
                                   const mq_pkt_desc* desc, uint32_t n, uint2* hpm, hipStream_t s) {
  const uint32_t blocks = (n + 255) / 256;
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL(mq_mixed_hp_kernel, dim3(blocks), dim3(256), 0, s, kt, n_rows, arena, arena_len, desc, n, hpm);
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
