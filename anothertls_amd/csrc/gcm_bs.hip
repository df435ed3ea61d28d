// AES-GCM seal/open for full-size TLS records with bitsliced AES on the VALU.
//
// Same contract as gcm.hip (crypto/aes/gcm.rs:42-157 Gcm::gcm per record, with the record
// framing of net/record.rs:162-240), for the records bs_taken() selects (gcm_common.h):
// 96-bit nonces, aligned buffers, records of >= 1023 full blocks -- the 16 KiB records of
// BASELINE.json's headline configs. The T-table kernel takes every other record.
//
// Why bitsliced: the T-table rounds are bound by LDS lookups (160 ds_read_b32 per block);
// bitsliced AES does the same work as v_bitop3_b32 / v_perm_b32 logic (aes_bs.h: a 94-op S-box
// circuit per byte, MixColumns as XOR networks), about 600 VALU ops per block, leaving the LDS
// to GHASH alone.
//
// Mapping: one wave seals/opens two records, A and B, together. AES block i of a record
// (counter J0 + i; i = 0 is E_K(J0), i >= 1 encrypts data block i - 1) belongs to lane i mod
// 64. A pass covers i in [1024p, 1024p + 1024) of both records: each lane holds one bitsliced
// state of 32 blocks -- plane bits 0-15 are A's blocks 1024p + 64k + lane (k = 0..15), bits
// 16-31 B's. Both records are wave-uniform, so their round keys sit in SGPRs and every round-key
// mask is a scalar value folded into a VALU operand (aes_bs.h Key2); only the counter bits
// differ per lane. After the rounds the keystream is transposed back to blocks and the data
// stream through with one 16-B load/store per lane (1 KiB contiguous per wave instruction).
//   * GHASH: GHASH input slot a = na - 1 + i (na AAD blocks first), so lane l folds the slots
//     congruent to its AES blocks with Horner steps Y <- Y * H^64 ^ B, the multiply being 32
//     lookups in the record's 4-bit table of H^64 (8 KiB LDS per record, gcm_common.h). The
//     lane's AAD block one stride before its first slot is its initial Y; lane 0 starts with AAD
//     block na - 1 (the slot of i = 0, which carries E_K(J0) instead of data).
//   * Blocks after the last full pass (partial data block, length block: <= 1 per lane) run
//     through a scalar T-table AES on an unreplicated 1 KiB T0 in LDS and the general byte path.
//   * Tag: lane l ends at slot a_l; Z = XOR over the wave of Y_l * H^(m - a_l) (bit-serial,
//     1 <= m - a_l <= 64), tag = E_K(J0) ^ Z.
// Occupancy: 256-thread workgroups with __launch_bounds__(256, 2): <= 256 VGPRs, two waves per
// SIMD (a lone wave issues VALU at half rate); LDS 1 KiB + 4 x 16 KiB per workgroup.
#include "gcm_common.h"
// after the HIP headers; fences keep each S-box / column's scalar key masks next to their use
#define ATLS_BS_FENCES 1
#include "aes_bs.h"

namespace atls {
namespace bsk {

constexpr int kWaves = 4;
constexpr uint32_t kT0Bytes = 1024;
constexpr uint32_t kTabBytes = 8192;
constexpr uint32_t kEOff = kT0Bytes + 2 * kWaves * kTabBytes;  // E_K(J0) of A and B, 32 B per wave
constexpr uint32_t kROff = kEOff + 32 * kWaves;                  // Shoup reduction table, 16 words
constexpr size_t kLds = kROff + 64;

using atls_bs::bmask;

// Scalar AES (one block per lane) with the unreplicated T0 at LDS address 0: T0[x] = {2S, S, S,
// 3S} little-endian; T1..T3 are rotations. Only the record tails use it.
template <int NR>
__device__ __forceinline__ void aes_tt1(uint32_t (&s)[4], const uint32_t* rkp) {
#pragma unroll
  for (int w = 0; w < 4; w++) s[w] ^= rkp[w];
#pragma unroll 1
  for (int r = 1; r < NR; r++) {
    uint32_t t[4];
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const uint32_t a = lds_u32((s[c] & 0xffu) << 2);
      const uint32_t b = lds_u32(((s[(c + 1) & 3] >> 8) & 0xffu) << 2);
      const uint32_t cc = lds_u32(((s[(c + 2) & 3] >> 16) & 0xffu) << 2);
      const uint32_t d = lds_u32((s[(c + 3) & 3] >> 24) << 2);
      t[c] = xor3(a, rotl32(b, 8), xor3(rotl32(cc, 16), rotl32(d, 24), rkp[4 * r + c]));
    }
#pragma unroll
    for (int c = 0; c < 4; c++) s[c] = t[c];
  }
  uint32_t t[4];
#pragma unroll
  for (int c = 0; c < 4; c++) {
    const uint32_t a = (lds_u32((s[c] & 0xffu) << 2) >> 8) & 0xffu;
    const uint32_t b = (lds_u32(((s[(c + 1) & 3] >> 8) & 0xffu) << 2) >> 8) & 0xffu;
    const uint32_t cc = (lds_u32(((s[(c + 2) & 3] >> 16) & 0xffu) << 2) >> 8) & 0xffu;
    const uint32_t d = (lds_u32((s[(c + 3) & 3] >> 24) << 2) >> 8) & 0xffu;
    t[c] = (a | (b << 8) | (cc << 16) | (d << 24)) ^ rkp[4 * NR + c];
  }
#pragma unroll
  for (int c = 0; c < 4; c++) s[c] = t[c];
}

typedef uint32_t v32u __attribute__((ext_vector_type(32)));

__device__ __forceinline__ v4u32 ld16(const uint8_t* p) { return *reinterpret_cast<const v4u32*>(p); }
__device__ __forceinline__ void st16(uint8_t* p, v4u32 v) { *reinterpret_cast<v4u32*>(p) = v; }

// Wave-uniform view of one record (SGPRs).
struct RecU {
  const KeySched* k;
  const uint8_t* src;
  uint8_t* dst;
  const uint8_t* aadp;  // RAW mode: AAD bytes
  uint32_t len, n_aead, nb, passes, aad_len, act, tls, ctype;
  uint32_t nraw[3];  // nonce as raw words (J0 = nonce || be32(1))
};

template <bool OPEN>
__device__ __forceinline__ RecU load_rec(const GcmArgs& A, uint32_t r, uint32_t act) {
  RecU u;
  const auto d = cptr(A.recs + (act ? r : 0u));
  u.act = act;
  u.k = A.ks + (act ? d->key_slot : 0u);
  u.src = A.in + d->in_off;
  u.dst = A.out + d->out_off;
  u.tls = d->mode == ATLS_MODE_TLS;
  u.ctype = d->content_type;
  u.len = d->len;
  u.n_aead = (u.tls && !OPEN) ? u.len + 1 : u.len;
  u.nb = (u.n_aead + 15u) / 16u;
  u.passes = act ? (u.len / 16u + 1u) / kBsPass : 0u;
  if (u.tls) {  // key_schedule.rs:51-64: nonce = iv ^ (0^4 || be64(seq))
    const auto siv = cptr(u.k->siv);
    const uint64_t seq = d->seq;
    u.nraw[0] = siv[0];
    u.nraw[1] = siv[1] ^ bswap32((uint32_t)(seq >> 32));
    u.nraw[2] = siv[2] ^ bswap32((uint32_t)seq);
    u.aad_len = 5;
    u.aadp = nullptr;
  } else {
    const uint8_t* iv = A.aux + d->aux_off;
#pragma unroll
    for (int w = 0; w < 3; w++)
      u.nraw[w] = uni((uint32_t)iv[4 * w] | ((uint32_t)iv[4 * w + 1] << 8) | ((uint32_t)iv[4 * w + 2] << 16) |
                      ((uint32_t)iv[4 * w + 3] << 24));
    u.aad_len = d->aad_len;
    u.aadp = iv + 12;
  }
  return u;
}

// This lane's initial GHASH value: lane 0 holds AAD block na-1 (slot of i = 0), lane l >= 65-na
// AAD block na-65+l (one stride before its first slot), zero-padded (bytes.rs:110-121).
__device__ __forceinline__ void init_y(const RecU& u, int lane, uint32_t (&y)[4]) {
  y[0] = y[1] = y[2] = y[3] = 0;
  if (!u.act) return;
  if (u.tls) {
    if (lane == 0) {  // AAD = record header (record.rs:176-183), length truncated to 16 bits
      const uint32_t L = u.n_aead + 16;
      y[0] = 0x17u | (0x03u << 8) | (0x03u << 16) | (((L >> 8) & 0xffu) << 24);
      y[1] = L & 0xffu;
    }
    return;
  }
  const int na = (int)((u.aad_len + 15u) / 16u);
  int ab = -1;
  if (na > 0) ab = lane == 0 ? na - 1 : (na + lane >= 65 ? na + lane - 65 : -1);
  if (ab >= 0) {
    const uint32_t off = 16u * (uint32_t)ab;
#pragma unroll
    for (int q = 0; q < 16; q++)
      if (off + q < u.aad_len) put_byte(y, q, u.aadp[off + q]);
  }
}

// Initial planes of one pass, AddRoundKey(rk0) included. State bytes 0-11 are the records'
// nonces (uniform: bits 0-15 A's, 16-31 B's), bytes 12-15 the big-endian 32-bit counter of
// block k: x + 64 (k mod 16) with x = 1 + 1024p + lane (gcm.rs:89-96, J0's counter is 1).
// Counter bits 0-5 are the lane's; bits 6-31 are (x >> 6) + (k mod 16), a bitsliced ripple
// adder against the constant planes of k mod 16.
__device__ __forceinline__ void init_planes(uint32_t (&pl)[16][8], const RecU& a, const RecU& b,
                                            const atls_bs::Key2& k0, uint32_t x) {
#pragma unroll
  for (int w = 0; w < 3; w++) {
    atls_bs::Key2 nk;
    nk.a[0] = a.nraw[w] ^ k0.a[w];
    nk.b[0] = b.nraw[w] ^ k0.b[w];
#pragma unroll
    for (int bb = 0; bb < 4; bb++)
#pragma unroll
      for (int t = 0; t < 8; t++) pl[4 * w + bb][7 - t] = nk.mask(0, 8 * bb + t);
  }
  uint32_t cp[32];
#pragma unroll
  for (int bt = 0; bt < 6; bt++) cp[bt] = bmask(x, bt);
  const uint32_t y = x >> 6;
  const uint32_t K[4] = {0xAAAAAAAAu, 0xCCCCCCCCu, 0xF0F0F0F0u, 0xFF00FF00u};
  uint32_t c = 0;
#pragma unroll
  for (int j = 0; j < 26; j++) {
    const uint32_t Y = bmask(y, j);
    if (j < 4) {
      cp[6 + j] = xor3(Y, K[j], c);
      c = __builtin_amdgcn_bitop3_b32(Y, K[j], c, 0xE8);  // majority
    } else {
      cp[6 + j] = Y ^ c;
      c = Y & c;
    }
  }
#pragma unroll
  for (int bit = 0; bit < 32; bit++) {
    const int q = 3 - (bit >> 3), t = bit & 7;  // counter byte 12 + q holds bits 8(3-q) ..
    pl[12 + q][7 - t] = cp[bit] ^ k0.mask(3, 8 * q + t);
  }
}

// Round key r of both records (SGPRs). The empty asm pins the words at the point of use: left
// free, the compiler hoists loop-invariant keys (round 0, round NR) and their 128 derived masks
// out of the pass loop, where they overflow the SGPRs.
__device__ __forceinline__ atls_bs::Key2 round_key(const RecU& a, const RecU& b, int r) {
  atls_bs::Key2 k;
  const v4u32 va = *cptr(reinterpret_cast<const v4u32*>(a.k->rk + 4 * r));
  const v4u32 vb = *cptr(reinterpret_cast<const v4u32*>(b.k->rk + 4 * r));
  k.a[0] = va.x; k.a[1] = va.y; k.a[2] = va.z; k.a[3] = va.w;
  k.b[0] = vb.x; k.b[1] = vb.y; k.b[2] = vb.z; k.b[3] = vb.w;
  asm volatile("" : "+s"(k.a[0]), "+s"(k.a[1]), "+s"(k.a[2]), "+s"(k.a[3]), "+s"(k.b[0]), "+s"(k.b[1]),
               "+s"(k.b[2]), "+s"(k.b[3]));
  return k;
}

// One record's tail item (lane's AES block i >= 1024 * passes, or the length block) and its
// GHASH step. Returns the (pos << 8 | byte) of the block's last non-zero plaintext byte, or -1.
template <int NR, bool OPEN>
__device__ __forceinline__ int64_t tail_item(const RecU& u, uint32_t i, uint32_t (&y)[4], uint32_t wb) {
  int64_t lastnz = -1;
  uint32_t B[4] = {0, 0, 0, 0};
  if (i <= u.nb) {
    uint32_t st[4] = {u.nraw[0], u.nraw[1], u.nraw[2], bswap32(1u + i)};
    aes_tt1<NR>(st, u.k->rk);
    const uint32_t off = 16u * (i - 1u);
    const uint32_t valid = min(16u, u.n_aead - off);
    uint32_t P[4] = {0, 0, 0, 0};
    if (off + 16u <= u.len) {
      const v4u32 v = ld16(u.src + off);
      P[0] = v.x; P[1] = v.y; P[2] = v.z; P[3] = v.w;
    } else {
#pragma unroll
      for (int q = 0; q < 16; q++)
        if ((uint32_t)q < valid) put_byte(P, q, (off + q < u.len) ? u.src[off + q] : u.ctype);  // record.rs:173
    }
    uint32_t C[4] = {P[0] ^ st[0], P[1] ^ st[1], P[2] ^ st[2], P[3] ^ st[3]};
    if (valid < 16u) {
#pragma unroll
      for (int w = 0; w < 4; w++) {
        const int lo = 4 * w;
        if ((int)valid < lo + 4) C[w] &= ((int)valid <= lo) ? 0u : (0xffffffffu >> (8 * (lo + 4 - valid)));
      }
#pragma unroll
      for (int q = 0; q < 16; q++)
        if ((uint32_t)q < valid) u.dst[off + q] = (uint8_t)get_byte(C, q);
    } else {
      const v4u32 cv = {C[0], C[1], C[2], C[3]};
      st16(u.dst + off, cv);
    }
#pragma unroll
    for (int w = 0; w < 4; w++) B[w] = OPEN ? P[w] : C[w];
    if (OPEN && u.tls) {
      const int j = last_nonzero(C, (int)valid);
      if (j >= 0) lastnz = ((int64_t)(off + j) << 8) | get_byte(C, j);
    }
  } else {  // length block: [len(A)]_64 || [len(C)]_64 in bits (gcm.rs:121)
    const uint64_t abits = (uint64_t)u.aad_len * 8u, cbits = (uint64_t)u.n_aead * 8u;
    B[0] = bswap32((uint32_t)(abits >> 32)); B[1] = bswap32((uint32_t)abits);
    B[2] = bswap32((uint32_t)(cbits >> 32)); B[3] = bswap32((uint32_t)cbits);
  }
  ghash_mul_tab(y, wb);
#pragma unroll
  for (int w = 0; w < 4; w++) y[w] ^= B[w];
  return lastnz;
}

// z = y * g in GF(2^128) (be words), Shoup's 4-bit method: a per-lane table of the 16 nibble
// multiples of g in LDS at tb (256 B per lane, entry n at ((n ^ lane) & 15) * 16 to spread banks)
// and the 16-word reduction table at kROff. 32 steps of z <- z * x^4 ^ M[nibble], about 11 VALU
// each, instead of 128 bit-serial steps. Same product as gf_mul_be (gcm.rs:21-40 gmult).
__device__ __forceinline__ void gf_mul_shoup(const uint32_t (&y)[4], const uint32_t (&g)[4], uint32_t tb, int lane,
                                             uint32_t (&z)[4]) {
  uint32_t P0[4], P1[4], P2[4], P3[4];
#pragma unroll
  for (int w = 0; w < 4; w++) P0[w] = P1[w] = g[w];
  gf_mulx_be(P1);
#pragma unroll
  for (int w = 0; w < 4; w++) P2[w] = P1[w];
  gf_mulx_be(P2);
#pragma unroll
  for (int w = 0; w < 4; w++) P3[w] = P2[w];
  gf_mulx_be(P3);
  const uint32_t sw = (uint32_t)lane & 15u;
#pragma unroll
  for (int n = 0; n < 16; n++) {
    v4u32 e;
    e.x = ((n & 8) ? P0[0] : 0u) ^ ((n & 4) ? P1[0] : 0u) ^ ((n & 2) ? P2[0] : 0u) ^ ((n & 1) ? P3[0] : 0u);
    e.y = ((n & 8) ? P0[1] : 0u) ^ ((n & 4) ? P1[1] : 0u) ^ ((n & 2) ? P2[1] : 0u) ^ ((n & 1) ? P3[1] : 0u);
    e.z = ((n & 8) ? P0[2] : 0u) ^ ((n & 4) ? P1[2] : 0u) ^ ((n & 2) ? P2[2] : 0u) ^ ((n & 1) ? P3[2] : 0u);
    e.w = ((n & 8) ? P0[3] : 0u) ^ ((n & 4) ? P1[3] : 0u) ^ ((n & 2) ? P2[3] : 0u) ^ ((n & 1) ? P3[3] : 0u);
    *reinterpret_cast<__attribute__((address_space(3))) v4u32*>(tb + ((n ^ sw) << 4)) = e;
  }
  wave_lds_sync();
  uint32_t z0 = 0, z1 = 0, z2 = 0, z3 = 0;
#pragma unroll
  for (int q = 31; q >= 0; q--) {
    if (q != 31) {  // z <- z * x^4: shift right 4, fold the 4 bits shifted out (x^124..x^127)
      const uint32_t r = lds_u32(kROff + ((z3 & 15u) << 2));
      z3 = __builtin_amdgcn_alignbit(z2, z3, 4);
      z2 = __builtin_amdgcn_alignbit(z1, z2, 4);
      z1 = __builtin_amdgcn_alignbit(z0, z1, 4);
      z0 = (z0 >> 4) ^ r;
    }
    const uint32_t nib = (y[q >> 3] >> (28 - 4 * (q & 7))) & 15u;  // coefficients x^4q .. x^(4q+3)
    const v4u32 m = lds_u4(tb + ((nib ^ sw) << 4));
    z0 ^= m.x; z1 ^= m.y; z2 ^= m.z; z3 ^= m.w;
  }
  z[0] = z0; z[1] = z1; z[2] = z2; z[3] = z3;
}

// Tag / open result of one record: combine the lanes' Horner values, add E_K(J0).
template <bool OPEN>
__device__ __forceinline__ void finish(const GcmArgs& A, const RecU& u, uint32_t r, const uint32_t (&y)[4],
                                       uint32_t e_addr, uint32_t tb, int64_t lastnz, int lane) {
  uint32_t z[4] = {0, 0, 0, 0};
  {
    const uint32_t l = (uint32_t)lane;
    const uint32_t i_last = l + 64u * ((u.nb + 1u - l) / 64u);
    const uint32_t e = u.nb + 2u - i_last;  // 1..64
    const uint32_t yb[4] = {bswap32(y[0]), bswap32(y[1]), bswap32(y[2]), bswap32(y[3])};
    uint32_t hp[4];
#pragma unroll
    for (int w = 0; w < 4; w++) hp[w] = u.k->hpow_be[e - 1][w];
    gf_mul_shoup(yb, hp, tb, lane, z);
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
#pragma unroll
    for (int w = 0; w < 4; w++) z[w] ^= __shfl_xor(z[w], off, 64);
  }
  if (OPEN) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      const int64_t o = __shfl_xor(lastnz, off, 64);
      lastnz = o > lastnz ? o : lastnz;
    }
  }
  if (lane == 0) {
    const v4u32 ev = lds_u4(e_addr);
    const uint32_t t0 = ev.x ^ bswap32(z[0]), t1 = ev.y ^ bswap32(z[1]), t2 = ev.z ^ bswap32(z[2]),
                   t3 = ev.w ^ bswap32(z[3]);
    if (!OPEN) {
      const v4u32 tv = {t0, t1, t2, t3};
      st16(A.tags_out + 16ull * r, tv);
    } else {
      const uint32_t* tg = reinterpret_cast<const uint32_t*>(A.tags_in + 16ull * r);
      const bool ok = (tg[0] == t0) & (tg[1] == t1) & (tg[2] == t2) & (tg[3] == t3);
      write_open_result(A, r, u.tls, u.len, ok, lastnz);
    }
  }
}

// Data block index loaded for AES block i (block 0, E_K(J0), loads block 0 and ignores it).
__device__ __forceinline__ uint32_t didx(uint32_t i) { return i ? i - 1u : 0u; }

template <int NR, bool OPEN>
__device__ __forceinline__ void bs_pair(const GcmArgs& A, uint32_t rA, uint32_t actA, uint32_t actB, uint32_t wbA, uint32_t wbB,
                        uint32_t eA, int lane) {
  const RecU a = load_rec<OPEN>(A, rA, actA);
  const RecU b = load_rec<OPEN>(A, rA + 1u, actB);
  const uint32_t eB = eA + 16u;
  uint32_t yA[4], yB[4];
  init_y(a, lane, yA);
  init_y(b, lane, yB);
  {
    const int p = lane >> 1, n0 = (lane & 1) * 8;
    uint32_t seed[4];
#pragma unroll
    for (int w = 0; w < 4; w++) seed[w] = a.k->p4_be[p][w];
    ghash_table_entries<8>(wbA, seed, p, n0);
#pragma unroll
    for (int w = 0; w < 4; w++) seed[w] = b.k->p4_be[p][w];
    ghash_table_entries<8>(wbB, seed, p, n0);
  }
  wave_lds_sync();

  uint32_t lzA = 0, lzB = 0;  // OPEN+TLS: AES index of the last block with a non-zero byte (0: none)
  const uint32_t p_wave = max(a.passes, b.passes);
#pragma unroll 1
  for (uint32_t p = 0; p < p_wave; p++) {
    const bool pa = p < a.passes, pb = p < b.passes;  // wave-uniform
    const uint32_t ibase = kBsPass * p + (uint32_t)lane;
    uint32_t pl[16][8];
    init_planes(pl, a, b, round_key(a, b, 0), 1u + ibase);
#pragma unroll 1
    for (int rr = 1; rr <= NR; rr++) {  // one copy of the S-box code for all rounds (I-cache)
      const atls_bs::Key2 km = round_key(a, b, rr);
      atls_bs::sub_bytes(pl);
      if (rr < NR) atls_bs::shift_mix_ark(pl, km);
      else atls_bs::shift_ark(pl, km);
    }
    v32u ks[4];  // keystream word w of block s = ks[w][s]; read with a uniform dynamic index
    {
      uint32_t kb[4][32];
      atls_bs::planes_to_blocks(pl, kb);
#pragma unroll
      for (int w = 0; w < 4; w++)
#pragma unroll
        for (int k = 0; k < 32; k++) ks[w][k] = kb[w][k];
    }
    // Stream the 32 blocks, 4 per iteration: iterations 0-3 record A, 4-7 record B (y / lz hold
    // the current record's values, swapped at the switch). Loads run one iteration ahead; a
    // record without this pass reads the other's blocks (always valid) and ignores them.
    const uint8_t* srcA = pa ? a.src : b.src;
    const uint8_t* srcB = pb ? b.src : a.src;
    v4u32 Pd[4];
#pragma unroll
    for (int j = 0; j < 4; j++) Pd[j] = ld16(srcA + 16u * didx(ibase + 64u * j));
#pragma unroll 1
    for (int it = 0; it < 8; it++) {
      if (it == 4) {
#pragma unroll
        for (int w = 0; w < 4; w++) { const uint32_t t = yA[w]; yA[w] = yB[w]; yB[w] = t; }
        const uint32_t t = lzA; lzA = lzB; lzB = t;
      }
      const bool recA = it < 4;
      const bool on = recA ? pa : pb;
      uint8_t* dst = recA ? a.dst : b.dst;
      const uint32_t wb = recA ? wbA : wbB;
      const bool tls = recA ? a.tls : b.tls;
      v4u32 Pn[4];
      if (it < 7) {
        const uint8_t* nsrc = it + 1 < 4 ? srcA : srcB;
#pragma unroll
        for (int j = 0; j < 4; j++) Pn[j] = ld16(nsrc + 16u * didx(ibase + 64u * (uint32_t)((4 * (it + 1) + j) & 15)));
      }
      if (on) {
#pragma unroll
        for (int j = 0; j < 4; j++) {
          const int st = 4 * it + j;
          const uint32_t i = ibase + 64u * (uint32_t)(st & 15);
          const v4u32 K = {ks[0][st], ks[1][st], ks[2][st], ks[3][st]};
          const v4u32 P = Pd[j];
          if (j == 0 && i == 0) {  // E_K(J0): lane 0 of pass 0; its GHASH slot (AAD) is already in y
            *reinterpret_cast<__attribute__((address_space(3))) v4u32*>(recA ? eA : eA + 16u) = K;
          } else {
            const v4u32 C = P ^ K;
            st16(dst + 16u * (i - 1u), C);
            const v4u32 Bv = OPEN ? P : C;
            if (OPEN && tls && (C.x | C.y | C.z | C.w) != 0u) lzA = i;
            ghash_mul_tab<true>(yA, wb);
            yA[0] ^= Bv.x; yA[1] ^= Bv.y; yA[2] ^= Bv.z; yA[3] ^= Bv.w;
          }
        }
      }
#pragma unroll
      for (int j = 0; j < 4; j++) Pd[j] = Pn[j];
    }
#pragma unroll
    for (int w = 0; w < 4; w++) { const uint32_t t = yA[w]; yA[w] = yB[w]; yB[w] = t; }
    { const uint32_t t = lzA; lzA = lzB; lzB = t; }
  }

  // ---- tails (<= 1 item per lane and record), then tags ----
  int64_t nzA = -1, nzB = -1;
  if (OPEN) {  // exact last non-zero byte of the pass blocks: reread this lane's own plaintext store
    if (lzA != 0) {
      const uint32_t off = 16u * (lzA - 1u);
      const v4u32 v = ld16(a.dst + off);
      const uint32_t c[4] = {v.x, v.y, v.z, v.w};
      const int j = last_nonzero(c, 16);
      nzA = ((int64_t)(off + (uint32_t)j) << 8) | get_byte(c, j);
    }
    if (lzB != 0) {
      const uint32_t off = 16u * (lzB - 1u);
      const v4u32 v = ld16(b.dst + off);
      const uint32_t c[4] = {v.x, v.y, v.z, v.w};
      const int j = last_nonzero(c, 16);
      nzB = ((int64_t)(off + (uint32_t)j) << 8) | get_byte(c, j);
    }
  }
  if (a.act) {
    const uint32_t i = kBsPass * a.passes + (uint32_t)lane;
    if (i <= a.nb + 1u) {
      const int64_t t = tail_item<NR, OPEN>(a, i, yA, wbA);
      nzA = t > nzA ? t : nzA;
    }
  }
  if (b.act) {
    const uint32_t i = kBsPass * b.passes + (uint32_t)lane;
    if (i <= b.nb + 1u) {
      const int64_t t = tail_item<NR, OPEN>(b, i, yB, wbB);
      nzB = t > nzB ? t : nzB;
    }
  }
  wave_lds_sync();  // GHASH tables are dead: their 16 KiB hold the lanes' combine tables
  const uint32_t tb = wbA + 256u * (uint32_t)lane;
  if (a.act) finish<OPEN>(A, a, rA, yA, eA, tb, nzA, lane);
  wave_lds_sync();
  if (b.act) finish<OPEN>(A, b, rA + 1u, yB, eB, tb, nzB, lane);
}

template <bool OPEN, int NR>
__global__ __launch_bounds__(64 * kWaves, 2) void gcm_bs_kernel(GcmArgs A) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) smem[i] = A.t0[i];
  if (threadIdx.x < 16) {  // R[r] = r(x) * x^128 mod P for the 4 bits leaving z * x^4 (bit 3 = x^124)
    const uint32_t r = threadIdx.x;
    smem[kROff / 4 + r] = ((r & 8) ? 0xE1000000u : 0u) ^ ((r & 4) ? 0x70800000u : 0u) ^ ((r & 2) ? 0x38400000u : 0u) ^
                          ((r & 1) ? 0x1C200000u : 0u);
  }
  __syncthreads();
  const int wave = (int)uni(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const uint32_t wbA = kT0Bytes + (uint32_t)wave * 2u * kTabBytes, wbB = wbA + kTabBytes;
  const uint32_t eA = kEOff + 32u * (uint32_t)wave;
  const uint32_t npairs = (A.n + 1u) / 2u;
  for (uint32_t q = blockIdx.x * kWaves + wave; q < npairs; q += gridDim.x * kWaves) {
    const uint32_t rA = 2u * q;
    const uint32_t cA = uni(bs_taken<OPEN>(A, rA));
    const uint32_t cB = rA + 1u < A.n ? uni(bs_taken<OPEN>(A, rA + 1u)) : 0u;
    if ((cA ? cA : cB) != (uint32_t)NR) continue;
    bs_pair<NR, OPEN>(A, rA, cA != 0, cB != 0, wbA, wbB, eA, lane);
    wave_lds_sync();  // this pair's table reads are done before the next pair rebuilds them
  }
}

}  // namespace bsk
}  // namespace atls

// Bitsliced kernels over the records bs_taken() accepts. nr_mask: bit 0/1/2 = some key slot
// has 10/12/14 rounds (one launch each).
extern "C" int atls_launch_gcm_bs(int open, const void* ks, const atls_rec* recs, uint32_t n, const uint8_t* in,
                                  const uint8_t* aux, uint8_t* out, uint8_t* tags_out, const uint8_t* tags_in,
                                  atls_open_result* res, const uint32_t* t0, uint32_t* err, uint32_t n_slots,
                                  int nr_mask, int grid, hipStream_t s) {
  if (n == 0) return 0;
  atls::GcmArgs A{(const atls::KeySched*)ks, recs, n, in, aux, out, tags_out, tags_in, res, t0, err, n_slots, 1u};
  const uint32_t want = ((n + 1) / 2 + atls::bsk::kWaves - 1) / atls::bsk::kWaves;
  const dim3 g((uint32_t)grid < want ? (uint32_t)grid : want), blk(64 * atls::bsk::kWaves);
  const size_t lds = atls::bsk::kLds;
#define ATLS_BS_LAUNCH(NR)                                                                 \
  if (open) hipLaunchKernelGGL((atls::bsk::gcm_bs_kernel<true, NR>), g, blk, lds, s, A);   \
  else hipLaunchKernelGGL((atls::bsk::gcm_bs_kernel<false, NR>), g, blk, lds, s, A);
  if (nr_mask & 1) { ATLS_BS_LAUNCH(10) }
  if (nr_mask & 2) { ATLS_BS_LAUNCH(12) }
  if (nr_mask & 4) { ATLS_BS_LAUNCH(14) }
#undef ATLS_BS_LAUNCH
  return hipGetLastError() == hipSuccess ? 0 : ATLS_INTERNAL_ERROR;
}
