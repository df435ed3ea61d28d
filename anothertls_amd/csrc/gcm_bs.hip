// AES-GCM seal/open for full-size TLS records with bitsliced AES on the VALU.
//
// Same contract as gcm.hip (crypto/aes/gcm.rs:42-157 Gcm::gcm per record, with the record
// framing of net/record.rs:162-240), for the records bs_taken() selects (gcm_common.h):
// 96-bit nonces, aligned buffers, records of >= 1023 full blocks -- the 16 KiB records of
// BASELINE.json's headline configs. The T-table kernel takes every other record.
//
// Why bitsliced: the T-table rounds are bound by LDS lookups (160 ds_read_b32 per block);
// bitsliced AES does the same work as v_bitop3_b32 / v_perm_b32 logic (aes_bs.h: a 94-op S-box
// circuit per byte, MixColumns as XOR networks), about 650 VALU ops per block, leaving the LDS
// to GHASH alone.
//
// Mapping: one record per half-wave (lanes 32h .. 32h+31), two records per wave. AES block i of
// a record (counter J0 + i; i = 0 is E_K(J0), i >= 1 encrypts data block i - 1) belongs to lane
// i mod 32. A pass covers i in [1024p, 1024p + 1024): each lane encrypts its 32 counter blocks
// 1024p + 32k + lane as one bitsliced state (aes_bs.h row-plane layout; the lane's round keys
// become 32 byte-mask words per round), transposes the keystream back to blocks and
// streams the data through with one 16-B load/store per lane (512 B contiguous per half-wave).
//   * GHASH: GHASH input slot a = na - 1 + i (na AAD blocks first), so lane l folds the slots
//     congruent to its AES blocks with Horner steps Y <- Y * H^32 ^ B, the multiply being 32
//     lookups in the record's 4-bit table of H^32 (8 KiB LDS per record, gcm_common.h). The
//     lane's AAD block one stride before its first slot is its initial Y; lane 0 starts with AAD
//     block na - 1 (the slot of i = 0, which carries E_K(J0) instead of data).
//   * Blocks after the last full pass (partial data block, length block: <= 2 per lane) run
//     through a scalar T-table AES on an unreplicated 1 KiB T0 in LDS and the general byte path,
//     the first one per lane before the passes (its GHASH input parked in LDS).
//   * Tag: lane l ends at slot a_l; Z = XOR over the half-wave of Y_l * H^(m - a_l) (Shoup 4-bit
//     multiply on a per-lane LDS table, 1 <= m - a_l <= 32), tag = E_K(J0) ^ Z.
// Occupancy: 256-thread workgroups with __launch_bounds__(256, 2): <= 256 VGPRs, two waves per
// SIMD (a lone wave issues VALU at half rate); LDS 1 KiB + 4 x 16 KiB per workgroup.
#include "gcm_common.h"
// after the HIP headers:
#include "aes_bs.h"

namespace atls {
namespace bsk {

constexpr int kWaves = 4;
constexpr uint32_t kT0Bytes = 1024;
constexpr uint32_t kTabBytes = 8192;
constexpr uint32_t kEOff = kT0Bytes + 2 * kWaves * kTabBytes;  // E_K(J0) per half-wave, 16 B each
constexpr uint32_t kSlotOff = kEOff + 32 * kWaves;               // per lane: parked tail item, 32 B
constexpr size_t kLds = kSlotOff + 64 * 32 * kWaves;

using atls_bs::bmask;

typedef uint32_t v32u __attribute__((ext_vector_type(32)));

// Phase timing (build with -DATLS_BS_STAMPS): per-phase shader-clock totals summed over all
// waves, read back with atls_debug_bs_stamps(). 0 setup, 1 AES rounds + transpose, 2 data
// stream + GHASH, 3 tails, 4 tag combine, 5 pairs.
#ifdef ATLS_BS_STAMPS
__device__ unsigned long long g_bs_stamps[8];
#define BS_STAMP(var) const uint64_t var = __builtin_amdgcn_s_memtime()
#else
#define BS_STAMP(var)
#endif

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

// Global (not flat) accesses: a flat load also counts in lgkmcnt, so every LDS wait of the GHASH
// steps would wait for the data loads in flight as well.
typedef __attribute__((address_space(1))) const v4u32 gv4c;
typedef __attribute__((address_space(1))) v4u32 gv4;
__device__ __forceinline__ v4u32 ld16(const uint8_t* p) { return *(gv4c*)(p); }
__device__ __forceinline__ void st16(uint8_t* p, v4u32 v) { *(gv4*)(p) = v; }
__device__ __forceinline__ v4u32 ld_rk(const uint32_t* rk, int r) { return *reinterpret_cast<const v4u32*>(rk + 4 * r); }

// One record as this lane sees it.
struct Rec {
  const KeySched* k;
  const uint8_t* src;
  uint8_t* dst;
  const uint8_t* aadp;  // RAW mode: AAD bytes
  uint32_t len, n_aead, nb, passes, aad_len, tls, ctype;
  uint32_t nraw[3];  // nonce as raw words (J0 = nonce || be32(1))
};

template <bool OPEN>
__device__ __forceinline__ Rec load_rec(const GcmArgs& A, uint32_t r, bool act) {
  Rec u;
  const atls_rec d = A.recs[act ? r : 0u];
  u.k = A.ks + (act ? d.key_slot : 0u);
  u.src = A.in + d.in_off;
  u.dst = A.out + d.out_off;
  u.tls = d.mode == ATLS_MODE_TLS;
  u.ctype = d.content_type;
  u.len = d.len;
  u.n_aead = (u.tls && !OPEN) ? u.len + 1 : u.len;
  u.nb = (u.n_aead + 15u) / 16u;
  u.passes = act ? (u.len / 16u + 1u) / kBsPass : 0u;
  if (u.tls) {  // key_schedule.rs:51-64: nonce = iv ^ (0^4 || be64(seq))
    u.nraw[0] = u.k->siv[0];
    u.nraw[1] = u.k->siv[1] ^ bswap32((uint32_t)(d.seq >> 32));
    u.nraw[2] = u.k->siv[2] ^ bswap32((uint32_t)d.seq);
    u.aad_len = 5;
    u.aadp = nullptr;
  } else {
    const uint8_t* iv = A.aux + d.aux_off;
#pragma unroll
    for (int w = 0; w < 3; w++)
      u.nraw[w] = (uint32_t)iv[4 * w] | ((uint32_t)iv[4 * w + 1] << 8) | ((uint32_t)iv[4 * w + 2] << 16) |
                  ((uint32_t)iv[4 * w + 3] << 24);
    u.aad_len = d.aad_len;
    u.aadp = iv + 12;
  }
  return u;
}

// This lane's initial GHASH value: lane 0 holds AAD block na-1 (slot of i = 0), lane l >= 33-na
// AAD block na-33+l (one stride before its first slot), zero-padded (bytes.rs:110-121).
__device__ __forceinline__ void init_y(const Rec& u, bool act, int l, uint32_t (&y)[4]) {
  y[0] = y[1] = y[2] = y[3] = 0;
  if (!act) return;
  if (u.tls) {
    if (l == 0) {  // AAD = record header (record.rs:176-183), length truncated to 16 bits
      const uint32_t L = u.n_aead + 16;
      y[0] = 0x17u | (0x03u << 8) | (0x03u << 16) | (((L >> 8) & 0xffu) << 24);
      y[1] = L & 0xffu;
    }
    return;
  }
  const int na = (int)((u.aad_len + 15u) / 16u);
  int ab = -1;
  if (na > 0) ab = l == 0 ? na - 1 : (na + l >= 33 ? na + l - 33 : -1);
  if (ab >= 0) {
    const uint32_t off = 16u * (uint32_t)ab;
#pragma unroll
    for (int q = 0; q < 16; q++)
      if (off + q < u.aad_len) put_byte(y, q, u.aadp[off + q]);
  }
}

// Initial state of one pass, AddRoundKey(rk0) included (aes_bs.h row-plane layout). Columns 0-2
// are the nonce (the same for all 32 blocks: all-0 / all-1 bytes), column 3 the big-endian
// 32-bit counter of block k = 8g + b: x + 32k with x = 1 + 1024p + lane (gcm.rs:89-96, J0's
// counter is 1). Counter bits 0-4 are the lane's; bits 5-31 are ((x + 256g) >> 5) + b, a
// bitsliced ripple adder against the constant patterns of b in byte 3 of each word.
__device__ __forceinline__ void init_state(atls_bs::State& st, const uint32_t (&nraw)[3], const v4u32 rk0,
                                           uint32_t x) {
  atls_bs::Masks m;
  {
    const uint32_t w[4] = {nraw[0] ^ rk0.x, nraw[1] ^ rk0.y, nraw[2] ^ rk0.z, rk0.w};
    atls_bs::make_masks(w, m);
  }
  const uint32_t B[3] = {0xAA000000u, 0xCC000000u, 0xF0000000u};
#pragma unroll
  for (int g = 0; g < 4; g++) {
    const uint32_t base = x + 256u * (uint32_t)g;
    uint32_t cp[32];
#pragma unroll
    for (int b = 0; b < 5; b++) cp[b] = bmask(base, b);
    const uint32_t y = base >> 5;
    uint32_t c = 0;
#pragma unroll
    for (int j = 0; j < 27; j++) {
      const uint32_t Y = bmask(y, j);
      if (j < 3) {
        cp[5 + j] = xor3(Y, B[j], c);
        c = __builtin_amdgcn_bitop3_b32(Y, B[j], c, 0xE8);  // majority
      } else {
        cp[5 + j] = Y ^ c;
        c = Y & c;
      }
    }
#pragma unroll
    for (int r = 0; r < 4; r++)
#pragma unroll
      for (int t = 0; t < 8; t++)  // row r of column 3 = counter byte 3 - r (big-endian)
        st[g][r][7 - t] = __builtin_amdgcn_bitop3_b32(m[r][7 - t], cp[8 * (3 - r) + t], 0xFF000000u, 0x78);  // m ^ (cp & C)
  }
}

// One tail item (AES block i >= 1024 * passes, or the length block): encrypts / decrypts and
// stores it, returns its GHASH input in B and the (pos << 8 | byte) of its last non-zero
// plaintext byte (or -1).
template <int NR, bool OPEN>
__device__ __forceinline__ int64_t tail_block(const Rec& u, uint32_t i, uint32_t (&B)[4]) {
  int64_t lastnz = -1;
  B[0] = B[1] = B[2] = B[3] = 0;
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
  return lastnz;
}

// z = y * g in GF(2^128) (be words), Shoup's 4-bit method: a per-lane table of the 16 nibble
// multiples of g in LDS at tb (256 B per lane, entry n at ((n ^ lane) & 15) * 16 to spread banks)
// read back once per nibble up front; then 31 VALU steps z <- z * x^4 ^ M[nibble] instead of 128
// bit-serial ones. Same product as gf_mul_be (gcm.rs:21-40 gmult).
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
  // the 32 lookups depend only on y: issue them all, then run the chain on the VALU
  v4u32 M[32];
#pragma unroll
  for (int q = 0; q < 32; q++) {
    const uint32_t nib = (y[q >> 3] >> (28 - 4 * (q & 7))) & 15u;  // coefficients x^4q .. x^(4q+3)
    M[q] = lds_u4(tb + ((nib ^ sw) << 4));
  }
  uint32_t z0 = M[31].x, z1 = M[31].y, z2 = M[31].z, z3 = M[31].w;
#pragma unroll
  for (int q = 30; q >= 0; q--) {
    // z <- z * x^4: shift right 4 and fold the 4 bits shifted out (x^124..x^127): bit 3 of them
    // (x^124) becomes x^128 = 1 + x + x^2 + x^7 (0xE1 << 24), the others the same shifted right
    const uint32_t r = (bmask(z3, 3) & 0xE1000000u) ^ (bmask(z3, 2) & 0x70800000u) ^ (bmask(z3, 1) & 0x38400000u) ^
                       (bmask(z3, 0) & 0x1C200000u);
    z3 = __builtin_amdgcn_alignbit(z2, z3, 4);
    z2 = __builtin_amdgcn_alignbit(z1, z2, 4);
    z1 = __builtin_amdgcn_alignbit(z0, z1, 4);
    z0 = xor3(z0 >> 4, r, M[q].x);
    z1 ^= M[q].y; z2 ^= M[q].z; z3 ^= M[q].w;
  }
  z[0] = z0; z[1] = z1; z[2] = z2; z[3] = z3;
}

// Data block index loaded for AES block i (block 0, E_K(J0), loads block 0 and ignores it).
__device__ __forceinline__ uint32_t didx(uint32_t i) { return i ? i - 1u : 0u; }

template <int NR, bool OPEN>
__device__ __forceinline__ void bs_pair(const GcmArgs& A, uint32_t r, bool act, uint32_t wb, uint32_t eaddr,
                                        uint32_t slot, int l, int lane) {
  BS_STAMP(t_start);
  uint64_t t_rounds = 0, t_data = 0;
  (void)t_rounds; (void)t_data;
  uint32_t y[4];
  const uint32_t* rkp;
  const uint8_t* src0;
  uint8_t* dst;
  uint32_t nraw[3], passes, tls;
  {  // only what the passes need stays live through them; the rest is reloaded for the tail
    const Rec u = load_rec<OPEN>(A, r, act);
    init_y(u, act, l, y);
    uint32_t seed[4];
#pragma unroll
    for (int w = 0; w < 4; w++) seed[w] = u.k->p4h32_be[l][w];
    ghash_table_entries<16>(wb, seed, l, 0);
    rkp = u.k->rk;
    src0 = u.src;
    dst = u.dst;
    nraw[0] = u.nraw[0]; nraw[1] = u.nraw[1]; nraw[2] = u.nraw[2];
    passes = u.passes;
    tls = u.tls;
    // The lane's first tail item (AES block 1024 * passes + l, or the length block) is done now,
    // with the record at hand; its GHASH input and the record scalars wait in LDS for the end of
    // the chain. Later items (only records whose tail passes 32 blocks) are done at the end.
    uint32_t B[4];
    const uint32_t i0 = kBsPass * u.passes + (uint32_t)l;
    int64_t nz0 = -1;
    if (act && i0 <= u.nb + 1u) nz0 = tail_block<NR, OPEN>(u, i0, B);
    const v4u32 bv = {B[0], B[1], B[2], B[3]};
    const v4u32 sv = {(uint32_t)nz0, (uint32_t)(nz0 >> 32), u.nb, u.len};
    *reinterpret_cast<__attribute__((address_space(3))) v4u32*>(slot) = bv;
    *reinterpret_cast<__attribute__((address_space(3))) v4u32*>(slot + 16u) = sv;
  }
  // a half-wave without the current pass loads the other half's blocks (always valid) and ignores
  // them; the shuffle runs here, with every lane active (ds_bpermute from an inactive lane is 0)
  const uint8_t* src_other = (const uint8_t*)(uintptr_t)__shfl_xor((unsigned long long)(uintptr_t)src0, 32, 64);
  wave_lds_sync();

  uint32_t lz = 0;  // OPEN+TLS: AES index of the last pass block with a non-zero byte (0: none)
  const uint32_t p_wave = max(__builtin_amdgcn_readlane(passes, 0), __builtin_amdgcn_readlane(passes, 32));
  BS_STAMP(t_setup);
#pragma unroll 1
  for (uint32_t p = 0; p < p_wave; p++) {
    BS_STAMP(t_pstart);
    const bool pact = p < passes;
    const uint32_t ibase = kBsPass * p + (uint32_t)l;
    const uint8_t* src = pact ? src0 : src_other;
    atls_bs::State st;
    init_state(st, nraw, ld_rk(rkp, 0), 1u + ibase);
    v4u32 kn = ld_rk(rkp, 1);
#pragma unroll 1
    for (int rr = 1; rr < NR; rr++) {
      v4u32 kv = kn;
      kn = ld_rk(rkp, rr + 1);  // in flight during this round's S-boxes
      atls_bs::sub_bytes(st);
      // pin the key here: left free, the scheduler builds the 32 masks before the S-boxes
      asm volatile("" : "+v"(kv.x), "+v"(kv.y), "+v"(kv.z), "+v"(kv.w));
      atls_bs::Masks m;
      {
        const uint32_t w[4] = {kv.x, kv.y, kv.z, kv.w};
        atls_bs::make_masks(w, m);
      }
      atls_bs::shift_mix_ark(st, m);
    }
    v4u32 Pd[4];  // the first data loads go out under the last round and the transposes
#pragma unroll
    for (int j = 0; j < 4; j++) Pd[j] = ld16(src + 16u * didx(ibase + 32u * j));
    __builtin_amdgcn_sched_barrier(0);
    atls_bs::sub_bytes(st);  // last round (a second copy of the S-box code)
    {
      atls_bs::Masks m;
      const uint32_t w[4] = {kn.x, kn.y, kn.z, kn.w};
      atls_bs::make_masks(w, m);
      atls_bs::shift_ark(st, m);
    }
    uint32_t ks[4][32];  // keystream word c of block k
#pragma unroll
    for (int g = 0; g < 4; g++) {
      uint32_t x[32];
      atls_bs::group_to_blocks(st[g], x);
#pragma unroll
      for (int c = 0; c < 4; c++)
#pragma unroll
        for (int b = 0; b < 8; b++) ks[c][8 * g + b] = x[8 * c + b];
    }
    BS_STAMP(t_p1);
    // Stream the 32 blocks (fully unrolled: the load ring stays in fixed registers, so no copy
    // waits on a load in flight); each step's load slot is refilled for the step 4 ahead.
#pragma unroll
    for (int kk = 0; kk < 32; kk++) {
      const uint32_t i = ibase + 32u * (uint32_t)kk;
      const v4u32 P = Pd[kk & 3];
      if (kk + 4 < 32) Pd[kk & 3] = ld16(src + 16u * (i + 127u));  // block kk + 4: data index i + 128 - 1
      if (pact) {
        const v4u32 K = {ks[0][kk], ks[1][kk], ks[2][kk], ks[3][kk]};
        const v4u32 C = P ^ K;
        const v4u32 Bv = OPEN ? P : C;
        if (kk == 0 && i == 0) {
          // E_K(J0): lane 0 of pass 0; its GHASH slot (AAD) is already in y, so no store and no step
          *reinterpret_cast<__attribute__((address_space(3))) v4u32*>(eaddr) = K;
        } else {
          st16(dst + 16u * (i - 1u), C);
          if (OPEN && tls && (C.x | C.y | C.z | C.w) != 0u) lz = i;
        }
        uint32_t yn[4] = {y[0], y[1], y[2], y[3]};
        ghash_mul_tab<8>(yn, wb);
        if (kk == 0 && i == 0) {
          yn[0] = y[0]; yn[1] = y[1]; yn[2] = y[2]; yn[3] = y[3];
        } else {
          yn[0] ^= Bv.x; yn[1] ^= Bv.y; yn[2] ^= Bv.z; yn[3] ^= Bv.w;
        }
        y[0] = yn[0]; y[1] = yn[1]; y[2] = yn[2]; y[3] = yn[3];
      }
    }
#ifdef ATLS_BS_STAMPS
    const uint64_t t_p2 = __builtin_amdgcn_s_memtime();
    t_rounds += t_p1 - t_pstart;
    t_data += t_p2 - t_p1;
#endif
  }

  // ---- tail: the parked first item, any further ones, then the tag ----
  const v4u32 bv = lds_u4(slot), sv = lds_u4(slot + 16u);
  const uint32_t nb = sv.z, len = sv.w;
  int64_t nz = (int64_t)(((uint64_t)sv.y << 32) | sv.x);
  const uint32_t i0 = kBsPass * passes + (uint32_t)l;
  if (act && i0 <= nb + 1u) {
    ghash_mul_tab(y, wb);
    y[0] ^= bv.x; y[1] ^= bv.y; y[2] ^= bv.z; y[3] ^= bv.w;
  }
  if (OPEN && lz != 0) {  // exact last non-zero byte of the pass blocks: reread this lane's own store
    const uint32_t off = 16u * (lz - 1u);
    const v4u32 v = ld16(dst + off);
    const uint32_t c[4] = {v.x, v.y, v.z, v.w};
    const int j = last_nonzero(c, 16);
    const int64_t t = ((int64_t)(off + (uint32_t)j) << 8) | get_byte(c, j);
    nz = t > nz ? t : nz;
  }
  if (uni(__builtin_amdgcn_ballot_w64(act && i0 + 32u <= nb + 1u) != 0)) {  // rare: a tail of > 32 items
    const Rec u = load_rec<OPEN>(A, r, act);
    if (act) {
#pragma unroll 1
      for (uint32_t i = i0 + 32u; i <= nb + 1u; i += 32u) {
        uint32_t B[4];
        const int64_t t = tail_block<NR, OPEN>(u, i, B);
        nz = t > nz ? t : nz;
        ghash_mul_tab(y, wb);
        y[0] ^= B[0]; y[1] ^= B[1]; y[2] ^= B[2]; y[3] ^= B[3];
      }
    }
  }
  wave_lds_sync();  // the GHASH table is dead: its 8 KiB hold the lanes' combine tables
  BS_STAMP(t_tail);
  uint32_t z[4] = {0, 0, 0, 0};
  {
    const uint32_t i_last = (uint32_t)l + 32u * ((nb + 1u - (uint32_t)l) / 32u);
    const uint32_t e = act ? nb + 2u - i_last : 1u;  // 1..32
    const uint32_t yb[4] = {bswap32(y[0]), bswap32(y[1]), bswap32(y[2]), bswap32(y[3])};
    uint32_t hp[4];
#pragma unroll
    for (int w = 0; w < 4; w++) hp[w] = reinterpret_cast<const KeySched*>(rkp - offsetof(KeySched, rk) / 4)->hpow_be[e - 1][w];
    gf_mul_shoup(yb, hp, wb + 256u * (uint32_t)l, l, z);
  }
#pragma unroll
  for (int off = 16; off >= 1; off >>= 1) {
#pragma unroll
    for (int w = 0; w < 4; w++) z[w] ^= __shfl_xor(z[w], off, 64);
  }
  if (OPEN) {
#pragma unroll
    for (int off = 16; off >= 1; off >>= 1) {
      const int64_t o = __shfl_xor(nz, off, 64);
      nz = o > nz ? o : nz;
    }
  }
  if (act && l == 0) {
    const v4u32 ev = lds_u4(eaddr);
    const uint32_t t0 = ev.x ^ bswap32(z[0]), t1 = ev.y ^ bswap32(z[1]), t2 = ev.z ^ bswap32(z[2]),
                   t3 = ev.w ^ bswap32(z[3]);
    if (!OPEN) {
      const v4u32 tv = {t0, t1, t2, t3};
      st16(A.tags_out + 16ull * r, tv);
    } else {
      const uint32_t* tg = reinterpret_cast<const uint32_t*>(A.tags_in + 16ull * r);
      const bool ok = (tg[0] == t0) & (tg[1] == t1) & (tg[2] == t2) & (tg[3] == t3);
      write_open_result(A, r, tls != 0, len, ok, nz);
    }
  }
#ifdef ATLS_BS_STAMPS
  const uint64_t t_end = __builtin_amdgcn_s_memtime();
  if (lane == 0) {
    atomicAdd(&g_bs_stamps[0], (unsigned long long)(t_setup - t_start));
    atomicAdd(&g_bs_stamps[1], (unsigned long long)t_rounds);
    atomicAdd(&g_bs_stamps[2], (unsigned long long)t_data);
    atomicAdd(&g_bs_stamps[3], (unsigned long long)(t_tail - t_setup - t_rounds - t_data));
    atomicAdd(&g_bs_stamps[4], (unsigned long long)(t_end - t_tail));
    atomicAdd(&g_bs_stamps[5], 1ull);
  }
#endif
}

// One launch per AES round count (10/12/14) present in the key table: each pair runs one.
template <bool OPEN, int NR>
__global__ __launch_bounds__(64 * kWaves, 2) void gcm_bs_kernel(GcmArgs A) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) smem[i] = A.t0[i];
  __syncthreads();
  const int wave = (int)uni(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int h = lane >> 5, l = lane & 31;
  const uint32_t wb = kT0Bytes + (uint32_t)(2 * wave + h) * kTabBytes;
  const uint32_t eaddr = kEOff + 16u * (uint32_t)(2 * wave + h);
  const uint32_t slot = kSlotOff + 32u * (uint32_t)(64 * wave + lane);
  const uint32_t npairs = (A.n + 1u) / 2u;
  for (uint32_t q = blockIdx.x * kWaves + wave; q < npairs; q += gridDim.x * kWaves) {
    const uint32_t rA = 2u * q;
    const uint32_t cA = uni(bs_taken<OPEN>(A, rA));
    const uint32_t cB = rA + 1u < A.n ? uni(bs_taken<OPEN>(A, rA + 1u)) : 0u;
    if ((cA ? cA : cB) != (uint32_t)NR) continue;
    bs_pair<NR, OPEN>(A, rA + (uint32_t)h, h ? cB != 0 : cA != 0, wb, eaddr, slot, l, lane);
    wave_lds_sync();  // this pair's table reads are done before the next pair rebuilds them
  }
}

}  // namespace bsk
}  // namespace atls

// Debug: copy out (and reset) the phase timers of a -DATLS_BS_STAMPS build; -1 otherwise.
extern "C" int atls_debug_bs_stamps(unsigned long long* out8) {
#ifdef ATLS_BS_STAMPS
  if (hipMemcpyFromSymbol(out8, HIP_SYMBOL(atls::bsk::g_bs_stamps), 64) != hipSuccess) return -1;
  unsigned long long z[8] = {0};
  return hipMemcpyToSymbol(HIP_SYMBOL(atls::bsk::g_bs_stamps), z, 64) == hipSuccess ? 0 : -1;
#else
  (void)out8;
  return -1;
#endif
}

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
