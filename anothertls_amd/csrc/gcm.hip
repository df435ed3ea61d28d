// AES-GCM seal/open for TLS records on gfx950 -- the hot path of BASELINE.json's north star.
//
// Restates crypto/aes/gcm.rs:42-157 (Gcm::gcm, Cipher for Gcm) for a whole batch of
// records, with the record-layer framing of net/record.rs:162-240 done on the device
// (inner plaintext = content||type, 5-byte AAD header, nonce = static_iv ^ be64(seq)).
//
// Kernel gcm_kernel<OPEN, 12 waves, NR>: 12 waves per workgroup, one workgroup per CU (the LDS --
// 64 KiB of T-tables + 8 KiB of GHASH table per wave = 160 KiB -- is what limits residency). A
// record's GHASH input is AAD blocks, ciphertext blocks, length block; its "slots" are s = 0..m,
// slot 0 = E_K(J0) (gcm.rs:76), slot s >= 1 = GHASH block s-1. Two ways to walk them:
//   * gcm_record: one record per wave, lane l owns slots s = l (mod 64): each 64-slot step moves
//     one contiguous 1 KiB run of the record (16 B per lane, coalesced). Per record: a GHASH table
//     of H^64 built in LDS, the counter cache, the lane combine.
//   * gcm_group (direct batches, key-grouped by plan.hip atls_launch_group): a run of 8 records of
//     one key slot and one step count per wave, G lanes per record (G = 8 for AES-128, 16 for
//     AES-192/256): lane gl of group g owns slots s = gl (mod G) of record g. One H^G table, one
//     counter cache and one lane combine serve 64 / G records. Runs come from a work counter.
// Per block:
//   * AES-CTR: T-table rounds with two tables (T0, T1 = rotl8 T0) replicated 32x in LDS so lane l
//     reads bank l & 31: conflict-free ds_read_b32. Counter-mode caching (Bernstein-Schwabe): a
//     step's counters differ in byte 15 only, so rounds 1-2 take 5 lookups (133 per AES-128 block).
//   * GHASH: lane-strided Horner Y <- Y * H^k ^ B (k = 64 or G) with a 4-bit table in LDS, 32
//     positions x 16 entries x 16 B; a position is exactly one 256-B bank row, so the 32
//     ds_read_b128 lookups never bank-conflict.
//   * Lane combine: Z = sum_l Y_l * H^(e_l), e_l the powers each lane's last block still needs, by
//     a transposed comb multiply, then a DPP + readlane XOR reduction; tag = E_K(J0) ^ Z.
// Bytes per record (roofline): read L, write L + 16 (tag) -- see DESIGN.md §4. The LDS array is
// the binding unit (394 array cycles per 64 blocks, ~75 % busy).
#include <cstdlib>

#include "gcm_common.h"
#include "chacha_q4.h"

namespace atls {

#ifndef ATLS_DBG_SKIP
#define ATLS_DBG_SKIP 0  // timing experiments only (wrong results): 1 lane combine, 2 general steps, 4 GHASH
                         // table, 8 GHASH multiply in general steps, 16 last step, 32 first step,
                         // 64 the last AES round's lookups
#endif
#ifndef ATLS_GEN_VEC
#define ATLS_GEN_VEC 0  // general steps: whole blocks of unaligned records by 16-byte accesses too (ld16 / st16).
                        // C5's general steps cost 12 % of its kernel interval (timing build ATLS_DBG_SKIP=2,
                        // profiles/r03/ab_c5_gcm_parts.log), but not through their byte accesses: C5 0.322 vs
                        // 0.323 ms, C2 unchanged (ab_gcm_general_vec.log, parity per variant); off
#endif
#ifndef ATLS_CTR_CACHE
#define ATLS_CTR_CACHE 1
#endif
#ifndef ATLS_GEN_MASK
#define ATLS_GEN_MASK 1  // a general step runs its AES rounds and GHASH product only on the lanes whose slot lies in the
                         // record (EXEC-masked LDS lookups; a C2 record's last step has 4 such lanes of 64). Same-box
                         // A/B, 3 rounds, parity first (profiles/r05/ab_genmask*.log): C5 seal 0.3175-0.321 -> 0.3148-
                         // 0.319 ms, open -1 %; C4 -0.3 %; C2 with a key per record unchanged (1.311-1.317 ms) at a
                         // 2 % higher clock. 0 = every lane
#endif

#ifndef ATLS_GCM_FAST_FIRST
#define ATLS_GCM_FAST_FIRST 0  // 1: a TLS record's first step (E_K(J0), AAD, 62 data blocks) without the general step's
                               // classification, when it holds 62 whole blocks (round 4 A/B on C5)
#endif
#ifndef ATLS_GCM_SPREAD
#define ATLS_GCM_SPREAD 1  // planned batches: work-list rows spread over the workgroups, odd rows reversed (gcm_kernel)
#endif
#ifndef ATLS_SINGLE_FAST_FIRST
#define ATLS_SINGLE_FAST_FIRST 1  // the same in the single-call kernel (gcm_single: one wave's latency, no occupancy)
#endif
#ifndef ATLS_PREFETCH
#define ATLS_PREFETCH 1  // fast steps load the next step's data block before their own AES rounds
#endif

#ifndef ATLS_GCM_DOUBLE
#define ATLS_GCM_DOUBLE 12  // lane groups of keys with >= this many rounds: two fast steps per pass, their
                            // AES rounds software-pipelined (aes_rounds_tt2). Same-box A/B
                            // (profiles/r02/ab_double.log): C4 780 -> 795 GiB/s, C2 883 -> 862 (so AES-128
                            // keeps single steps); 99 = off
#endif

#ifndef ATLS_DBG_SHARED_GHASH
#define ATLS_DBG_SHARED_GHASH 0  // timing experiment only (wrong tags): one GHASH table per workgroup,
                                 // 16 waves per CU, to price the residency a per-key table would buy
#endif
// LDS: AES tables first, row x = 256 B = {T0[x] x32 banks | T1[x] x32 banks} (64 KiB), then one
// 8 KiB GHASH table per wave.
// Lane l reads bank (l & 31): conflict-free ds_read_b32.
constexpr int kTabBytes = 65536;
constexpr int kGhashBytes = 8192;
constexpr size_t lds_bytes(int waves) { return kTabBytes + (size_t)(ATLS_DBG_SHARED_GHASH ? 1 : waves) * kGhashBytes; }

// The lane combine's product Y_l * H^e_l of gcm_record (gcm_common.h): through the wave's GHASH table
// region, except in the shared-table timing build where other waves still read it.
// AES-256 batches keep the register comb: the LDS form measured 1.3 % slower on C4 (its records mostly take
// the lane-group kernel, whose code the change still reaches); the single call (LAT) takes the LDS form.
#ifndef ATLS_COMB_AES256
#define ATLS_COMB_AES256 0
#endif
template <int NR, bool LAT>
__device__ __forceinline__ void lane_comb(const uint32_t (&yb)[4], const uint32_t (&hp)[4], uint32_t (&z)[4],
                                          uint32_t wb, int lane) {
  if (ATLS_COMB_LDS && !ATLS_DBG_SHARED_GHASH && (LAT || NR != 14 || ATLS_COMB_AES256)) gf_mul_comb_lds<ATLS_COMB_LDS == 2 ? 2 : 1>(yb, hp, z, wb, lane);
  else gf_mul_comb(yb, hp, z);
}

// The GHASH product of every record kernel: the compiler's schedule of the 32 lookups. The former ATLS_GHASH_W
// switch (ghash_mul_tab_wide, W lookups per LDS round trip) was removed in round 6: re-tried at W = 16 it gave wrong
// tags on some records of the mixed parity batch (tests/test_gpu_parity.py), and no round measured it faster.
__device__ __forceinline__ void ghash_mul(uint32_t (&y)[4], uint32_t wb) { ghash_mul_tab(y, wb); }

// Round-key words from the key schedule: a wave-uniform address, so one s_load_dwordx4.
__device__ __forceinline__ v4u32 kload4(const uint32_t* p) {
  return *(const __attribute__((address_space(4))) v4u32*)(p);
}

// ---- AES (two-table T-table rounds on raw-word state) -------------------------------------
// T0[x] = {2S,S,S,3S} (LE), T1 = rotl8(T0). With T2 = rotl16(T0), T3 = rotl16(T1):
//   col_c = T0[s_c.b0] ^ T1[s_{c+1}.b1] ^ rotl16(T0[s_{c+2}.b2] ^ T1[s_{c+3}.b3] ^ rotl16(rk_c)).
// Table address of byte k of state word w for this lane's bank: (byte << 8) | lb, one v_perm_b32
// (selector byte 0 <- lb, byte 1 <- w.byte_k, bytes 2-3 <- 0); lb = 4*(lane & 31); T1 at +128.
#define TA(w, sh) perm((w), lb, 0x0c0c0000u | ((4u + (sh) / 8u) << 8))

// One middle round; kr = rotl16 of the round key words. The compiler's own interleaving of
// lookups and XORs measured faster than issuing all 16 lookups first (tools/ubench/step_ubench).
__device__ __forceinline__ void tt_round(uint32_t (&s)[4], const uint32_t* kr, uint32_t lb) {
  const uint32_t s0 = s[0], s1 = s[1], s2 = s[2], s3 = s[3];
#pragma unroll
  for (int c = 0; c < 4; c++) {
    const uint32_t a = (c == 0 ? s0 : c == 1 ? s1 : c == 2 ? s2 : s3);
    const uint32_t bb = (c == 0 ? s1 : c == 1 ? s2 : c == 2 ? s3 : s0);
    const uint32_t cc = (c == 0 ? s2 : c == 1 ? s3 : c == 2 ? s0 : s1);
    const uint32_t dd = (c == 0 ? s3 : c == 1 ? s0 : c == 2 ? s1 : s2);
    const uint32_t u = xor3(lds_u32(TA(cc, 16)), lds_u32(TA(dd, 24) + 128), kr[c]);
    s[c] = xor3(lds_u32(TA(a, 0)), lds_u32(TA(bb, 8) + 128), rot16(u));
  }
}

// Final round (SubBytes, ShiftRows, AddRoundKey): S[x] = byte 1 of T0[x] = byte 2, 3 of T1[x].
__device__ __forceinline__ void tt_final(uint32_t (&s)[4], const uint32_t* kf, uint32_t lb) {
  const uint32_t s0 = s[0], s1 = s[1], s2 = s[2], s3 = s[3];
#pragma unroll
  for (int c = 0; c < 4; c++) {
    const uint32_t a = (c == 0 ? s0 : c == 1 ? s1 : c == 2 ? s2 : s3);
    const uint32_t bb = (c == 0 ? s1 : c == 1 ? s2 : c == 2 ? s3 : s0);
    const uint32_t cc = (c == 0 ? s2 : c == 1 ? s3 : c == 2 ? s0 : s1);
    const uint32_t dd = (c == 0 ? s3 : c == 1 ? s0 : c == 2 ? s1 : s2);
    // {T0[a].b1, T0[b].b1} | {T1[c].b2, T1[d].b3}, then ^ rk: two v_perm + one v_bitop3 ((x|y)^z)
    const uint32_t lo = perm(lds_u32(TA(bb, 8)), lds_u32(TA(a, 0)), 0x0c0c0501u);
    const uint32_t hi = perm(lds_u32(TA(dd, 24) + 128), lds_u32(TA(cc, 16) + 128), 0x07020c0cu);
    s[c] = __builtin_amdgcn_bitop3_b32(lo, hi, kf[c], 0x56);
  }
}

// Rounds R0 .. NR on a state that went through rounds 0 .. R0-1. rk / rkr: the record's round
// keys and their rotl16, held in (wave-uniform) registers for the whole record -- measured
// faster than a rolled round loop with a scalar load per round.
template <int NR, int R0>
__device__ __forceinline__ void aes_rounds_tt(uint32_t (&s)[4], const uint32_t* rk, const uint32_t* rkr,
                                              uint32_t lb) {
#pragma unroll
  for (int r = R0; r < NR; r++) tt_round(s, rkr + 4 * r, lb);
  if (ATLS_DBG_SKIP & 64) {
#pragma unroll
    for (int c = 0; c < 4; c++) s[c] ^= rk[4 * NR + c];
  } else {
    tt_final(s, rk + 4 * NR, lb);
  }
}

// A prefetch address: the block at `want` if it lies within the first `lim` bytes, else this
// step's own block `cur` (loaded again, unused). The load is issued by every lane either way: a
// lane-predicated load would make the compiler's counter wait for the prefetches of this step
// too (s_waitcnt vmcnt(0)) before it may use the blocks prefetched for it.
__device__ __forceinline__ uint32_t pf_off(uint32_t want, uint32_t cur, uint32_t lim) {
  return want + 16u <= lim ? want : cur;
}

// Two independent blocks through rounds R0 .. NR as a two-stage software pipeline: a round's 16
// lookups of one block are issued, then the other block's XORs of its previous round (and its
// next lookups) run while they are in flight. sched_barrier keeps the stages in this order, so a
// wave keeps 16 lookups in flight while it computes (one block per lane leaves it none).
// Lookups of one round of one block, as tt_round (FIN: as tt_final, T0 for a / bb, T1 for cc / dd).
__device__ __forceinline__ void tt_look(const uint32_t (&s)[4], uint32_t lb, bool fin, uint32_t (&L)[16]) {
  const uint32_t s0 = s[0], s1 = s[1], s2 = s[2], s3 = s[3];
#pragma unroll
  for (int c = 0; c < 4; c++) {
    const uint32_t a = (c == 0 ? s0 : c == 1 ? s1 : c == 2 ? s2 : s3);
    const uint32_t bb = (c == 0 ? s1 : c == 1 ? s2 : c == 2 ? s3 : s0);
    const uint32_t cc = (c == 0 ? s2 : c == 1 ? s3 : c == 2 ? s0 : s1);
    const uint32_t dd = (c == 0 ? s3 : c == 1 ? s0 : c == 2 ? s1 : s2);
    L[4 * c] = lds_u32(TA(cc, 16) + (fin ? 128u : 0u));
    L[4 * c + 1] = lds_u32(TA(dd, 24) + 128);
    L[4 * c + 2] = lds_u32(TA(a, 0));
    L[4 * c + 3] = lds_u32(TA(bb, 8) + (fin ? 0u : 128u));
  }
}
__device__ __forceinline__ void tt_comb(uint32_t (&s)[4], const uint32_t (&L)[16], const uint32_t* kr) {
#pragma unroll
  for (int c = 0; c < 4; c++) s[c] = xor3(L[4 * c + 2], L[4 * c + 3], rot16(xor3(L[4 * c], L[4 * c + 1], kr[c])));
}
__device__ __forceinline__ void tt_comb_final(uint32_t (&s)[4], const uint32_t (&L)[16], const uint32_t* kf) {
#pragma unroll
  for (int c = 0; c < 4; c++) {
    const uint32_t lo = perm(L[4 * c + 3], L[4 * c + 2], 0x0c0c0501u);
    const uint32_t hi = perm(L[4 * c + 1], L[4 * c], 0x07020c0cu);
    s[c] = __builtin_amdgcn_bitop3_b32(lo, hi, kf[c], 0x56);
  }
}
template <int NR, int R0>
__device__ __forceinline__ void aes_rounds_tt2(uint32_t (&a)[4], uint32_t (&b)[4], const uint32_t* rk, const uint32_t* rkr,
                                               uint32_t lb) {
  uint32_t La[16], Lb[16];
  tt_look(a, lb, R0 == NR, La);
  __builtin_amdgcn_sched_barrier(0);
  tt_look(b, lb, R0 == NR, Lb);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int r = R0; r < NR; r++) {
    tt_comb(a, La, rkr + 4 * r);
    tt_look(a, lb, r + 1 == NR, La);
    __builtin_amdgcn_sched_barrier(0);
    tt_comb(b, Lb, rkr + 4 * r);
    tt_look(b, lb, r + 1 == NR, Lb);
    __builtin_amdgcn_sched_barrier(0);
  }
  tt_comb_final(a, La, rk + 4 * NR);
  tt_comb_final(b, Lb, rk + 4 * NR);
}

#ifndef ATLS_TT_ISSUE_ALL
#define ATLS_TT_ISSUE_ALL 1  // lane-group fast steps issue a round's 16 lookups before any of its XORs: C2 -0.4 to
                             // -0.7 %, C4 -0.5 %, C5 -0.8 % kernel time over two same-box A/Bs of 3 rounds each
                             // (profiles/r02/ab_issue16*.log); the same for one-record-per-wave steps and with
                             // the GHASH lookups spread over the rounds measured no better
#endif
// Rounds R0 .. NR of one block, each round's 16 lookups issued before its XORs (tt_look / tt_comb).
template <int NR, int R0>
__device__ __forceinline__ void aes_rounds_tt1(uint32_t (&a)[4], const uint32_t* rk, const uint32_t* rkr, uint32_t lb) {
  uint32_t L[16];
#pragma unroll
  for (int r = R0; r < NR; r++) {
    tt_look(a, lb, false, L);
    __builtin_amdgcn_sched_barrier(0);
    tt_comb(a, L, rkr + 4 * r);
    __builtin_amdgcn_sched_barrier(0);
  }
  tt_look(a, lb, true, L);
  __builtin_amdgcn_sched_barrier(0);
  tt_comb_final(a, L, rk + 4 * NR);
}

template <int NR>
__device__ __forceinline__ void aes_encrypt_tt(uint32_t (&s)[4], const uint32_t* rk, const uint32_t* rkr,
                                               uint32_t lb) {
#pragma unroll
  for (int i = 0; i < 4; i++) s[i] ^= rk[i];
  aes_rounds_tt<NR, 1>(s, rk, rkr, lb);
}

// ---- counter-mode caching (Bernstein & Schwabe, "New AES software speed records", 2008) ----
// In one 64-slot step the counters are ctr = 256*hi + lo with hi wave-uniform, so the 64 counter
// blocks differ only in byte 15. Round 1 then has ONE lane-varying lookup (byte 15 -> T3 into
// column 0) and round 2 FOUR (column 0 of the round-1 state feeds one byte of each column); the
// other 27 lookups and round-key XORs fold into five words that depend on (record, hi) only:
//   c0   = T3[lo ^ rk0.b15] ^ U0            (round-1 column 0; columns 1-3 are V1..V3)
//   out0 = T0[c0.b0] ^ K0,  K0 = T1[V1.b1] ^ T2[V2.b2] ^ T3[V3.b3] ^ rk2_0
//   out1 = T3[c0.b3] ^ K1,  K1 = T0[V1.b0] ^ T1[V2.b1] ^ T2[V3.b2] ^ rk2_1
//   out2 = T2[c0.b2] ^ K2,  K2 = T0[V2.b0] ^ T1[V3.b1] ^ T3[V1.b3] ^ rk2_2
//   out3 = T1[c0.b1] ^ K3,  K3 = T0[V3.b0] ^ T2[V1.b2] ^ T3[V2.b3] ^ rk2_3
// AES-128 does 133 lookups per block instead of 160. Lane j of the wave holds the five words for
// hi = hi0 + j (built once per record); a step reads its hi's words with v_readlane.
struct CtrCache {
  uint32_t u0r, k0, k1r, k2r, k3;  // u0r = rot16(U0), k1r = rot16(K1), k2r = rot16(K2)
};

// nraw: nonce bytes 0..11 as raw words; hi: this lane's counter high part (ctr >> 8).
__device__ __forceinline__ CtrCache ctr_cache_build(const uint32_t (&nraw)[3], uint32_t hi, const uint32_t* rk,
                                                    const uint32_t* rkr, uint32_t lb) {
  const uint32_t s0 = nraw[0] ^ rk[0], s1 = nraw[1] ^ rk[1], s2 = nraw[2] ^ rk[2];
  const uint32_t s3 = bswap32(hi << 8) ^ rk[3];  // lo = 0: byte 15 never enters U0 / V1..V3
  const uint32_t u0 = xor3(lds_u32(TA(s0, 0)), lds_u32(TA(s1, 8) + 128), rot16(lds_u32(TA(s2, 16)) ^ rkr[4]));
  const uint32_t* kr1 = rkr + 4;
  uint32_t v[4];
#pragma unroll
  for (int c = 1; c < 4; c++) {
    const uint32_t a = (c == 1 ? s1 : c == 2 ? s2 : s3), bb = (c == 1 ? s2 : c == 2 ? s3 : s0);
    const uint32_t cc = (c == 1 ? s3 : c == 2 ? s0 : s1), dd = (c == 1 ? s0 : c == 2 ? s1 : s2);
    const uint32_t u = xor3(lds_u32(TA(cc, 16)), lds_u32(TA(dd, 24) + 128), kr1[c]);
    v[c] = xor3(lds_u32(TA(a, 0)), lds_u32(TA(bb, 8) + 128), rot16(u));
  }
  CtrCache C;
  C.u0r = rot16(u0);
  // T2[x] = rot16(T0[x]), T3[x] = rot16(T1[x])
  C.k0 = xor3(lds_u32(TA(v[1], 8) + 128), rot16(lds_u32(TA(v[2], 16)) ^ lds_u32(TA(v[3], 24) + 128)), rk[8]);
  C.k1r = rot16(xor3(lds_u32(TA(v[1], 0)), lds_u32(TA(v[2], 8) + 128), rot16(lds_u32(TA(v[3], 16))) ^ rk[9]));
  C.k2r = rot16(xor3(lds_u32(TA(v[2], 0)), lds_u32(TA(v[3], 8) + 128), rot16(lds_u32(TA(v[1], 24) + 128)) ^ rk[10]));
  C.k3 = xor3(lds_u32(TA(v[3], 0)), rot16(lds_u32(TA(v[1], 16)) ^ lds_u32(TA(v[2], 24) + 128)), rk[11]);
  return C;
}

// Rounds 1 and 2 of one lane's counter block from the cache; addr1 = T0 address of
// lo ^ rk0.b15 for this lane's bank. Leaves the state after round 2.
__device__ __forceinline__ void aes_ctr_r12(uint32_t (&s)[4], uint32_t addr1, const CtrCache& C, uint32_t lb) {
  const uint32_t c0r = lds_u32(addr1 + 128) ^ C.u0r;  // rot16 of round-1 column 0
  // bytes of c0 = rot16(c0r): c0.b0 = c0r.b2, c0.b1 = c0r.b3, c0.b2 = c0r.b0, c0.b3 = c0r.b1
  s[0] = lds_u32(TA(c0r, 16)) ^ C.k0;
  s[1] = rot16(lds_u32(TA(c0r, 8) + 128) ^ C.k1r);
  s[2] = rot16(lds_u32(TA(c0r, 0)) ^ C.k2r);
  s[3] = lds_u32(TA(c0r, 24) + 128) ^ C.k3;
}
#undef TA

// Phase timing (build with -DATLS_TT_STAMPS): shader-clock totals over all records, read back with
// atls_debug_tt_stamps(). 0 setup (tables, counter cache), 1 fast steps, 2 general steps,
// 3 lane combine + tag, 4 records, 5 fast steps, 6 general steps; general steps split: 8 the first step's
// cycles, 9 the later ones', 10 until their data loads landed, 11 their AES, 12 first steps counted.
#ifdef ATLS_TT_STAMPS
__device__ unsigned long long g_tt_stamps[16];
#define TT_STAMP(var) const uint64_t var = __builtin_amdgcn_s_memtime()
#else
#define TT_STAMP(var)
#endif

// The last (general) step of a record without loads of its own (ATLS_GEN_PN, round 4 A/B, off): a wave's
// vector-memory counter counts its stores too and drains in order, so a load issued after the fast steps'
// stores waits for all of them (tools/tt_stamps.py: a C5 record's last step took 13x a fast step's wave
// time). The fast step before it already loads the general step's whole blocks (Pn); with the switch the
// lane whose block is partial loads the input's last 16 bytes instead of a dummy and the general step
// takes both from Pn. The step's wave time falls 2.8x (C5) but the launch does not get shorter (the other
// waves were covering the wait) and the open kernel gets 8 % slower (registers): DESIGN §4.2.
#ifndef ATLS_GEN_PN
#define ATLS_GEN_PN 0
#endif

// Deferred last steps (round 6). A one-record-per-wave record of S slots runs ceil(S / 64) wave
// steps; its last step holds rem = S - 64 floor((S - 1) / 64) slots, yet costs a whole step's LDS lookups and VALU
// issue (a C2 record: 1,028 slots, the 17th step 4 lanes of 64 -- 5.5 % of C2 with a key per record,
// profiles/r05/ab_keyrec_parts.log; the LDS array serves a lane group whether 4 or 32 of its lanes are enabled).
// With ATLS_GCM_TAIL = T > 0, a batch launch's record whose last step has rem <= T slots stops after its full
// steps: the lane combine runs for the first S - rem slots (Z' = the GHASH state after them), and lane 0 leaves
// Z', E_K(J0) and (opens) the content-type scan in the launch's tail workspace. gcm_tail_kernel then finishes
// those records one per lane: the rem slots' counter blocks by T-table AES with the lane's own round keys,
// their ciphertext, Z' <- (Z' ^ B) * H over the rem GHASH blocks (comb multiply, per-lane H), the tag or the
// open's verdict. Records that go through lane groups, the single call, WIRE records and non-96-bit IVs keep
// their last step.
// Measured and left off (profiles/r06/tail/: parity green, 60 tests; same box, 3 interleaved rounds, engine switch
// ATLS_GCM_TAIL_ON): C2 with a key per record 1.293-1.299 ms deferred vs 1.252-1.259 not, C2 1.050-1.060 vs
// 1.025-1.037, C4 shard 2.621-2.635 vs 2.569-2.612, C5 whole within noise. rocprof (keyrec): the record kernel
// 1.2218 vs 1.2486 ms (-27 us, 2.2 %: the kernel is not bound by the steps it no longer runs) and the tail kernel
// 74 us for 65,536 records (key-schedule gathers from HBM, one AES block and one comb product per lane). Even a free
// tail kernel would buy 2 %; 0 compiles every piece of it out.
#ifndef ATLS_GCM_TAIL
#define ATLS_GCM_TAIL 0
#endif
struct TailState {  // one deferred record (48 B): Z' (be words), E_K(J0) (raw words), open scan, record index
  uint32_t z[4];
  uint32_t e[4];
  int64_t lastnz;
  uint32_t rec;
  uint32_t pad;
};
// Tail workspace: [0] deferred count, [1] tail workgroups done, [2..3] pad, then TailState[n] from byte 16.
constexpr size_t kTailHdr = 16;

// LAT: the single-call kernel's record (one wave's latency, no occupancy to keep): the branch-free first
// step (ATLS_SINGLE_FAST_FIRST) and the LDS lane combine at every key size.
// LN: the threads that share the record -- 64 (one wave: the batch kernels), or 256 (the single-call
// kernel's four waves: slot s goes to thread s mod 256, so a 1.5 KiB record is one step and a 16 KiB one
// five instead of seventeen). With LN = 256, wb is the base of eight 8 KiB LDS areas: the 4-bit tables of
// H^64, H^128, H^192 (lane-combine multipliers past H^64) and H^256 (the Horner factor), one per-lane comb
// area per wave, then 256 B where the waves exchange their partial tags and content-type scans.
template <int NR, bool OPEN, bool LAT = false, int LN = 64>
__device__ void gcm_record(const GcmArgs& A, const atls_rec& d, const KeySched* k, uint32_t rec_idx,
                           uint32_t lb, uint32_t wb, int lane) {
  TT_STAMP(t_start);
#ifdef ATLS_TT_STAMPS
  uint64_t t_fast = 0, t_gen = 0, n_fast = 0, n_gen = 0, t_gen0 = 0, t_genl = 0, t_ld = 0, t_aes = 0, n_gen0 = 0;
#endif
  uint32_t rk[4 * (NR + 1)], rkr[4 * (NR + 1)];
#pragma unroll
  for (int i = 0; i < 4 * (NR + 1); i++) {
    rk[i] = cptr(k->rk)[i];  // wave-uniform: scalar loads
    rkr[i] = cptr(k->rkr)[i];
  }
  // TLS and WIRE: nonce from (static IV, seq), one AAD block; WIRE also frames the record
  const bool wire = d.mode == ATLS_MODE_WIRE;
  const bool tls = d.mode != ATLS_MODE_RAW;
  const uint32_t len = d.len;
  const uint32_t n_aead = (tls && !OPEN) ? len + 1 : len;  // record.rs:172-173 inner plaintext
  const uint8_t* rec_in = A.in + d.in_off;
  const uint8_t* src = rec_in + ((OPEN && wire) ? 5u : 0u);
  uint8_t* dst = A.out + d.out_off + ((!OPEN && wire) ? 5u : 0u);
  // Unaligned records (wire framing) keep the vector fast steps (ld16/st16); the few general
  // steps go bytewise for them (vector accesses there cost registers the seal kernel lacks).
  const bool src_al = ((reinterpret_cast<uintptr_t>(src)) & 15u) == 0;
  const bool dst_al = ((reinterpret_cast<uintptr_t>(dst)) & 15u) == 0;
  // ---- nonce / J0 (gcm.rs:59-74) and AAD ----
  uint32_t j0[4];  // be words
  bool is96 = true;
  uint32_t hdr0 = 0, hdr1 = 0;  // TLS AAD header, raw words
  const uint8_t* aadp = nullptr;
  uint32_t aad_len = 5;
  bool hdr_ok = true;
  if (tls) {
    // key_schedule.rs:51-64: nonce = iv ^ (0^4 || be64(seq)); J0 = nonce || 0x00000001.
    const uint64_t seq = d.seq;
    j0[0] = bswap32(k->siv[0]);
    j0[1] = bswap32(k->siv[1]) ^ (uint32_t)(seq >> 32);
    j0[2] = bswap32(k->siv[2]) ^ (uint32_t)seq;
    j0[3] = 1u;
    if (OPEN && wire) {  // the received header is the AAD (record.rs:219)
      hdr_ok = wire_header(rec_in, len, hdr0, hdr1);
    } else {
      const uint32_t L = n_aead + 16;  // record.rs:176-183, truncated to 16 bits
      hdr0 = 0x17u | (0x03u << 8) | (0x03u << 16) | (((L >> 8) & 0xffu) << 24);
      hdr1 = L & 0xffu;
    }
  } else {
    const uint8_t* iv = A.aux + d.aux_off;
    const uint32_t iv_len = d.iv_len;
    aadp = iv + iv_len;
    aad_len = d.aad_len;
    if (iv_len == 12) {
      j0[0] = ((uint32_t)iv[0] << 24) | ((uint32_t)iv[1] << 16) | ((uint32_t)iv[2] << 8) | iv[3];
      j0[1] = ((uint32_t)iv[4] << 24) | ((uint32_t)iv[5] << 16) | ((uint32_t)iv[6] << 8) | iv[7];
      j0[2] = ((uint32_t)iv[8] << 24) | ((uint32_t)iv[9] << 16) | ((uint32_t)iv[10] << 8) | iv[11];
      j0[3] = 1u;
    } else {
      // J0 = GHASH_H(IV || 0-pad || [len(IV)]_64), gcm.rs:59-70. Rare (RAW mode only): every
      // lane computes it redundantly with the bit-serial multiply.
      is96 = false;
      uint32_t N[4] = {0, 0, 0, 0};
      for (uint32_t i = 0; i < iv_len; i += 16) {
        uint32_t blk[4] = {0, 0, 0, 0};
#pragma unroll
        for (int q = 0; q < 16; q++)
          if (i + q < iv_len) blk[q >> 2] |= (uint32_t)iv[i + q] << (24 - 8 * (q & 3));
        for (int w = 0; w < 4; w++) blk[w] ^= N[w];
        gf_mul_be(blk, k->h_be, N);
      }
      N[3] ^= iv_len * 8u;
      uint32_t t[4] = {N[0], N[1], N[2], N[3]};
      gf_mul_be(t, k->h_be, j0);
    }
  }

  const uint32_t na = tls ? 1u : (aad_len + 15u) / 16u;
  const uint32_t nb = (n_aead + 15u) / 16u;
  const uint32_t m = na + nb + 1u;  // GHASH blocks: AAD, data, length
  const uint32_t S = m + 1u;        // slots: E(J0) + GHASH blocks
  const uint32_t in_bytes = len;    // bytes readable from src
  // ATLS_GCM_TAIL: a sparse last step is left to gcm_tail_kernel; the steps and the lane combine run over the
  // first S_run slots (S_run = S otherwise)
  const uint32_t rem = S - (uint32_t)LN * ((S - 1u) / (uint32_t)LN);
  const bool defer = ATLS_GCM_TAIL > 0 && LN == 64 && !LAT && A.tail != nullptr && is96 && na == 1u && !wire &&
                     S > (uint32_t)LN && S <= 64u * 256u && rem <= (uint32_t)ATLS_GCM_TAIL;
  const uint32_t S_run = defer ? S - rem : S, m_run = S_run - 1u;

  // A record of one step (S <= 64: AEAD up to 976 B in TLS mode) multiplies nothing by H^64:
  // Y starts at 0 and the lane combine applies every power, so it skips the table.
  const bool one_step = S <= (uint32_t)LN;
  if constexpr (LN == 64) {
    if (!one_step) {
      uint32_t seed[4];
#pragma unroll
      for (int w = 0; w < 4; w++) seed[w] = k->p4_be[lane >> 1][w];
      if (!(ATLS_DBG_SKIP & 4)) ghash_table_entries<8>(wb, seed, lane >> 1, (lane & 1) * 8);
      wave_lds_sync();
    }
  } else {
    // wave b builds the table of H^(64 (b + 1)): H^64 = hpow[63], H^128 = (H^64)^2, H^192 = (H^48)^4,
    // H^256 = (H^64)^4 -- squarings only; lane l the entries 8 (l & 1) .. +7 of position l / 2
    // (only the tables this record uses: H^(64 (b+1)) when some lane's e - 1 reaches it, H^256 past one step)
    const uint32_t b = (uint32_t)lane >> 6;
    if (b < 3u ? S >= 64u * (b + 1u) + 2u : S > (uint32_t)LN) {
      const uint32_t p = ((uint32_t)lane >> 1) & 31u;
      uint32_t v[4];
#pragma unroll
      for (int w = 0; w < 4; w++) v[w] = k->hpow_be[b == 2u ? 47 : 63][w];
      if (b >= 1u) gf_square(v);
      if (b >= 2u) gf_square(v);
      gf_mulxk(v, 4u * p);
      ghash_table_entries<8>(wb + b * (uint32_t)kGhashBytes, v, (int)p, (lane & 1) * 8);
    }
    __syncthreads();
  }
  const uint32_t wh = LN == 64 ? wb : wb + 3u * (uint32_t)kGhashBytes;  // the Horner factor's table

  uint32_t y[4] = {0, 0, 0, 0};
  uint32_t e0 = 0, e1 = 0, e2 = 0, e3 = 0;  // E_K(J0), lane 0
  int64_t lastnz = -1;                      // OPEN+TLS: (pos << 8 | byte) of last non-zero pt byte
  // Slots [64, fast_end) are full 16-byte data blocks that lie wholly inside the input and
  // output: for them the step below runs branch-free (no classification, no partial handling).
  const uint32_t full_blocks = min(in_bytes, n_aead) / 16u;
  const uint32_t fast_end = is96 ? na + 1u + full_blocks : 0u;

  // Counter cache (CtrCache): every 64-slot step's counters share ctr >> 8 when the counter of slot
  // `base` is a multiple of 64 -- records with one AAD block (all TLS records) and a 96-bit IV.
  // Lane j holds the words of hi = j, enough for records below 2^14 blocks (256 KiB).
  const bool use_cache = ATLS_CTR_CACHE && is96 && na == 1u && S <= 64u * 256u;
  const uint32_t nraw[3] = {bswap32(j0[0]), bswap32(j0[1]), bswap32(j0[2])};
  const uint32_t lane_addr = ((uint32_t)lane << 8) | lb;  // T0 address of byte value `lane`
  const uint32_t k15 = rk[3] >> 24;                       // rk0 byte 15
  CtrCache cc{};
  if (use_cache) cc = ctr_cache_build(nraw, (uint32_t)lane & 63u, rk, rkr, lb);
  // AES of this lane's counter block via the cache; j = the step's (wave-uniform) ctr >> 8.
  auto aes_cached = [&](uint32_t (&st4)[4], uint32_t addr1, uint32_t j) {
    const CtrCache cj{(uint32_t)__builtin_amdgcn_readlane((int)cc.u0r, (int)j),
                      (uint32_t)__builtin_amdgcn_readlane((int)cc.k0, (int)j),
                      (uint32_t)__builtin_amdgcn_readlane((int)cc.k1r, (int)j),
                      (uint32_t)__builtin_amdgcn_readlane((int)cc.k2r, (int)j),
                      (uint32_t)__builtin_amdgcn_readlane((int)cc.k3, (int)j)};
    aes_ctr_r12(st4, addr1, cj, lb);
    aes_rounds_tt<NR, 3>(st4, rk, rkr, lb);
  };

  // Lane combine exponent (see below): s_last = the lane's last slot holding a GHASH block (slots
  // 1..m), -1 if none.
  int64_t s_last = -1;
  if (lane == 0) { if (m_run >= (uint32_t)LN) s_last = (int64_t)(m_run / LN) * LN; }
  else if ((uint32_t)lane <= m_run) s_last = (int64_t)lane + (int64_t)((m_run - (uint32_t)lane) / LN) * LN;
  const uint32_t e_comb = s_last >= 1 ? S_run - (uint32_t)s_last : 1u;  // 1..LN
  // the lane's combine multiplier H^e_comb, loaded now so its latency hides under the steps
  uint32_t hp[4];
#pragma unroll
  for (int w = 0; w < 4; w++) hp[w] = k->hpow_be[(e_comb - 1u) & 63u][w];
  if (LN > 64) {  // H^e = H^(e mod 64) * H^(64 kk) by the table of H^(64 kk)
    const uint32_t kk = (e_comb - 1u) >> 6;
    if (kk) {
      uint32_t r[4] = {bswap32(hp[0]), bswap32(hp[1]), bswap32(hp[2]), bswap32(hp[3])};
      ghash_mul_tab(r, wb + (kk - 1u) * (uint32_t)kGhashBytes);
#pragma unroll
      for (int w = 0; w < 4; w++) hp[w] = bswap32(r[w]);
    }
  }

  // Software pipelining (ATLS_PREFETCH): a fast step issues the load of the next step's block
  // (1 KiB further) before its own AES rounds, so the HBM latency hides under a whole step instead
  // of the last rounds; `pref` (wave-uniform) says Pn holds this step's block.
  uint4 Pn = make_uint4(0u, 0u, 0u, 0u);
  bool pref = false, gen_pn = false;
  const uint32_t lim = min(in_bytes, n_aead);
  const bool first_fast = (LAT ? ATLS_SINGLE_FAST_FIRST : ATLS_GCM_FAST_FIRST) && use_cache && !(OPEN && wire) && fast_end >= (uint32_t)LN;  // TLS / WIRE / RAW (one AAD block)
  TT_STAMP(t_setup);
  for (uint32_t base = 0; base < S_run; base += LN) {
    TT_STAMP(t_step);
    const uint32_t s = base + (uint32_t)lane;
    if (base >= (uint32_t)LN && base + LN <= fast_end) {  // wave-uniform
      const uint32_t off = (s - 1u - na) * 16u;
      const uint4 Pu = pref ? Pn : ld16(src + off);
      if (ATLS_PREFETCH) {  // every lane of a fast next step holds a whole block (fast_end)
        const uint32_t offn = off + 16u * LN;
        pref = base + 2u * LN <= fast_end;
        gen_pn = ATLS_GEN_PN && !pref;  // the next step is a general one: its blocks come from Pn too
        Pn = ld16(src + (offn + 16u <= lim ? offn : (ATLS_GEN_PN && offn < lim && lim >= 16u) ? lim - 16u : off));
      }
      const v4u32 P = {Pu.x, Pu.y, Pu.z, Pu.w};
      uint32_t st[4];
      if (use_cache) {
        const uint32_t c0 = j0[3] + base - na;  // counter of lane 0, a multiple of LN
        aes_cached(st, lane_addr ^ (((c0 & 0xffu) ^ k15) << 8), c0 >> 8);
      } else {
        st[0] = nraw[0]; st[1] = nraw[1]; st[2] = nraw[2];
        st[3] = bswap32(j0[3] + (s - na));
        aes_encrypt_tt<NR>(st, rk, rkr, lb);
      }
      const v4u32 C = {P.x ^ st[0], P.y ^ st[1], P.z ^ st[2], P.w ^ st[3]};
      st16(dst + off, make_uint4(C.x, C.y, C.z, C.w));
      if (OPEN && tls) lastnz = block_last_nz(C.x, C.y, C.z, C.w, off, lastnz);
      const v4u32 Bv = OPEN ? P : C;
      ghash_mul(y, wh);
      y[0] ^= Bv.x; y[1] ^= Bv.y; y[2] ^= Bv.z; y[3] ^= Bv.w;
#ifdef ATLS_TT_STAMPS
      t_fast += __builtin_amdgcn_s_memtime() - t_step;
      n_fast++;
#endif
      continue;
    }
    if ((LAT ? ATLS_SINGLE_FAST_FIRST : ATLS_GCM_FAST_FIRST) && base == 0u && first_fast) {
      // The first step without classification (round 4 A/B): lane 0 E_K(J0) (counter 1),
      // lane 1 the TLS AAD block, lanes 2..63 data blocks 0..61 (counters 2..63) -- whole blocks when
      // the record has at least 62 of them. Same counter cache as the fast steps (ctr >> 8 = 0).
      const uint32_t off = lane >= 2 ? ((uint32_t)lane - 2u) * 16u : 0u;
      const uint4 Pu = ld16(src + off);
      if (ATLS_PREFETCH) {  // the next step's block, as a fast step loads it
        const uint32_t offn = ((uint32_t)lane + LN - 2u) * 16u;
        pref = 2u * LN <= fast_end;
        Pn = ld16(src + (offn + 16u <= lim ? offn : off));
      }
      uint32_t st[4];
      const uint32_t lo = lane == 0 ? 1u : (uint32_t)lane;  // the counter's low byte (J0 for lane 0)
      aes_cached(st, ((lo << 8) | lb) ^ (k15 << 8), 0u);
      const v4u32 C = {Pu.x ^ st[0], Pu.y ^ st[1], Pu.z ^ st[2], Pu.w ^ st[3]};
      if (lane >= 2) st16(dst + off, make_uint4(C.x, C.y, C.z, C.w));
      if (OPEN && tls && lane >= 2) lastnz = block_last_nz(C.x, C.y, C.z, C.w, off, lastnz);
      if (lane == 0) { e0 = st[0]; e1 = st[1]; e2 = st[2]; e3 = st[3]; }
      if (lane == 1) {  // Y = 0 before the first step: Y = B, the AAD block
        if (tls) {
          y[0] = hdr0; y[1] = hdr1;
        } else {
#pragma unroll
          for (int q = 0; q < 16; q++)
            if ((uint32_t)q < aad_len) put_byte(y, q, aadp[q]);
        }
      }
      if (lane >= 2) {
        y[0] = OPEN ? Pu.x : C.x; y[1] = OPEN ? Pu.y : C.y; y[2] = OPEN ? Pu.z : C.z; y[3] = OPEN ? Pu.w : C.w;
      }
#ifdef ATLS_TT_STAMPS
      t_fast += __builtin_amdgcn_s_memtime() - t_step;  // counted with the fast steps
      n_fast++;
#endif
      continue;
    }
    pref = false;
    const bool use_pn = gen_pn;  // this general step follows a fast step that loaded its blocks
    gen_pn = false;
    if (ATLS_DBG_SKIP & 2) continue;
    if ((ATLS_DBG_SKIP & 16) && base + 64u >= S) continue;
    if ((ATLS_DBG_SKIP & 32) && base == 0u) continue;
    // counter block J0 + c (gcm.rs:89-96): c = s - na for data block s - 1 - na, 0 for slots 0..na
    const uint32_t c = (s > na) ? (s - na) : 0u;
    uint32_t cb[4] = {j0[0], j0[1], j0[2], j0[3]};
    if (is96) {
      cb[3] = j0[3] + c;  // (Yi & !0xFFFFFFFF) | counter, counter mod 2^32
    } else {            // Yi + counter as a 128-bit add
      uint64_t lo = (((uint64_t)cb[2] << 32) | cb[3]) + c;
      uint64_t hi = ((uint64_t)cb[0] << 32) | cb[1];
      if (lo < c) hi++;
      cb[0] = (uint32_t)(hi >> 32); cb[1] = (uint32_t)hi; cb[2] = (uint32_t)(lo >> 32); cb[3] = (uint32_t)lo;
    }
    uint32_t st[4];
#pragma unroll
    for (int w = 0; w < 4; w++) st[w] = bswap32(cb[w]);
    // issue the data load before the AES rounds so HBM latency hides under them
    uint32_t P[4] = {0, 0, 0, 0};
    const uint32_t g = s - 1;
    if (s >= 1 && s <= m && g >= na && g < na + nb) {
      const uint32_t off = (g - na) * 16;
      if (use_pn) {
        // Pn holds this block (off + 16 <= lim) or the input's last 16 bytes (off < lim): shift the block's
        // nv = lim - off bytes down from byte 16 - nv; past the input only the TLS content type (record.rs:173)
        const uint32_t t[4] = {Pn.x, Pn.y, Pn.z, Pn.w};
        if (off + 16u <= lim) {
          P[0] = t[0]; P[1] = t[1]; P[2] = t[2]; P[3] = t[3];
        } else {
          const uint32_t nv = off < lim ? lim - off : 0u, sh = 16u - nv, ws = sh >> 2, bs = sh & 3u;
          auto wd = [&](uint32_t i) { return i == 0 ? t[0] : i == 1 ? t[1] : i == 2 ? t[2] : i == 3 ? t[3] : 0u; };
#pragma unroll
          for (int w = 0; w < 4; w++) {
            uint32_t v = __builtin_amdgcn_alignbyte(wd((uint32_t)w + ws + 1u), wd((uint32_t)w + ws), bs);
            const int lo = 4 * w;
            if ((int)nv < lo + 4) v &= ((int)nv <= lo) ? 0u : (0xffffffffu >> (8 * (lo + 4 - (int)nv)));
            P[w] = nv ? v : 0u;
          }
          const uint32_t valid = min(16u, n_aead - off);
          if (nv < valid) P[nv >> 2] |= (uint32_t)d.content_type << (8 * (nv & 3u));
        }
      } else if (off + 16 <= in_bytes && (ATLS_GEN_VEC || src_al)) {
        const uint4 v = ATLS_GEN_VEC ? ld16(src + off) : *reinterpret_cast<const uint4*>(src + off);
        P[0] = v.x; P[1] = v.y; P[2] = v.z; P[3] = v.w;
      } else {
        const uint32_t valid = min(16u, n_aead - off);
#pragma unroll
        for (int q = 0; q < 16; q++) {  // compile-time byte index keeps P in registers
          if ((uint32_t)q < valid) {
            const uint32_t byte = (off + q < in_bytes) ? src[off + q] : (uint32_t)d.content_type;  // record.rs:173
            P[q >> 2] |= byte << (8 * (q & 3));
          }
        }
      }
    }
#ifdef ATLS_TT_STAMPS
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // timing build: the step's loads landed
    const uint64_t t_l = __builtin_amdgcn_s_memtime();
    t_ld += t_l - t_step;
#endif
    const bool live = !ATLS_GEN_MASK || s <= m;  // ATLS_GEN_MASK: lanes past the record skip the AES and GHASH work
    if (use_cache) {  // ctr = 1 for slots 0..na, else 1 + s - na: the step's ctr >> 8 is lane 63's
      const uint32_t ctr = cb[3];
      uint32_t hi;
      if constexpr (LN == 64) {
        hi = (uint32_t)__builtin_amdgcn_readlane((int)ctr, 63) >> 8;
      } else {  // the step's last slot's counter, across the waves
        const uint32_t sl = base + LN - 1u;
        hi = (j0[3] + (sl > na ? sl - na : 0u)) >> 8;
      }
      if (live) aes_cached(st, perm((ctr & 0xffu) ^ k15, lb, 0x0c0c0400u), hi);
    } else if (live) {
      aes_encrypt_tt<NR>(st, rk, rkr, lb);
    }
#ifdef ATLS_TT_STAMPS
    asm volatile("" ::"v"(st[0]), "v"(st[1]), "v"(st[2]), "v"(st[3]));
    t_aes += __builtin_amdgcn_s_memtime() - t_l;
#endif
    if (s == 0) { e0 = st[0]; e1 = st[1]; e2 = st[2]; e3 = st[3]; }
    uint32_t B[4] = {0, 0, 0, 0};
    if (s >= 1 && s <= m) {
      if (g < na) {  // AAD block (gcm.rs:78-87), zero-padded at the end (bytes.rs:110-121)
        if (tls) {
          B[0] = hdr0; B[1] = hdr1;
        } else {
          const uint32_t off = g * 16;
#pragma unroll
          for (int q = 0; q < 16; q++)
            if (off + q < aad_len) put_byte(B, q, aadp[off + q]);
        }
      } else if (g < na + nb) {  // data block (gcm.rs:89-119)
        const uint32_t off = (g - na) * 16;
        const uint32_t valid = min(16u, n_aead - off);
        uint32_t C[4] = {P[0] ^ st[0], P[1] ^ st[1], P[2] ^ st[2], P[3] ^ st[3]};
        if (valid < 16) {  // (data ^ Ek) >> overflow: only `valid` bytes exist
#pragma unroll
          for (int w = 0; w < 4; w++) {
            const int lo = 4 * w;
            if ((int)valid < lo + 4) C[w] &= ((int)valid <= lo) ? 0u : (0xffffffffu >> (8 * (lo + 4 - valid)));
          }
        }
        if (valid == 16 && (ATLS_GEN_VEC || dst_al)) {
          if (ATLS_GEN_VEC) st16(dst + off, make_uint4(C[0], C[1], C[2], C[3]));
          else *reinterpret_cast<uint4*>(dst + off) = make_uint4(C[0], C[1], C[2], C[3]);
        } else {
#pragma unroll
          for (int q = 0; q < 16; q++)
            if ((uint32_t)q < valid) dst[off + q] = (uint8_t)get_byte(C, q);
        }
        if (OPEN) {
#pragma unroll
          for (int w = 0; w < 4; w++) B[w] = P[w];  // GHASH over the ciphertext input
          if (tls) {
            const int j = last_nonzero(C, (int)valid);
            if (j >= 0) lastnz = ((int64_t)(off + j) << 8) | ((C[j >> 2] >> (8 * (j & 3))) & 0xffu);
          }
        } else {
#pragma unroll
          for (int w = 0; w < 4; w++) B[w] = C[w];
        }
      } else {  // length block: [len(A)]_64 || [len(C)]_64 in bits (gcm.rs:121)
        const uint64_t abits = (uint64_t)(tls ? 5u : aad_len) * 8u, cbits = (uint64_t)n_aead * 8u;
        B[0] = bswap32((uint32_t)(abits >> 32)); B[1] = bswap32((uint32_t)abits);
        B[2] = bswap32((uint32_t)(cbits >> 32)); B[3] = bswap32((uint32_t)cbits);
      }
    }
    // Y <- Y * H^64 ^ B on the lanes that hold a GHASH block; the others keep Y (s_last below).
    uint32_t yn[4] = {y[0], y[1], y[2], y[3]};
    if (base && !(ATLS_DBG_SKIP & 8) && live) ghash_mul(yn, wh);  // Y = 0 before the first step
    if (s >= 1 && s <= m) {
#pragma unroll
      for (int w = 0; w < 4; w++) y[w] = yn[w] ^ B[w];
    }
#ifdef ATLS_TT_STAMPS
    {
      const uint64_t dt = __builtin_amdgcn_s_memtime() - t_step;
      t_gen += dt;
      n_gen++;
      if (base == 0) { t_gen0 += dt; n_gen0++; } else t_genl += dt;
    }
#endif
  }
  TT_STAMP(t_loop);

  // ---- lane combine: Z = sum_l Y_l * H^(S - s_last(l)) ----
  uint32_t z[4] = {0, 0, 0, 0};
  const uint32_t wc = LN == 64 ? wb : wb + (4u + ((uint32_t)lane >> 6)) * (uint32_t)kGhashBytes;  // comb area
  if (s_last >= 1) {
    const uint32_t yb[4] = {bswap32(y[0]), bswap32(y[1]), bswap32(y[2]), bswap32(y[3])};
    lane_comb<NR, LAT>(yb, hp, z, wc, lane & 63);
  }
#pragma unroll
  for (int w = 0; w < 4; w++) z[w] = wave_xor(z[w]);
  const uint32_t xa = wb + 8u * (uint32_t)kGhashBytes;  // LN = 256: the waves' exchange area
  if (LN > 64) {
    if (OPEN) {  // the content-type scan's wave maxima travel with the partial tags
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) {
        const int64_t o = __shfl_xor(lastnz, off, 64);
        lastnz = o > lastnz ? o : lastnz;
      }
    }
    if ((lane & 63) == 0) {
      auto* x4 = reinterpret_cast<__attribute__((address_space(3))) v4u32*>(xa + 16u * ((uint32_t)lane >> 6));
      *x4 = v4u32{z[0], z[1], z[2], z[3]};
      if (OPEN) *reinterpret_cast<__attribute__((address_space(3))) int64_t*>(xa + 64u + 8u * ((uint32_t)lane >> 6)) = lastnz;
    }
    __syncthreads();
    if (lane == 0) {
#pragma unroll
      for (int w = 1; w < LN / 64; w++) {
        const v4u32 o = lds_u4(xa + 16u * (uint32_t)w);
        z[0] ^= o.x; z[1] ^= o.y; z[2] ^= o.z; z[3] ^= o.w;
        if (OPEN) {
          const int64_t ol = *reinterpret_cast<const __attribute__((address_space(3))) int64_t*>(xa + 64u + 8u * (uint32_t)w);
          lastnz = ol > lastnz ? ol : lastnz;
        }
      }
    }
  }
  if (defer) {  // the record's last slots, tag and verdict: gcm_tail_kernel
    if (OPEN && tls) {
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) {
        const int64_t o = __shfl_xor(lastnz, off, 64);
        lastnz = o > lastnz ? o : lastnz;
      }
    }
    if (lane == 0) {
      uint32_t* hdr = reinterpret_cast<uint32_t*>(A.tail);
      const uint32_t slot = atomicAdd(hdr, 1u);
      TailState* ts = reinterpret_cast<TailState*>(A.tail + kTailHdr) + slot;
      st16(reinterpret_cast<uint8_t*>(ts->z), make_uint4(z[0], z[1], z[2], z[3]));
      st16(reinterpret_cast<uint8_t*>(ts->e), make_uint4(e0, e1, e2, e3));
      ts->lastnz = lastnz;
      ts->rec = rec_idx;
    }
    return;
  }
  const uint32_t t0 = e0 ^ bswap32(z[0]), t1 = e1 ^ bswap32(z[1]), t2 = e2 ^ bswap32(z[2]), t3 = e3 ^ bswap32(z[3]);

  if (!OPEN) {
    if (lane == 0) {
      if (A.tags_out) st16(A.tags_out + 16ull * rec_idx, make_uint4(t0, t1, t2, t3));
      if (wire) {  // header || ciphertext || tag (record.rs:175-197)
        uint8_t* h = dst - 5;
        h[0] = (uint8_t)hdr0; h[1] = (uint8_t)(hdr0 >> 8); h[2] = (uint8_t)(hdr0 >> 16);
        h[3] = (uint8_t)(hdr0 >> 24); h[4] = (uint8_t)hdr1;
        st16(dst + n_aead, make_uint4(t0, t1, t2, t3));
      }
    }
  } else {
    // content-type scan (record.rs:229-237): wave max of (pos << 8 | byte) (LN = 256: done above)
    if (LN == 64) {
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) {
        const int64_t o = __shfl_xor(lastnz, off, 64);
        lastnz = o > lastnz ? o : lastnz;
      }
    }
    if (lane == 0) {
      const uint4 tg = ld16(wire ? src + len : A.tags_in + 16ull * rec_idx);  // WIRE: tag follows the ct
      const bool ok = (tg.x == t0) & (tg.y == t1) & (tg.z == t2) & (tg.w == t3);
      write_open_result(A, rec_idx, tls, len, ok, lastnz, hdr_ok);
    }
  }
#ifdef ATLS_TT_STAMPS
  TT_STAMP(t_end);
  if (lane == 0) {
    atomicAdd(&g_tt_stamps[0], (unsigned long long)(t_setup - t_start));
    atomicAdd(&g_tt_stamps[1], (unsigned long long)t_fast);
    atomicAdd(&g_tt_stamps[2], (unsigned long long)t_gen);
    atomicAdd(&g_tt_stamps[3], (unsigned long long)(t_end - t_loop));
    atomicAdd(&g_tt_stamps[4], 1ull);
    atomicAdd(&g_tt_stamps[5], (unsigned long long)n_fast);
    atomicAdd(&g_tt_stamps[6], (unsigned long long)n_gen);
    atomicAdd(&g_tt_stamps[8], (unsigned long long)t_gen0);
    atomicAdd(&g_tt_stamps[9], (unsigned long long)t_genl);
    atomicAdd(&g_tt_stamps[10], (unsigned long long)t_ld);
    atomicAdd(&g_tt_stamps[11], (unsigned long long)t_aes);
    atomicAdd(&g_tt_stamps[12], (unsigned long long)n_gen0);
  }
#endif
}

// ---- lane groups: 64/G records of one key per wave ------------------------------------------
// Key-grouped direct batches (plan.hip atls_launch_group): a run of records that share a key slot
// and a step count is sealed / opened by one wave, G lanes per record. The slots are those of
// gcm_record with lane gl = lane % G owning s = gl (mod G) of its group's record; the Horner
// multiplier is H^G (table from the key schedule's p4g seeds) and one lane combine, one table
// build and one counter-cache build serve 64/G records. A 16 KiB record's 1,028 slots fill
// 64.25 sixteen-lane steps instead of 16.06 wave steps plus a per-record tail, combine and table.
#ifndef ATLS_GCM_GROUP_LANES_128
#define ATLS_GCM_GROUP_LANES_128 8  // lanes per AES-128 record in a lane group (8, 16 or 32)
#endif
#ifndef ATLS_GCM_GROUP_LANES_256
#define ATLS_GCM_GROUP_LANES_256 16  // AES-192 / AES-256 records
#endif
// 8 lanes measured faster for AES-128 (C2 854 -> 873 GiB/s) and slower for AES-256 (C4 790 ->
// 745), same-box A/B (profiles/r02/ab_gcm_group_variants.log)
#ifndef ATLS_GROUP_TAIL
#define ATLS_GROUP_TAIL 4  // the last (TAIL / 4) x (waves in the grid) grouped records run as single records
#endif
#ifndef ATLS_GROUP_SHARES
#define ATLS_GROUP_SHARES 1  // work counters of a grouped batch (1..8): shares of region A by blockIdx % shares
                             // (8 measured no faster than 1: C2 850 vs 857 GiB/s, same-box A/B)
#endif
template <int NR>
constexpr int group_lanes() { return NR == 10 ? ATLS_GCM_GROUP_LANES_128 : ATLS_GCM_GROUP_LANES_256; }


// XOR of x over the lane's G-lane group: DPP within 8- / 16-lane rows, then rows by readlane.
template <int G>
__device__ __forceinline__ uint32_t group_xor(uint32_t x) {
  x ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false);
  x ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, false);
  x ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x141, 0xF, 0xF, false);
  if (G >= 16) x ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x140, 0xF, 0xF, false);
  if (G == 32) {
    const uint32_t a = (uint32_t)(__builtin_amdgcn_readlane((int)x, 0) ^ __builtin_amdgcn_readlane((int)x, 16));
    const uint32_t b = (uint32_t)(__builtin_amdgcn_readlane((int)x, 32) ^ __builtin_amdgcn_readlane((int)x, 48));
    x = (__lane_id() < 32) ? a : b;
  }
  return x;
}

// Whether the records at pos[0..ng) form a lane group: all accepted, one key slot, TLS or
// WIRE framing, the same number of G-slot steps, and few enough steps for the counter cache
// (lane gl holds ctr >> 8 = gl). Wave-uniform.
template <bool OPEN, int G>
__device__ __forceinline__ bool group_ok(const GcmArgs& A, const uint32_t* pos, uint32_t ng, uint32_t& key) {
  uint32_t steps0 = 0;
  for (uint32_t j = 0; j < ng; j++) {
    const uint32_t r = uni(cptr(pos)[j]);
    if (r >= A.n) return false;
    const atls_rec d = A.recs[r];
    if (direct_reject(d, A.ks, A.n_slots, OPEN) || d.mode == ATLS_MODE_RAW) return false;
    if (j == 0) key = d.key_slot;
    else if (d.key_slot != key) return false;
    const uint64_t n_aead = (uint64_t)d.len + (OPEN ? 0u : 1u);
    const uint64_t S = (n_aead + 15u) / 16u + 3u;  // E(J0), AAD, data, length
    if (S > (uint64_t)G * 256u) return false;
    const uint32_t steps = (uint32_t)((S + G - 1u) / G);
    if (j == 0) steps0 = steps;
    else if (steps != steps0) return false;
  }
  return true;
}

template <int NR, bool OPEN, int G>
__device__ void gcm_group(const GcmArgs& A, const KeySched* k, uint32_t rec_idx, uint32_t lb, uint32_t wb, int lane) {
  const uint32_t gl = (uint32_t)lane & (G - 1u);
  uint32_t rk[4 * (NR + 1)], rkr[4 * (NR + 1)];
#pragma unroll
  for (int i = 0; i < 4 * (NR + 1); i++) {
    rk[i] = cptr(k->rk)[i];  // one key for the whole wave
    rkr[i] = cptr(k->rkr)[i];
  }
  const atls_rec d = A.recs[rec_idx];  // this lane's group's record
  const bool wire = d.mode == ATLS_MODE_WIRE;
  const uint32_t len = d.len;
  const uint32_t n_aead = OPEN ? len : len + 1u;  // record.rs:172-173 inner plaintext
  const uint8_t* rec_in = A.in + d.in_off;
  const uint8_t* src = rec_in + ((OPEN && wire) ? 5u : 0u);
  uint8_t* dst = A.out + d.out_off + ((!OPEN && wire) ? 5u : 0u);
  const bool src_al = ((reinterpret_cast<uintptr_t>(src)) & 15u) == 0;
  const bool dst_al = ((reinterpret_cast<uintptr_t>(dst)) & 15u) == 0;
  // nonce = iv ^ (0^4 || be64(seq)) as raw words (key_schedule.rs:51-64); J0 = nonce || 1
  const uint64_t seq = d.seq;
  const uint32_t nraw[3] = {k->siv[0], k->siv[1] ^ bswap32((uint32_t)(seq >> 32)), k->siv[2] ^ bswap32((uint32_t)seq)};
  uint32_t hdr0, hdr1;
  bool hdr_ok = true;
  if (OPEN && wire) {
    hdr_ok = wire_header(rec_in, len, hdr0, hdr1);  // record.rs:219
  } else {
    const uint32_t L = n_aead + 16u;  // record.rs:176-183
    hdr0 = 0x17u | (0x03u << 8) | (0x03u << 16) | (((L >> 8) & 0xffu) << 24);
    hdr1 = L & 0xffu;
  }
  const uint32_t nb = (n_aead + 15u) / 16u;
  const uint32_t m = nb + 2u;  // GHASH blocks: AAD, data, length
  const uint32_t S = m + 1u;   // slots
  const uint32_t steps = uni((S + G - 1u) / G);  // the same for every group (group_ok)
  const uint32_t fast_end = 2u + min(len, n_aead) / 16u;  // slots [G, fast_end): whole 16-B data blocks

  if (steps > 1u) {
    uint32_t seed[4];
#pragma unroll
    for (int w = 0; w < 4; w++) seed[w] = k->p4g_be[G == 8 ? 0 : G == 16 ? 1 : 2][lane >> 1][w];
    ghash_table_entries<8>(wb, seed, lane >> 1, (lane & 1) * 8);
    wave_lds_sync();
  }
  uint32_t y[4] = {0, 0, 0, 0};
  uint32_t e0 = 0, e1 = 0, e2 = 0, e3 = 0;  // E_K(J0), lane gl = 0
  int64_t lastnz = -1;
  const uint32_t k15 = rk[3] >> 24;
  const uint32_t gl_addr = (gl << 8) | lb;  // T0 address of byte value gl
  const CtrCache cc = ctr_cache_build(nraw, gl, rk, rkr, lb);
  const int gsrc = lane & ~(G - 1);
  CtrCache cur{};

  int64_t s_last = -1;  // the lane's last GHASH slot (1..m)
  if (gl == 0) { if (m >= (uint32_t)G) s_last = (int64_t)(m / G) * G; }
  else if (gl <= m) s_last = (int64_t)gl + (int64_t)((m - gl) / G) * G;
  const uint32_t e_comb = s_last >= 1 ? S - (uint32_t)s_last : 1u;  // 1..G
  uint32_t hp[4];
#pragma unroll
  for (int w = 0; w < 4; w++) hp[w] = k->hpow_be[e_comb - 1][w];

  // ATLS_PREFETCH as in gcm_record: Pn / Pn2 hold the blocks of the next one or two fast steps
  uint4 Pn = make_uint4(0u, 0u, 0u, 0u), Pn2 = make_uint4(0u, 0u, 0u, 0u);
  bool pref = false;
  const uint32_t lim = min(len, n_aead);
  for (uint32_t t = 0; t < steps; t++) {
    const uint32_t base = t * (uint32_t)G;
    if ((base & 255u) == 0u) {  // a new ctr >> 8 (the same for every slot of the step): its cache words
      const int sl = gsrc + (int)(base >> 8);
      cur.u0r = (uint32_t)__shfl((int)cc.u0r, sl, 64);
      cur.k0 = (uint32_t)__shfl((int)cc.k0, sl, 64);
      cur.k1r = (uint32_t)__shfl((int)cc.k1r, sl, 64);
      cur.k2r = (uint32_t)__shfl((int)cc.k2r, sl, 64);
      cur.k3 = (uint32_t)__shfl((int)cc.k3, sl, 64);
    }
    const uint32_t s = base + gl;
    const bool fast = base >= (uint32_t)G && base + G <= fast_end;
    if (__builtin_amdgcn_ballot_w64(!fast) == 0) {  // every group: whole data blocks only
      const uint32_t off = (s - 2u) * 16u;
      const uint4 Pu = pref ? Pn : ld16(src + off);
      // ATLS_GCM_DOUBLE: the next step is fast too and shares this step's counter-cache words
      const bool dbl = NR >= ATLS_GCM_DOUBLE && ((base + G) & 255u) != 0u &&
                       __builtin_amdgcn_ballot_w64(!(base + 2u * G <= fast_end)) == 0;
      if (dbl) {
        const uint32_t off2 = off + 16u * G;
        const uint4 Pv = pref ? Pn2 : ld16(src + off2);
        if (ATLS_PREFETCH) {  // the blocks of steps t + 2 and t + 3 (used only if those are fast)
          Pn = ld16(src + pf_off(off2 + 16u * G, off, lim));
          Pn2 = ld16(src + pf_off(off2 + 32u * G, off, lim));
          pref = true;
        }
        uint32_t sa[4], sb[4];
        aes_ctr_r12(sa, gl_addr ^ (((base & 0xffu) ^ k15) << 8), cur, lb);  // ctr = s
        aes_ctr_r12(sb, gl_addr ^ ((((base + G) & 0xffu) ^ k15) << 8), cur, lb);  // ctr = s + G
        aes_rounds_tt2<NR, 3>(sa, sb, rk, rkr, lb);
        const uint32_t C[4] = {Pu.x ^ sa[0], Pu.y ^ sa[1], Pu.z ^ sa[2], Pu.w ^ sa[3]};
        const uint32_t D[4] = {Pv.x ^ sb[0], Pv.y ^ sb[1], Pv.z ^ sb[2], Pv.w ^ sb[3]};
        st16(dst + off, make_uint4(C[0], C[1], C[2], C[3]));
        st16(dst + off2, make_uint4(D[0], D[1], D[2], D[3]));
        if (OPEN) lastnz = block_last_nz(D[0], D[1], D[2], D[3], off2, block_last_nz(C[0], C[1], C[2], C[3], off, lastnz));
        ghash_mul(y, wb);
        if (OPEN) { y[0] ^= Pu.x; y[1] ^= Pu.y; y[2] ^= Pu.z; y[3] ^= Pu.w; }
        else { y[0] ^= C[0]; y[1] ^= C[1]; y[2] ^= C[2]; y[3] ^= C[3]; }
        ghash_mul(y, wb);
        if (OPEN) { y[0] ^= Pv.x; y[1] ^= Pv.y; y[2] ^= Pv.z; y[3] ^= Pv.w; }
        else { y[0] ^= D[0]; y[1] ^= D[1]; y[2] ^= D[2]; y[3] ^= D[3]; }
        t++;
        continue;
      }
      if (ATLS_PREFETCH) {
        const uint32_t offn = off + 16u * G;
        Pn = ld16(src + pf_off(offn, off, lim));
        Pn2 = ld16(src + pf_off(offn + 16u * G, off, lim));
        pref = true;  // used only if the next step is fast, and then every lane's load was in range
      }
      uint32_t st[4];
      aes_ctr_r12(st, gl_addr ^ (((base & 0xffu) ^ k15) << 8), cur, lb);  // ctr = s
      if (ATLS_TT_ISSUE_ALL) aes_rounds_tt1<NR, 3>(st, rk, rkr, lb);
      else aes_rounds_tt<NR, 3>(st, rk, rkr, lb);
      const uint32_t C[4] = {Pu.x ^ st[0], Pu.y ^ st[1], Pu.z ^ st[2], Pu.w ^ st[3]};
      st16(dst + off, make_uint4(C[0], C[1], C[2], C[3]));
      if (OPEN) lastnz = block_last_nz(C[0], C[1], C[2], C[3], off, lastnz);
      ghash_mul(y, wb);
      if (OPEN) { y[0] ^= Pu.x; y[1] ^= Pu.y; y[2] ^= Pu.z; y[3] ^= Pu.w; }
      else { y[0] ^= C[0]; y[1] ^= C[1]; y[2] ^= C[2]; y[3] ^= C[3]; }
      continue;
    }
    // general step: slot 0 = E_K(J0), slot 1 = AAD, slots 2..m-1 data, slot m = length block
    pref = false;
    const bool data = s >= 2u && s + 1u <= m;
    uint32_t P[4] = {0, 0, 0, 0};
    if (data) {
      const uint32_t off = (s - 2u) * 16u;
      if (off + 16u <= len && (ATLS_GEN_VEC || src_al)) {
        const uint4 v = ATLS_GEN_VEC ? ld16(src + off) : *reinterpret_cast<const uint4*>(src + off);
        P[0] = v.x; P[1] = v.y; P[2] = v.z; P[3] = v.w;
      } else {
        const uint32_t valid = min(16u, n_aead - off);
#pragma unroll
        for (int q = 0; q < 16; q++) {
          if ((uint32_t)q < valid) {
            const uint32_t byte = (off + q < len) ? src[off + q] : (uint32_t)d.content_type;  // record.rs:173
            P[q >> 2] |= byte << (8 * (q & 3));
          }
        }
      }
    }
    const uint32_t ctr = s > 1u ? s : 1u;  // J0 + (s - 1) for data slots
    uint32_t st[4];
    aes_ctr_r12(st, perm((ctr & 0xffu) ^ k15, lb, 0x0c0c0400u), cur, lb);
    aes_rounds_tt<NR, 3>(st, rk, rkr, lb);
    if (s == 0) { e0 = st[0]; e1 = st[1]; e2 = st[2]; e3 = st[3]; }
    uint32_t B[4] = {0, 0, 0, 0};
    if (s == 1u) {
      B[0] = hdr0; B[1] = hdr1;
    } else if (data) {
      const uint32_t off = (s - 2u) * 16u;
      const uint32_t valid = min(16u, n_aead - off);
      uint32_t C[4] = {P[0] ^ st[0], P[1] ^ st[1], P[2] ^ st[2], P[3] ^ st[3]};
      if (valid < 16) {
#pragma unroll
        for (int w = 0; w < 4; w++) {
          const int lo = 4 * w;
          if ((int)valid < lo + 4) C[w] &= ((int)valid <= lo) ? 0u : (0xffffffffu >> (8 * (lo + 4 - valid)));
        }
      }
      if (valid == 16 && (ATLS_GEN_VEC || dst_al)) {
        if (ATLS_GEN_VEC) st16(dst + off, make_uint4(C[0], C[1], C[2], C[3]));
        else *reinterpret_cast<uint4*>(dst + off) = make_uint4(C[0], C[1], C[2], C[3]);
      } else {
#pragma unroll
        for (int q = 0; q < 16; q++)
          if ((uint32_t)q < valid) dst[off + q] = (uint8_t)get_byte(C, q);
      }
      if (OPEN) {
#pragma unroll
        for (int w = 0; w < 4; w++) B[w] = P[w];
        const int j = last_nonzero(C, (int)valid);
        if (j >= 0) lastnz = ((int64_t)(off + j) << 8) | ((C[j >> 2] >> (8 * (j & 3))) & 0xffu);
      } else {
#pragma unroll
        for (int w = 0; w < 4; w++) B[w] = C[w];
      }
    } else if (s == m) {  // [len(A)]_64 || [len(C)]_64 in bits (gcm.rs:121)
      const uint64_t cbits = (uint64_t)n_aead * 8u;
      B[0] = 0; B[1] = bswap32(40u);
      B[2] = bswap32((uint32_t)(cbits >> 32)); B[3] = bswap32((uint32_t)cbits);
    }
    uint32_t yn[4] = {y[0], y[1], y[2], y[3]};
    if (base) ghash_mul(yn, wb);
    if (s >= 1u && s <= m) {
#pragma unroll
      for (int w = 0; w < 4; w++) y[w] = yn[w] ^ B[w];
    }
  }

  uint32_t z[4] = {0, 0, 0, 0};
  if (s_last >= 1) {
    const uint32_t yb[4] = {bswap32(y[0]), bswap32(y[1]), bswap32(y[2]), bswap32(y[3])};
    gf_mul_comb(yb, hp, z);
  }
#pragma unroll
  for (int w = 0; w < 4; w++) z[w] = group_xor<G>(z[w]);
  const uint32_t t0 = e0 ^ bswap32(z[0]), t1 = e1 ^ bswap32(z[1]), t2 = e2 ^ bswap32(z[2]), t3 = e3 ^ bswap32(z[3]);
  if (!OPEN) {
    if (gl == 0) {
      if (A.tags_out) st16(A.tags_out + 16ull * rec_idx, make_uint4(t0, t1, t2, t3));
      if (wire) {  // header || ciphertext || tag (record.rs:175-197)
        uint8_t* h = dst - 5;
        h[0] = (uint8_t)hdr0; h[1] = (uint8_t)(hdr0 >> 8); h[2] = (uint8_t)(hdr0 >> 16);
        h[3] = (uint8_t)(hdr0 >> 24); h[4] = (uint8_t)hdr1;
        st16(dst + n_aead, make_uint4(t0, t1, t2, t3));
      }
    }
  } else {
#pragma unroll
    for (int off = G / 2; off >= 1; off >>= 1) {  // content-type scan (record.rs:229-237), group max
      const int64_t o = __shfl_xor(lastnz, off, 64);
      lastnz = o > lastnz ? o : lastnz;
    }
    if (gl == 0) {
      const uint4 tg = ld16(wire ? src + len : A.tags_in + 16ull * rec_idx);
      const bool ok = (tg.x == t0) & (tg.y == t1) & (tg.z == t2) & (tg.w == t3);
      write_open_result(A, rec_idx, true, len, ok, lastnz, hdr_ok);
    }
  }
}

// One record by the whole wave (gcm_record), after the direct-mode descriptor check.
template <int NR, bool OPEN, bool LAT = false, int LN = 64>
__device__ __forceinline__ void gcm_one(const GcmArgs& A, uint32_t r, uint32_t lb, uint32_t wb, int lane) {
  {
    atls_rec d = A.recs[r];
    d.key_slot = uni(d.key_slot);
    d.len = uni(d.len);
    d.mode = (uint8_t)uni(d.mode);
    if (!A.idx) {  // direct mode: reject as the plan would
      const uint32_t st = uni(direct_reject(d, A.ks, A.n_slots, OPEN));
      if (st) {
        if (lane == 0) {
          atomicOr(A.err, 1u);
          if (OPEN) {
            atls_open_result rr = {0, (uint8_t)st, 0, {0, 0}};
            A.res[r] = rr;
          }
        }
        return;
      }
    }
    gcm_record<NR, OPEN, LAT, LN>(A, d, A.ks + d.key_slot, r, lb, wb, lane);
    wave_lds_sync();  // table reads of this record done before the next record rebuilds it
  }
}

// WAVES waves per workgroup (one record per wave at a time), one workgroup per CU: the LDS
// footprint (64 KiB tables + 8 KiB per wave) is what limits residency. One launch per AES round
// count (a kernel holds only that count's round keys); the waves take the records of that round
// count's work list (plan.hip, longest first) round-robin, spread over the workgroups, or a key-grouped direct batch's lane
// groups from a work counter.
// In-kernel clock (diagnostic build -DATLS_CLK_STAMPS, MI355X_MICROARCH.md "DVFS give-back" item 6): every
// wave adds its s_memtime and s_memrealtime spans over the whole kernel body to g_clk_stamps (read back and
// reset by atls_debug_clk_stamps); the clock is 100 MHz x sum(shader ticks) / sum(constant ticks). Checks
// atls_clock_probe, which reads the same counters from a wave beside the kernel (tools/clock_check.py).
#ifdef ATLS_CLK_STAMPS
__device__ unsigned long long g_clk_stamps[4];
#endif
template <bool OPEN, int kWaves, int NR>
__device__ __forceinline__ void gcm_kernel_body(const GcmArgs& A);

// BESIDE: the seal kernel of a mixed batch, which runs beside the ChaCha20-Poly1305 side kernel (engine.cpp
// run_batch): capped at 128 VGPRs (minimum ATLS_GCM_MINW = 4 waves per SIMD), so that a 128-VGPR ChaCha20-Poly1305
// wave (chacha_kernel<false, true>) still fits on each SIMD beside the workgroup's three AES-GCM waves (3 x 128 +
// 128 = 512). The seal kernel had grown to 129 VGPRs (136 allocated: 3 x 136 + 128 > 512), which kept the two
// kernels of a C5 seal off each other's SIMDs. Same-box A/B, 3 rounds, parity first (profiles/r06/ab_minw.log):
// with the cap on every 12-wave kernel C5 seal 0.276-0.281 -> 0.254-0.260 ms (shard), 2.030-2.049 -> 1.900-1.932
// ms (whole), but C2 seal 0.981-0.987 -> 1.006-1.007 ms and the opens 1-3 % slower -- so only this instance is
// capped (C2 and every open keep the 168 cap; the open kernel is at 128 anyway).
#ifndef ATLS_GCM_MINW
#define ATLS_GCM_MINW 4
#endif
template <bool OPEN, int kWaves, int NR, bool BESIDE = false>
__global__ __launch_bounds__(64 * kWaves, BESIDE ? ATLS_GCM_MINW : 1) void gcm_kernel(GcmArgs A) {
#ifdef ATLS_CLK_STAMPS
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  gcm_kernel_body<OPEN, kWaves, NR>(A);
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(&g_clk_stamps[0], t1 - t0);
    atomicAdd(&g_clk_stamps[1], r1 - r0);
    atomicAdd(&g_clk_stamps[2], 1ull);
  }
#else
  gcm_kernel_body<OPEN, kWaves, NR>(A);
#endif
}

#ifndef ATLS_TT_B128
#define ATLS_TT_B128 1  // 0: the replicated T-table rows written one word per store (round 4)
#endif
// The replicated T-tables (row x: T0[x] x32 | T1[x] x32, T1 = rotl8 T0) at LDS address 0, by NT threads: T0
// through the (still unused) GHASH area with one global load per thread instead of a dependent load per LDS
// word, then each row 16 bytes per store (four copies of one entry), the loop unrolled so the row reads of
// several stores are in flight at once. Ends with a barrier.
template <int NT>
__device__ __forceinline__ void build_ttables(uint32_t* smem, const uint32_t* t0, int t) {
  for (int i = t; i < 256; i += NT) smem[kTabBytes / 4 + i] = t0[i];
  __syncthreads();
  if (ATLS_TT_B128) {
#pragma unroll 8
    for (int i = t; i < kTabBytes / 16; i += NT) {
      const uint32_t v = smem[kTabBytes / 4 + (i >> 4)];
      const uint32_t w = (i & 8) ? rotl32(v, 8) : v;
      reinterpret_cast<uint4*>(smem)[i] = make_uint4(w, w, w, w);
    }
  } else {
    for (int i = t; i < kTabBytes / 4; i += NT) {
      const uint32_t v = smem[kTabBytes / 4 + (i >> 6)];
      smem[i] = (i & 32) ? rotl32(v, 8) : v;
    }
  }
  __syncthreads();
}

template <bool OPEN, int kWaves, int NR>
__device__ __forceinline__ void gcm_kernel_body(const GcmArgs& A) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  build_ttables<64 * kWaves>(smem, A.t0, (int)threadIdx.x);
  const int wave = (int)uni(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const uint32_t lb = 4u * (uint32_t)(lane & 31);
  const uint32_t wb = (uint32_t)kTabBytes + (ATLS_DBG_SHARED_GHASH ? 0u : (uint32_t)wave * kGhashBytes);
  const WorkList W{A.idx, A.plan, NR == 10 ? kListGcm10 : NR == 12 ? kListGcm12 : kListGcm14, A.n};
  const uint32_t stride = gridDim.x * kWaves;
  if (!A.gidx) {  // one record per wave
    // The work list runs longest first, `stride` positions per row. Row-major round-robin gave
    // workgroup b (one per CU) the 12 adjacent positions 12b..12b+11 of every row, i.e. CU 0 the
    // longest records of each row: on C5's AES records the busiest CU carried 1.18x the mean CU load.
    // Position p of a row goes to wave p / gridDim.x of workgroup p % gridDim.x (every CU samples the
    // whole row), and odd rows run backwards (the waves that took long records take short ones next):
    // 1.01x (simulated on the C5 shard).
    const uint32_t cnt = uni(W.size());
    const uint32_t p = ATLS_GCM_SPREAD ? (uint32_t)wave * gridDim.x + blockIdx.x : blockIdx.x * kWaves + wave;
    for (uint32_t row = 0; row * stride < cnt; row++) {
      const uint32_t q = row * stride + ((ATLS_GCM_SPREAD && (row & 1u)) ? stride - 1u - p : p);
      if (q < cnt) gcm_one<NR, OPEN>(A, uni(W.record(q)), lb, wb, lane);
    }
    if (A.done && cnt == 1u && blockIdx.x == 0 && wave == 0) signal_done(A.done, A.done_val, lane);
    return;
  }
  // Key-grouped direct batch (plan.h): region B (records that form no lane group) round-robin
  // first, then region A's lane-group runs from a work counter (ATLS_GROUP_SHARES counters over
  // shares of the runs), the last ~stride records one per unit, so the waves finish within about
  // one record of each other. (Round-robin runs instead: C4 688 vs 782 GiB/s, same-box A/B.)
  constexpr int kGroupLanes = group_lanes<NR>();
  static_assert(kGroupLanes == 8 || kGroupLanes == 16 || kGroupLanes == 32, "lane groups of 8, 16 or 32");
  static_assert(kGroupRun % (64 / kGroupLanes) == 0, "the plan's runs hold whole lane groups");
  constexpr uint32_t NG = 64 / kGroupLanes;
  const uint32_t n_a = uni(cptr(&A.ghdr->n_a)[0]), n_b = uni(cptr(&A.ghdr->n_b)[0]);
  {
    uint32_t p = blockIdx.x * kWaves + wave;
    uint32_t r = p < n_b ? uni(cptr(A.gidx)[n_a + p]) : 0u;
    for (; p < n_b; p += stride) {
      const uint32_t rn = p + stride < n_b ? uni(cptr(A.gidx)[n_a + p + stride]) : 0u;  // next index, early
      if (r < A.n) gcm_one<NR, OPEN>(A, r, lb, wb, lane);  // (the plan writes indices < n only)
      r = rn;
    }
  }
  const uint32_t nx = gridDim.x < (uint32_t)ATLS_GROUP_SHARES ? gridDim.x : (uint32_t)ATLS_GROUP_SHARES;
  const uint32_t x = blockIdx.x % nx;
  const uint32_t nq = n_a / NG;  // runs (n_a is a multiple of kGroupRun)
  const uint32_t q0 = (uint32_t)((uint64_t)nq * x / nx), sq = (uint32_t)((uint64_t)nq * (x + 1u) / nx) - q0;
  const uint32_t tail_q = stride * ATLS_GROUP_TAIL / (4u * nx * NG);
  const uint32_t nrun = sq > tail_q ? sq - tail_q : 0u;
  const uint32_t n_units = nrun + NG * (sq - nrun);
  if (n_units == 0) return;
  for (;;) {
    uint32_t v = 0;
    if (lane == 0) v = atomicAdd(&A.ghdr->work[x], 1u);
    const uint32_t u = uni(v);
    if (u >= n_units) break;
    uint32_t key = 0;
    if (u < nrun && group_ok<OPEN, kGroupLanes>(A, A.gidx + NG * (q0 + u), NG, key)) {
      const uint32_t mine = A.gidx[NG * (q0 + u) + (uint32_t)lane / kGroupLanes];  // this lane group's record
      gcm_group<NR, OPEN, kGroupLanes>(A, A.ks + key, mine, lb, wb, lane);
      wave_lds_sync();
      continue;
    }
    const uint32_t p0 = u < nrun ? NG * (q0 + u) : NG * (q0 + nrun) + (u - nrun), cnt = u < nrun ? NG : 1u;
#pragma unroll 1
    for (uint32_t j = 0; j < cnt; j++) {
      const uint32_t r = uni(cptr(A.gidx)[p0 + j]);
      if (r < A.n) gcm_one<NR, OPEN>(A, r, lb, wb, lane);
    }
  }
}

// ---- deferred last steps (ATLS_GCM_TAIL) ----------------------------------------------------
// A deferred record's last rem slots (data blocks and the length block; S_run >= 64 puts the AAD in the full
// steps) on kTailLanes lanes: lane gl takes tail slots i = gl, gl + kTailLanes, ... -- the counter block by T-table
// AES with the lane's own round keys (vector loads from its key schedule) against the workgroup's replicated
// T-tables, the ciphertext, and the slot's GHASH term. From Z' = X_{S_run - 1}, the Horner steps X <- (X ^ B_i) * H
// over the rem blocks (gcm.rs:88-121) unroll to X = (Z' ^ B_0) * H^rem ^ sum_{i >= 1} B_i * H^(rem - i), so each
// term is one independent product by a power from the key schedule (hpow_be, gf_mul_comb: the reference's gmult
// product, gcm.rs:21-40) and the group XORs its terms -- one AES block and one product deep per lane.
constexpr int kTailLanes = 4;
template <int NR, bool OPEN>
__device__ __forceinline__ void tail_record(const GcmArgs& A, const TailState& ts, uint32_t lb, uint32_t gl) {
  const uint32_t r = ts.rec;
  const atls_rec d = A.recs[r];
  const KeySched* k = A.ks + d.key_slot;
  const bool tls = d.mode != ATLS_MODE_RAW;  // (WIRE records are never deferred)
  const uint32_t len = d.len;
  const uint32_t n_aead = (tls && !OPEN) ? len + 1 : len;
  const uint32_t na = 1u, nb = (n_aead + 15u) / 16u, m = na + nb + 1u, S = m + 1u;
  const uint32_t rem = S - 64u * ((S - 1u) / 64u), S_run = S - rem;
  uint32_t x[4] = {0, 0, 0, 0};
  int64_t lastnz = -1;
  if (gl < rem) {
    uint32_t rk[4 * (NR + 1)], rkr[4 * (NR + 1)];
#pragma unroll
    for (int i = 0; i < NR + 1; i++) {
      const uint4 a = ld16(reinterpret_cast<const uint8_t*>(k->rk + 4 * i));
      const uint4 b = ld16(reinterpret_cast<const uint8_t*>(k->rkr + 4 * i));
      rk[4 * i] = a.x; rk[4 * i + 1] = a.y; rk[4 * i + 2] = a.z; rk[4 * i + 3] = a.w;
      rkr[4 * i] = b.x; rkr[4 * i + 1] = b.y; rkr[4 * i + 2] = b.z; rkr[4 * i + 3] = b.w;
    }
    const uint8_t* src = A.in + d.in_off;
    uint8_t* dst = A.out + d.out_off;
    uint32_t j0[3];  // be words of the 96-bit nonce; J0 = nonce || 1 (gcm.rs:59-74)
    if (tls) {
      const uint64_t seq = d.seq;
      j0[0] = bswap32(k->siv[0]);
      j0[1] = bswap32(k->siv[1]) ^ (uint32_t)(seq >> 32);
      j0[2] = bswap32(k->siv[2]) ^ (uint32_t)seq;
    } else {
      const uint8_t* iv = A.aux + d.aux_off;
#pragma unroll
      for (int w = 0; w < 3; w++)
        j0[w] = ((uint32_t)iv[4 * w] << 24) | ((uint32_t)iv[4 * w + 1] << 16) | ((uint32_t)iv[4 * w + 2] << 8) | iv[4 * w + 3];
    }
    const uint32_t aad_len = tls ? 5u : d.aad_len;
    for (uint32_t i = gl; i < rem; i += (uint32_t)kTailLanes) {
      const uint32_t sl = S_run + i, g = sl - 1u;  // slot sl holds GHASH block g
      uint32_t B[4] = {0, 0, 0, 0};
      if (g < na + nb) {  // data block, counter J0 + sl - na (gcm.rs:89-96)
        const uint32_t off = (g - na) * 16u, valid = min(16u, n_aead - off);
        uint32_t st[4] = {bswap32(j0[0]), bswap32(j0[1]), bswap32(j0[2]), bswap32(1u + (sl - na))};
        aes_encrypt_tt<NR>(st, rk, rkr, lb);
        uint32_t P[4] = {0, 0, 0, 0};
        if (valid == 16u && off + 16u <= len) {
          const uint4 v = ld16(src + off);
          P[0] = v.x; P[1] = v.y; P[2] = v.z; P[3] = v.w;
        } else {
          for (uint32_t q = 0; q < valid; q++)  // past the input only the TLS content type (record.rs:173)
            P[q >> 2] |= ((off + q < len) ? (uint32_t)src[off + q] : (uint32_t)d.content_type) << (8 * (q & 3));
        }
        uint32_t C[4] = {P[0] ^ st[0], P[1] ^ st[1], P[2] ^ st[2], P[3] ^ st[3]};
#pragma unroll
        for (int w = 0; w < 4; w++) {  // only `valid` bytes exist
          const int lo = 4 * w;
          if ((int)valid < lo + 4) C[w] &= ((int)valid <= lo) ? 0u : (0xffffffffu >> (8 * (lo + 4 - (int)valid)));
        }
        if (valid == 16u) {
          st16(dst + off, make_uint4(C[0], C[1], C[2], C[3]));
        } else {
          for (uint32_t q = 0; q < valid; q++) dst[off + q] = (uint8_t)(C[q >> 2] >> (8 * (q & 3)));
        }
        if (OPEN && tls) {
          const int jn = last_nonzero(C, (int)valid);
          if (jn >= 0) lastnz = ((int64_t)(off + (uint32_t)jn) << 8) | ((C[jn >> 2] >> (8 * (jn & 3))) & 0xffu);
        }
#pragma unroll
        for (int w = 0; w < 4; w++) B[w] = OPEN ? P[w] : C[w];
      } else {  // length block: [len(A)]_64 || [len(C)]_64 in bits (gcm.rs:121)
        const uint64_t abits = (uint64_t)aad_len * 8u, cbits = (uint64_t)n_aead * 8u;
        B[0] = bswap32((uint32_t)(abits >> 32)); B[1] = bswap32((uint32_t)abits);
        B[2] = bswap32((uint32_t)(cbits >> 32)); B[3] = bswap32((uint32_t)cbits);
      }
      uint32_t v[4] = {bswap32(B[0]), bswap32(B[1]), bswap32(B[2]), bswap32(B[3])}, hp[4], pr[4];
      if (i == 0) {
#pragma unroll
        for (int w = 0; w < 4; w++) v[w] ^= ts.z[w];
      }
#pragma unroll
      for (int w = 0; w < 4; w++) hp[w] = k->hpow_be[rem - i - 1u][w];  // H^(rem - i)
      gf_mul_comb(v, hp, pr);
#pragma unroll
      for (int w = 0; w < 4; w++) x[w] ^= pr[w];
    }
  }
  // the group's terms and (opens) content-type scans; lanes of a group are adjacent, the group is whole
#pragma unroll
  for (int off = kTailLanes / 2; off >= 1; off >>= 1) {
#pragma unroll
    for (int w = 0; w < 4; w++) x[w] ^= (uint32_t)__shfl_xor((int)x[w], off, kTailLanes);
    if (OPEN) {
      const int64_t o = __shfl_xor(lastnz, off, kTailLanes);
      lastnz = o > lastnz ? o : lastnz;
    }
  }
  if (gl != 0) return;
  if (OPEN && ts.lastnz > lastnz) lastnz = ts.lastnz;  // nothing non-zero in the tail: the full steps' scan
  const uint32_t t0 = ts.e[0] ^ bswap32(x[0]), t1 = ts.e[1] ^ bswap32(x[1]), t2 = ts.e[2] ^ bswap32(x[2]),
                 t3 = ts.e[3] ^ bswap32(x[3]);
  if (!OPEN) {
    if (A.tags_out) st16(A.tags_out + 16ull * r, make_uint4(t0, t1, t2, t3));
  } else {
    const uint4 tg = ld16(A.tags_in + 16ull * r);
    const bool ok = (tg.x == t0) & (tg.y == t1) & (tg.z == t2) & (tg.w == t3);
    write_open_result(A, r, tls, len, ok, lastnz, true);
  }
}

// The deferred records of the launch(es) just before it on the stream, kTailLanes threads per record; the last
// workgroup to finish zeroes the workspace's counters for the next batch (no memset launch).
constexpr int kTailThreads = 256;
template <bool OPEN>
__global__ __launch_bounds__(kTailThreads) void gcm_tail_kernel(GcmArgs A) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  uint32_t* hdr = reinterpret_cast<uint32_t*>(A.tail);
  const uint32_t cnt = __hip_atomic_load(hdr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  constexpr uint32_t kPer = kTailThreads / kTailLanes;  // records per workgroup pass
  if (blockIdx.x * kPer < cnt) {
    build_ttables<kTailThreads>(smem, A.t0, (int)threadIdx.x);
    const uint32_t lb = 4u * (threadIdx.x & 31u), gl = threadIdx.x % (uint32_t)kTailLanes;
    const TailState* st = reinterpret_cast<const TailState*>(A.tail + kTailHdr);
    for (uint32_t i0 = blockIdx.x * kPer; i0 < cnt; i0 += gridDim.x * kPer) {  // workgroup-uniform trip count
      const uint32_t i = i0 + threadIdx.x / (uint32_t)kTailLanes;
      if (i < cnt) {
        const TailState ts = st[i];
        const uint32_t nr = A.ks[A.recs[ts.rec].key_slot].nr;
        if (nr == 10) tail_record<10, OPEN>(A, ts, lb, gl);
        else if (nr == 12) tail_record<12, OPEN>(A, ts, lb, gl);
        else tail_record<14, OPEN>(A, ts, lb, gl);
      }
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    if (atomicAdd(hdr + 1, 1u) == gridDim.x - 1u) {  // every workgroup has read the count
      __hip_atomic_store(hdr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(hdr + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// The single call with its descriptor, IV || AAD, input and received tag in the launch's argument block
// (kSingleInline bytes at most; chacha.hip chacha_single has the same layout): 4 waves build the T-tables,
// wave 0 seals / opens the record and sets the completion flag. The record's key schedule (device memory)
// is read as soon as the wave starts, not after a descriptor read from mapped host memory.
struct GcmSingle {
  GcmArgs A;
  atls_rec d;          // in_off / aux_off relative to bytes
  uint32_t tag_off;    // open: the received tag at bytes + tag_off
  uint32_t pad[3];
  uint8_t bytes[kSingleInline];
};
constexpr int kSingleWaves = 4;
// T-tables, then gcm_record<LN = 256>'s eight 8 KiB areas and its 256-B exchange area
constexpr size_t kSingleLds = (size_t)kTabBytes + 8u * (size_t)kGhashBytes + 256u;
static_assert(kSingleLds <= 160u * 1024u, "the single-call kernel's LDS");
// One record by a 4-wave workgroup (the single call): T-tables, then the record by all four waves
// (gcm_record LN = 256); every wave's stores have left before wave 0 raises the completion flag.
template <bool OPEN, int NR>
__device__ __forceinline__ void single_record(const GcmArgs& A) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  build_ttables<64 * kSingleWaves>(smem, A.t0, (int)threadIdx.x);
  const int t = (int)threadIdx.x;
  gcm_one<NR, OPEN, true, 64 * kSingleWaves>(A, 0u, 4u * (uint32_t)(t & 31), (uint32_t)kTabBytes, t);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t < 64) signal_done(A.done, A.done_val, t);
}

template <bool OPEN, int NR>
__global__ __launch_bounds__(64 * kSingleWaves) void gcm_single(GcmSingle) {
  // the argument block itself (the only explicit argument, at offset 0), read in place: naming the
  // by-value parameter's members by address would copy all of it to scratch first
  const GcmSingle* S = (const GcmSingle*)__builtin_amdgcn_kernarg_segment_ptr();
  GcmArgs A = S->A;
  A.recs = &S->d;
  A.in = S->bytes;
  A.aux = S->bytes;
  if (OPEN) A.tags_in = S->bytes + S->tag_off;
  single_record<OPEN, NR>(A);
}

// The single call's records that do not fit the argument block: descriptor and data in the pinned block
// (or a device copy of it), the same 4-wave record.
template <bool OPEN, int NR>
__global__ __launch_bounds__(64 * kSingleWaves) void gcm_single_ptr(GcmArgs A) {
  single_record<OPEN, NR>(A);
}

// ---- The resident single-call server (opt-in, ATLS_SINGLE_RESIDENT=1) ----------------------
// A launch costs 5.9-6.4 us before the first instruction and after the flag (tools/single_call_floor.hip:
// empty_launch_*_flag_spin_us); a wave that stays resident and polls a doorbell word in mapped host memory
// answers in 1.7 us, 4.2 us with 1,552 B read from and written to mapped memory (resident_wave_doorbell_*).
// single_resident is one workgroup serving every call context of the process, both suites (a resident kernel
// holds its hardware queue, and the process has few: one server, not one per context or suite). The mapped
// block has a slot per context (doorbell, flag, request, reply) and a common area (alive, stop). Lanes 0..7 of
// wave 0 poll the slots' doorbells (s_sleep between polls; the other waves wait at the barrier); a slot whose
// doorbell differs from the value last served there holds request v = the doorbell value: its header and the
// largest request a slot holds come into LDS in one round trip of 16-byte loads, the record is sealed / opened
// from LDS into LDS -- ChaCha20-Poly1305 by q4_record (chacha_q4.h), AES-GCM by the single call's 4-wave
// gcm_record over the T-tables this server built once, when its first AES-GCM request came -- the reply goes
// out in 16-byte stores, then the slot's flag := v. The server leaves on the stop word or after idle_us
// without a request, writing alive := 0 as its last store -- an exit every wave reaches whatever the host does
// (the host sets the stop word at exit).
struct ResidentReq {
  const KeySched* ks;   // the key slot's schedule (device memory)
  atls_rec d;           // in_off / aux_off index bytes, key_slot 0 (ks is the slot's), out_off indexes the reply
  uint32_t tag_off;     // open: the received tag at bytes + tag_off
  uint32_t open;
  uint32_t nr;          // 0: ChaCha20-Poly1305; 10 / 12 / 14: AES-GCM with that many rounds
  uint32_t pad0;
  const uint32_t* t0;   // AES-GCM: the 256-entry T-table (global memory) the LDS tables are built from
  uint32_t* err;        // AES-GCM: the engine's sticky error word (the descriptor check's)
  uint64_t pad1[5];
};
static_assert(sizeof(ResidentReq) == 128, "resident request header");
constexpr int kResSlots = 8;
constexpr size_t kResBell = 0, kResFlag = 64, kResReq = 256, kResTag = 512, kResRes = 528, kResBytes = 1024,
                 kResOut = 8192, kResSlotBytes = 16384, kResCommon = kResSlots * kResSlotBytes, kResAlive = kResCommon,
                 kResStopAt = kResCommon + 64;
static_assert(kResReq + sizeof(ResidentReq) <= kResTag, "resident request header");
static_assert(kResBytes + kSingleInline <= kResOut && kResOut + kSingleInline + 16 <= kResSlotBytes, "resident slot");

template <int NR, bool OPEN>
__device__ __forceinline__ void resident_gcm(const ResidentReq& R, const atls_rec* rec, const uint8_t* in, uint8_t* out,
                                             uint8_t* sl) {
  const GcmArgs A{R.ks, rec, 1u, in, in, out, sl + kResTag, in + R.tag_off, (atls_open_result*)(sl + kResRes), R.t0,
                  nullptr, nullptr, R.err, 1u, nullptr, nullptr, nullptr, 0u};
  const int t = (int)threadIdx.x;
  gcm_one<NR, OPEN, true, 64 * kSingleWaves>(A, 0u, 4u * (uint32_t)(t & 31), (uint32_t)kTabBytes, t);
}

// The server's LDS past the AES-GCM area: the server has no static LDS, so the T-tables the GCM code addresses
// absolutely (TA: byte value << 8 | lane) sit at LDS address 0 as in the single-call kernels.
struct ResidentLds {
  uint4 stage_in[kSingleInline / 16], stage_out[kSingleInline / 16];
  uint4 hdr[sizeof(ResidentReq) / 16];
  atls_rec rec;
  int cmd_slot;
  uint32_t cmd_v;
  uint32_t pad[2];
  Q4Lds q4;
};
constexpr size_t kResidentLds = kSingleLds + sizeof(ResidentLds);
static_assert(kSingleLds % 16 == 0 && kResidentLds <= 160u * 1024u, "the resident server's LDS");

// GCM = false: a ChaCha20-Poly1305-only server (ATLS_SINGLE_RESIDENT=1); GCM = true serves both suites (=2). The
// server with the AES-GCM path (217 VGPRs against 100) first kept the request header in registers and spilled two
// of its fields to scratch on every request: its ChaCha20-Poly1305 calls were 0.9 us slower
// (profiles/r05/single/ab_resident_gcm*.log). With the header read from LDS where it is used the difference is
// 0-0.3 us (resident_modes_noscratch.log).
template <bool GCM>
__global__ __launch_bounds__(64 * kSingleWaves) void single_resident(uint8_t* blk, uint32_t idle_us) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];  // AES-GCM: T-tables, GHASH areas (kSingleLds)
  ResidentLds& S = *reinterpret_cast<ResidentLds*>(smem + kSingleLds / 4);
  int& cmd_slot = S.cmd_slot;
  uint32_t& cmd_v = S.cmd_v;
  uint4* hdr = S.hdr;
  uint4* stage_in = S.stage_in;
  uint4* stage_out = S.stage_out;
  atls_rec& rec = S.rec;
  const int t = (int)threadIdx.x;
  bool tables = false;  // the AES T-tables are in LDS (built at this server's first AES-GCM request)
  // lane i < 8 of wave 0 keeps the last value it served for slot i (the flag the host set before this server)
  uint32_t served = 0;
  if (t < kResSlots)
    served = __hip_atomic_load((uint32_t*)(blk + (size_t)t * kResSlotBytes + kResFlag), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
  for (;;) {
    if (t < 64) {  // wave 0: lanes 0..7 watch the slots' doorbells (one uncached load per lane and poll)
      const uint32_t* bell = (const uint32_t*)(blk + (size_t)(t < kResSlots ? t : 0) * kResSlotBytes + kResBell);
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      int slot = -1;
      uint32_t v = 0;
      for (uint32_t it = 0;; it++) {
        const uint32_t b = t < kResSlots ? __hip_atomic_load(bell, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : 0u;
        const unsigned long long m = __ballot(t < kResSlots && b != 0u && b != served);
        if (m) {
          slot = __builtin_ffsll((long long)m) - 1;
          v = (uint32_t)__shfl((int)b, slot, 64);
          break;
        }
        if ((it & 15u) == 15u) {
          const uint32_t stop = __builtin_amdgcn_readfirstlane(
              __hip_atomic_load((uint32_t*)(blk + kResStopAt), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
          if (stop || __builtin_amdgcn_s_memrealtime() - t0 > 100ull * idle_us) break;  // told to stop, or idle
        }
        __builtin_amdgcn_s_sleep(1);
      }
      if (t == 0) {
        cmd_slot = slot;
        cmd_v = v;
      }
      if (slot >= 0 && t == slot) served = v;
    }
    __syncthreads();
    const int slot = cmd_slot;
    const uint32_t v = cmd_v;
    if (slot < 0) break;
    uint8_t* sl = blk + (size_t)slot * kResSlotBytes;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // the request the host wrote before the doorbell
    // header and every byte a request can hold, in one round trip (the request's own size is in the header)
    constexpr int kIn = (int)(kSingleInline / 16), kHdr = (int)(sizeof(ResidentReq) / 16);
    if (t < kIn) stage_in[t] = ((const uint4*)(sl + kResBytes))[t];
    else if (t < kIn + kHdr) hdr[t - kIn] = ((const uint4*)(sl + kResReq))[t - kIn];
    __syncthreads();  // (also: every wave has read the command before wave 0 may overwrite it)
    // the request header stays in LDS: each path reads its fields where it uses them (copied into registers up
    // front, the AES-GCM path's fields were spilled to scratch on every request)
    const ResidentReq& RL = *reinterpret_cast<const ResidentReq*>(hdr);
    const uint32_t nr = __builtin_amdgcn_readfirstlane(RL.nr), open = __builtin_amdgcn_readfirstlane(RL.open);
    const uint32_t rlen = __builtin_amdgcn_readfirstlane(RL.d.len);
    if (nr == 0) {
      ResidentReq R;
      __builtin_memcpy(&R, hdr, sizeof R);
      atls_rec dl = R.d;
      dl.out_off = 0;
      if (open)
        q4_record<true>(R.ks, dl, (const uint8_t*)stage_in, R.tag_off, (uint8_t*)stage_out, sl + kResTag,
                        (atls_open_result*)(sl + kResRes), S.q4);
      else
        q4_record<false>(R.ks, dl, (const uint8_t*)stage_in, R.tag_off, (uint8_t*)stage_out, sl + kResTag,
                         (atls_open_result*)(sl + kResRes), S.q4);
    } else if constexpr (GCM) {
      if (!tables) {  // T0 through the (still unused) GHASH area, then the replicated rows (single_record)
        build_ttables<64 * kSingleWaves>(smem, RL.t0, t);
        tables = true;
      }
      if (t == 0) {  // the descriptor gcm_one reads: out_off indexes the reply, the slot's schedule is ks
        rec = RL.d;
        rec.out_off = 0;
        rec.key_slot = 0;
      }
      __syncthreads();
      const uint8_t* in = (const uint8_t*)stage_in;
      uint8_t* out = (uint8_t*)stage_out;
      if (nr == 10) {
        if (open) resident_gcm<10, true>(RL, &rec, in, out, sl);
        else resident_gcm<10, false>(RL, &rec, in, out, sl);
      } else if (nr == 12) {
        if (open) resident_gcm<12, true>(RL, &rec, in, out, sl);
        else resident_gcm<12, false>(RL, &rec, in, out, sl);
      } else {
        if (open) resident_gcm<14, true>(RL, &rec, in, out, sl);
        else resident_gcm<14, false>(RL, &rec, in, out, sl);
      }
    }
    __syncthreads();  // the reply is whole in LDS
    const uint32_t nout = (rlen + 15u) / 16u;
    for (uint32_t i = (uint32_t)t; i < nout; i += 64u * kSingleWaves) ((uint4*)(sl + kResOut))[i] = stage_out[i];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // every wave's stores have left
    if (t == 0) __hip_atomic_store((uint32_t*)(sl + kResFlag), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (t == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    __hip_atomic_store((uint32_t*)(blk + kResAlive), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

}  // namespace atls

extern "C" int atls_launch_gcm_single(int open, int nr, const void* ks, uint32_t n_slots, const atls_rec* d,
                                      const uint8_t* bytes, uint32_t nbytes, uint32_t tag_off, uint8_t* out,
                                      uint8_t* tags_out, atls_open_result* res, const uint32_t* t0, uint32_t* err,
                                      uint32_t* done, uint32_t done_val, hipStream_t s) {
  if (nbytes > atls::kSingleInline || !done) return ATLS_INTERNAL_ERROR;
  atls::GcmSingle S;
  S.A = atls::GcmArgs{(const atls::KeySched*)ks, nullptr, 1u, nullptr, nullptr, out, tags_out, nullptr, res, t0,
                      nullptr, nullptr, err, n_slots, nullptr, nullptr, done, done_val};
  S.d = *d;
  S.tag_off = tag_off;
  __builtin_memcpy(S.bytes, bytes, nbytes);
  const dim3 block(64 * atls::kSingleWaves);
  const size_t lds = atls::kSingleLds;
#define ATLS_SINGLE(NR)                                                                          \
  if (open) hipLaunchKernelGGL((atls::gcm_single<true, NR>), dim3(1), block, lds, s, S);         \
  else hipLaunchKernelGGL((atls::gcm_single<false, NR>), dim3(1), block, lds, s, S);
  if (nr == 10) { ATLS_SINGLE(10) }
  else if (nr == 12) { ATLS_SINGLE(12) }
  else if (nr == 14) { ATLS_SINGLE(14) }
  else return ATLS_INTERNAL_ERROR;
#undef ATLS_SINGLE
  return hipGetLastError() == hipSuccess ? 0 : ATLS_INTERNAL_ERROR;
}

// nr_mask: bit 0/1/2 = key slots with 10/12/14 rounds exist (one launch each); bit 3 = the seal runs beside a
// ChaCha20-Poly1305 kernel (a mixed batch: the kernel instance capped at 128 VGPRs). plan/idx: the
// batch plan of atls_launch_plan, or idx = nullptr for a direct batch (one round count only; the
// kernel validates and reports through err). gidx/ghdr: a direct batch's key groups
// (atls_launch_group) or nullptr. grid: workgroups per launch (one per CU). done / done_val: a
// one-record direct launch signals completion there (the single call), else ignored.
extern "C" int atls_launch_gcm(int open, const void* ks, const atls_rec* recs, uint32_t n, const uint8_t* in,
                               const uint8_t* aux, uint8_t* out, uint8_t* tags_out, const uint8_t* tags_in,
                               atls_open_result* res, const uint32_t* t0, const uint32_t* idx, void* plan,
                               uint32_t* err, uint32_t n_slots, int nr_mask, const uint32_t* gidx,
                               const uint32_t* ghdr, int grid, hipStream_t s, uint32_t* done, uint32_t done_val,
                               uint8_t* tail_ws) {
  if (n == 0) return 0;
  atls::GcmArgs A{(const atls::KeySched*)ks, recs, n, in, aux, out, tags_out, tags_in, res, t0, idx,
                  (atls::PlanHdr*)plan, err, n_slots, idx ? nullptr : gidx,
                  (atls::GroupHdr*)const_cast<uint32_t*>(ghdr), n == 1 ? done : nullptr, done_val,
                  (n == 1 && done) ? nullptr : tail_ws};
  if (n == 1 && done && !idx && !gidx && __builtin_popcount((unsigned)nr_mask) == 1) {  // the single call's longer records: 4 waves
    const dim3 b1(64 * atls::kSingleWaves);
#define ATLS_SINGLE_PTR(NR)                                                                            \
  if (open) hipLaunchKernelGGL((atls::gcm_single_ptr<true, NR>), dim3(1), b1, atls::kSingleLds, s, A);  \
  else hipLaunchKernelGGL((atls::gcm_single_ptr<false, NR>), dim3(1), b1, atls::kSingleLds, s, A);
    if (nr_mask & 1) { ATLS_SINGLE_PTR(10) }
    else if (nr_mask & 2) { ATLS_SINGLE_PTR(12) }
    else if (nr_mask & 4) { ATLS_SINGLE_PTR(14) }
#undef ATLS_SINGLE_PTR
    return hipGetLastError() == hipSuccess ? 0 : ATLS_INTERNAL_ERROR;
  }
  static const int waves = [] {
    const char* v = getenv("ATLS_GCM_WAVES");
    const int w = v ? atoi(v) : 12;
    if (ATLS_DBG_SHARED_GHASH && w == 16) return 16;
    return (w == 4 || w == 8 || w == 12) ? w : 12;
  }();
  uint32_t want = (n + waves - 1) / waves;
  uint32_t g = (uint32_t)grid < want ? (uint32_t)grid : want;
  const dim3 block(64 * waves);
  const size_t lds = atls::lds_bytes(waves);
  // nr_mask bit 3: a mixed batch's seal beside the ChaCha20-Poly1305 kernel (gcm_kernel BESIDE, AES-128 / -256)
  const bool beside = (nr_mask & 8) && !open && waves == 12;
#define ATLS_LAUNCH_NR(W, NR)                                                                           \
  if (open) hipLaunchKernelGGL((atls::gcm_kernel<true, W, NR>), dim3(g), block, lds, s, A);             \
  else if (W == 12 && NR != 12 && beside)                                                               \
    hipLaunchKernelGGL((atls::gcm_kernel<false, W, NR, W == 12 && NR != 12>), dim3(g), block, lds, s, A); \
  else hipLaunchKernelGGL((atls::gcm_kernel<false, W, NR>), dim3(g), block, lds, s, A);
#define ATLS_LAUNCH(W)                                 \
  if (waves == W) {                                    \
    if (nr_mask & 1) { ATLS_LAUNCH_NR(W, 10) }         \
    if (nr_mask & 2) { ATLS_LAUNCH_NR(W, 12) }         \
    if (nr_mask & 4) { ATLS_LAUNCH_NR(W, 14) }         \
  }
  ATLS_LAUNCH(4) ATLS_LAUNCH(8) ATLS_LAUNCH(12)
#if ATLS_DBG_SHARED_GHASH
  ATLS_LAUNCH(16)
#endif
#undef ATLS_LAUNCH
#undef ATLS_LAUNCH_NR
  if (A.tail && ATLS_GCM_TAIL > 0) {  // the deferred last steps of the launch(es) above (ATLS_GCM_TAIL)
    constexpr uint32_t per = atls::kTailThreads / atls::kTailLanes;
    const uint32_t want_t = (n + per - 1u) / per, cap_t = 4u * (uint32_t)grid;
    const size_t lds_t = atls::kTabBytes + 1024;  // the T-tables and build_ttables' staging row
    if (open) hipLaunchKernelGGL(atls::gcm_tail_kernel<true>, dim3(want_t < cap_t ? want_t : cap_t), dim3(atls::kTailThreads), lds_t, s, A);
    else hipLaunchKernelGGL(atls::gcm_tail_kernel<false>, dim3(want_t < cap_t ? want_t : cap_t), dim3(atls::kTailThreads), lds_t, s, A);
  }
  return hipGetLastError() == hipSuccess ? 0 : ATLS_INTERNAL_ERROR;
}

// Bytes of the tail workspace a batch of n records needs (engine.cpp; 0 when the build defers nothing).
extern "C" size_t atls_gcm_tail_bytes(uint32_t n) {
  return ATLS_GCM_TAIL > 0 ? atls::kTailHdr + sizeof(atls::TailState) * (size_t)n : 0;
}

// Compile-time experiment switches this library was built with (include/atls.h
// atls_build_flags): 0 for the product build, which must compute the reference's results.
extern "C" unsigned atls_chacha_dbg(void);  // chacha.hip: its timing-build switch (ATLS_CHACHA_DBG)
extern "C" unsigned atls_build_flags(void) {
  unsigned f = 0;
  if (ATLS_DBG_SKIP || atls_chacha_dbg()) f |= ATLS_BUILD_DBG_SKIP;
  if (ATLS_DBG_SHARED_GHASH) f |= ATLS_BUILD_DBG_SHARED_GHASH;
  if (!ATLS_CTR_CACHE) f |= ATLS_BUILD_NO_CTR_CACHE;
  if (ATLS_GHASH_ROT) f |= ATLS_BUILD_GHASH_ROT;
#ifdef ATLS_TT_STAMPS
  f |= ATLS_BUILD_TT_STAMPS;
#endif
#ifdef ATLS_CLK_STAMPS
  f |= ATLS_BUILD_CLK_STAMPS;
#endif
  return f;
}

// Debug: copy out (and reset) the in-kernel clock sums of a -DATLS_CLK_STAMPS build: {sum of shader-clock
// ticks, sum of 100 MHz ticks, waves}; -1 otherwise.
extern "C" int atls_debug_clk_stamps(unsigned long long* out) {
#ifdef ATLS_CLK_STAMPS
  unsigned long long h[4], z[4] = {};
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(atls::g_clk_stamps), sizeof(h)) != hipSuccess) return -1;
  if (hipMemcpyToSymbol(HIP_SYMBOL(atls::g_clk_stamps), z, sizeof(z)) != hipSuccess) return -1;
  for (int i = 0; i < 4; i++) out[i] = h[i];
  return 0;
#else
  (void)out;
  return -1;
#endif
}

// Debug: copy out (and reset) the phase timers of a -DATLS_TT_STAMPS build; -1 otherwise.
extern "C" int atls_debug_tt_stamps(unsigned long long* out) {
#ifdef ATLS_TT_STAMPS
  unsigned long long h[16], z[16] = {};
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(atls::g_tt_stamps), sizeof(h)) != hipSuccess) return -1;
  if (hipMemcpyToSymbol(HIP_SYMBOL(atls::g_tt_stamps), z, sizeof(z)) != hipSuccess) return -1;
  for (int i = 0; i < 16; i++) out[i] = h[i];
  return 0;
#else
  (void)out;
  return -1;
#endif
}

// The resident single-call server on stream s (single_resident): blk = the mapped block's device address; gcm:
// the server also takes AES-GCM calls.
extern "C" int atls_launch_single_resident(uint8_t* blk, uint32_t idle_us, int gcm, hipStream_t s) {
  const dim3 b(64 * atls::kSingleWaves);
  if (gcm) hipLaunchKernelGGL(atls::single_resident<true>, dim3(1), b, atls::kResidentLds, s, blk, idle_us);
  else hipLaunchKernelGGL(atls::single_resident<false>, dim3(1), b, atls::kResidentLds, s, blk, idle_us);
  return hipGetLastError() == hipSuccess ? 0 : ATLS_INTERNAL_ERROR;
}
