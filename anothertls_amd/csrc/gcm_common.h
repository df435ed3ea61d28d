// Pieces of the AES-GCM record kernel (gcm.hip): LDS/VALU helpers, the 4-bit GHASH tables, the
// comb multiply of the lane combine, byte helpers for partial blocks and the kernel argument block.
#pragma once
#include "plan.h"

namespace atls {

__device__ __forceinline__ void wave_lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint32_t rot16(uint32_t x) { return (x << 16) | (x >> 16); }
__device__ __forceinline__ uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel) {
  return __builtin_amdgcn_perm(hi, lo, sel);
}

// Read-only data (key schedules, descriptors) through the constant address space: loads from a
// wave-uniform address become scalar loads into SGPRs.
template <typename T>
__device__ __forceinline__ const __attribute__((address_space(4))) T* cptr(const T* p) {
  return (const __attribute__((address_space(4))) T*)(p);
}

__device__ __forceinline__ uint32_t lds_u32(uint32_t byte_addr) {
  return *reinterpret_cast<const __attribute__((address_space(3))) uint32_t*>(byte_addr);
}
typedef uint32_t v4u32 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ v4u32 lds_u4(uint32_t byte_addr) {
  return *reinterpret_cast<const __attribute__((address_space(3))) v4u32*>(byte_addr);
}

// ---- GHASH ---------------------------------------------------------------------------------
// A table at LDS byte address wb (256-B aligned, < 2^24): entry [p][n] = (nibble n at position
// p) * H^e, raw words, p = 2*byte + (low nibble ? 1 : 0) covering x^(4p)..x^(4p+3) (n's bit 3
// is x^(4p)). A position's 16 entries x 16 B fill exactly one 256-B bank row, so lookups never
// bank-conflict. This writes entries n0 .. n0+CNT-1 of position p from seed = x^(4p) * H^e.
// ATLS_GHASH_ROT (CNT = 8, lane = 2p + n0/8, the caller's layout): write j of a lane stores
// entry n0 + ((j + lane) & 7). A ds_write_b128 serves lanes in groups of 8 with bank (a/4) mod
// 32; in entry order all 8 hit one 16-B bank quad (8-way, 6 % of the GCM kernel's LDS cycles),
// rotated they hit 8 different quads. Off by default: conflict-free but no faster,
// and the run-time entry index adds 2.4 % VALU instructions.
#ifndef ATLS_GHASH_ROT
#define ATLS_GHASH_ROT 0
#endif
template <int CNT>
__device__ __forceinline__ void ghash_table_entries(uint32_t wb, const uint32_t (&seed_be)[4], int p, int n0) {
  uint32_t P0[4], P1[4], P2[4], P3[4];
#pragma unroll
  for (int w = 0; w < 4; w++) P0[w] = seed_be[w];
#pragma unroll
  for (int w = 0; w < 4; w++) P1[w] = P0[w];
  gf_mulx_be(P1);
#pragma unroll
  for (int w = 0; w < 4; w++) P2[w] = P1[w];
  gf_mulx_be(P2);
#pragma unroll
  for (int w = 0; w < 4; w++) P3[w] = P2[w];
  gf_mulx_be(P3);
  uint32_t r0[4], r1[4], r2[4], r3[4];
#pragma unroll
  for (int w = 0; w < 4; w++) {
    r0[w] = bswap32(P0[w]); r1[w] = bswap32(P1[w]); r2[w] = bswap32(P2[w]); r3[w] = bswap32(P3[w]);
  }
#pragma unroll
  for (int j = 0; j < CNT; j++) {
    const int nv = (ATLS_GHASH_ROT && CNT == 8) ? n0 + ((j + 2 * p + (n0 >> 3)) & 7) : n0 + j;
    uint32_t e[4];
#pragma unroll
    for (int w = 0; w < 4; w++)
      e[w] = ((nv & 8) ? r0[w] : 0u) ^ ((nv & 4) ? r1[w] : 0u) ^ ((nv & 2) ? r2[w] : 0u) ^ ((nv & 1) ? r3[w] : 0u);
    v4u32 ev = {e[0], e[1], e[2], e[3]};
    *reinterpret_cast<__attribute__((address_space(3))) v4u32*>(wb + (uint32_t)(p * 256 + nv * 16)) = ev;
  }
}

// y <- y * H^e (raw words) via 32 table lookups. Each nibble's table offset (n * 16) is the
// nibble's byte of (y & 0xF0F0F0F0) or ((y << 4) & 0xF0F0F0F0), OR-ed onto the table base.
// GROUP > 0: lookups go out GROUP at a time (4*GROUP VGPRs in flight instead of up to 128), each
// group followed by a scheduling fence.
template <int GROUP = 0>
__device__ __forceinline__ void ghash_mul_tab(uint32_t (&y)[4], uint32_t wb) {
  uint32_t a0 = 0, a1 = 0, a2 = 0, a3 = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const uint32_t hi4 = y[i] & 0xF0F0F0F0u, lo4 = (y[i] << 4) & 0xF0F0F0F0u;
#pragma unroll
    for (int b = 0; b < 4; b++) {
      const uint32_t byte = 4 * i + b;
      // address = wb | (nibble << 4): byte 0 from the nibble's byte, bytes 1-2 from wb (one v_perm)
      const uint32_t sel = 0x0c020100u | (4u + b);
      const v4u32 eh = lds_u4(perm(hi4, wb, sel) + (2 * byte) * 256);
      const v4u32 el = lds_u4(perm(lo4, wb, sel) + (2 * byte + 1) * 256);
      a0 = xor3(a0, eh.x, el.x); a1 = xor3(a1, eh.y, el.y); a2 = xor3(a2, eh.z, el.z); a3 = xor3(a3, eh.w, el.w);
    }
    if (GROUP > 0 && ((i + 1) * 8) % (GROUP > 0 ? GROUP : 1) == 0) __builtin_amdgcn_sched_barrier(0);
  }
  y[0] = a0; y[1] = a1; y[2] = a2; y[3] = a3;
}

// The same product with W lookups issued before their first use (4W VGPRs in flight): 32 / W
// LDS round trips per multiply, where the compiler alone waits after every few lookups. Microbenchmarks only
// (tools/ubench/step_ubench.hip, corun_ubench.hip): in the record kernels it failed parity at W = 16 (round 6).
template <int W>
__device__ __forceinline__ void ghash_mul_tab_wide(uint32_t (&y)[4], uint32_t wb) {
  uint32_t a0 = 0, a1 = 0, a2 = 0, a3 = 0;
#pragma unroll
  for (int g = 0; g < 32; g += W) {
    v4u32 e[W];
#pragma unroll
    for (int q = 0; q < W; q++) {
      const int byte = (g + q) >> 1, i = byte >> 2, b = byte & 3;
      const uint32_t nib4 = ((g + q) & 1) ? (y[i] << 4) & 0xF0F0F0F0u : y[i] & 0xF0F0F0F0u;
      e[q] = lds_u4(perm(nib4, wb, 0x0c020100u | (4u + b)) + (g + q) * 256);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int q = 0; q < W; q += 2) {
      a0 = xor3(a0, e[q].x, e[q + 1].x); a1 = xor3(a1, e[q].y, e[q + 1].y);
      a2 = xor3(a2, e[q].z, e[q + 1].z); a3 = xor3(a3, e[q].w, e[q + 1].w);
    }
  }
  y[0] = a0; y[1] = a1; y[2] = a2; y[3] = a3;
}

// z = x * p in GF(2^128), be words: the same product as gf_mul_be (gcm.rs:21-40 gmult), as a
// transposed comb. With Q_w = p * X^(32w) and c(i) the coefficient of X^i in x (bit 31 - i%32 of
// word i/32): x*p = sum_{j<32} X^j * T_j, T_j = sum_w c(32w + j) Q_w. Horner over j = 31..0 costs
// one multiply-by-X and 16 masked XORs per j: 32 iterations instead of gf_mul_be's 128.
__device__ __forceinline__ void gf_mul_comb(const uint32_t (&x)[4], const uint32_t (&p)[4], uint32_t (&z)[4]) {
  uint32_t q[4][4];
#pragma unroll
  for (int c = 0; c < 4; c++) q[0][c] = p[c];
#pragma unroll
  for (int t = 1; t < 4; t++) {  // q[t] = q[t-1] * X^32: word shift; word 3 folds back via X^128 = 1+X+X^2+X^7
    const uint32_t w = q[t - 1][3];
    q[t][0] = w ^ (w >> 1) ^ (w >> 2) ^ (w >> 7);
    q[t][1] = q[t - 1][0] ^ (w << 31) ^ (w << 30) ^ (w << 25);
    q[t][2] = q[t - 1][1];
    q[t][3] = q[t - 1][2];
  }
  uint32_t z0 = 0, z1 = 0, z2 = 0, z3 = 0;
  // Rolled: the unrolled form lets the compiler materialise all 128 masks at once.
#pragma unroll 1
  for (int j = 31; j >= 0; j--) {
    {  // z <- z * X (a no-op on the first pass, z = 0)
      const uint32_t r = (uint32_t)((int32_t)(z3 << 31) >> 31) & 0xE1000000u;
      z3 = __builtin_amdgcn_alignbit(z2, z3, 1);
      z2 = __builtin_amdgcn_alignbit(z1, z2, 1);
      z1 = __builtin_amdgcn_alignbit(z0, z1, 1);
      z0 = (z0 >> 1) ^ r;
    }
#pragma unroll
    for (int w = 0; w < 4; w++) {
      const uint32_t m = (uint32_t)((int32_t)(x[w] << j) >> 31);  // c(32w + j): bit 31 - j of x[w]
      z0 ^= m & q[w][0]; z1 ^= m & q[w][1]; z2 ^= m & q[w][2]; z3 ^= m & q[w][3];
    }
  }
  z[0] = z0; z[1] = z1; z[2] = z2; z[3] = z3;
}

// The same product through per-lane tables in the LDS at tb (the wave's 8 KiB GHASH table, whose
// last product has been read by then: a wave's LDS operations run in order), lane l's entry n at
// tb + n*1024 + l*16 (a ds_read_b128 lane group's 16 lanes hit 16 different bank quads whatever n
// each reads). The lookups do not depend on z, so they issue ahead of the Horner chain.
//   MODE 1: entry n (0..7) = XOR of Q_w over the set bits w of n; one lookup serves words 0-2 of
//           x, word 3 keeps its masked XORs: 45 -> 25 VALU instructions per j.
//   MODE 2: entries 0..3 from (Q_0, Q_1), 4..7 from (Q_2, Q_3); two lookups per j, no masked XORs:
//           ~20 VALU instructions and twice the LDS reads.
// ATLS_COMB_LDS picks the mode for gcm_record (0 = gf_mul_comb); the lane-group kernel keeps
// gf_mul_comb, where the LDS form measured no faster (C2) or 1 % slower (C4).
#ifndef ATLS_COMB_LDS
#define ATLS_COMB_LDS 1
#endif
#ifndef ATLS_COMB_UNROLL
#define ATLS_COMB_UNROLL 4
#endif
template <int MODE>
__device__ __forceinline__ void gf_mul_comb_lds(const uint32_t (&x)[4], const uint32_t (&p)[4], uint32_t (&z)[4],
                                                uint32_t tb, int lane) {
  uint32_t q[4][4];
#pragma unroll
  for (int c = 0; c < 4; c++) q[0][c] = p[c];
#pragma unroll
  for (int t = 1; t < 4; t++) {
    const uint32_t w = q[t - 1][3];
    q[t][0] = w ^ (w >> 1) ^ (w >> 2) ^ (w >> 7);
    q[t][1] = q[t - 1][0] ^ (w << 31) ^ (w << 30) ^ (w << 25);
    q[t][2] = q[t - 1][1];
    q[t][3] = q[t - 1][2];
  }
  const uint32_t la = tb + (uint32_t)lane * 16u;
#pragma unroll
  for (int n = 0; n < 8; n++) {
    v4u32 e;
#pragma unroll
    for (int c = 0; c < 4; c++) {
      if (MODE == 1) e[c] = ((n & 1) ? q[0][c] : 0u) ^ ((n & 2) ? q[1][c] : 0u) ^ ((n & 4) ? q[2][c] : 0u);
      else e[c] = ((n & 1) ? q[(n >> 2) * 2][c] : 0u) ^ ((n & 2) ? q[(n >> 2) * 2 + 1][c] : 0u);
    }
    *reinterpret_cast<__attribute__((address_space(3))) v4u32*>(la + (uint32_t)n * 1024u) = e;
  }
  uint32_t z0 = 0, z1 = 0, z2 = 0, z3 = 0;
#pragma unroll ATLS_COMB_UNROLL
  for (int j = 31; j >= 0; j--) {
    const uint32_t b = 31u - (uint32_t)j;  // c(32w + j) = bit b of x[w]
    const uint32_t r = (uint32_t)__builtin_amdgcn_sbfe((int)z3, 0, 1) & 0xE1000000u;  // z <- z * X
    const uint32_t s3 = __builtin_amdgcn_alignbit(z2, z3, 1);
    const uint32_t s2 = __builtin_amdgcn_alignbit(z1, z2, 1);
    const uint32_t s1 = __builtin_amdgcn_alignbit(z0, z1, 1);
    const uint32_t s0 = z0 >> 1;
    if (MODE == 1) {
      const uint32_t idx = __builtin_amdgcn_ubfe(x[0], b, 1) | (__builtin_amdgcn_ubfe(x[1], b, 1) << 1) |
                           (__builtin_amdgcn_ubfe(x[2], b, 1) << 2);
      const v4u32 t = lds_u4(la + (idx << 10));
      const uint32_t m = (uint32_t)__builtin_amdgcn_sbfe((int)x[3], b, 1);
      z0 = xor3(s0, r, t.x ^ (m & q[3][0]));
      z1 = xor3(s1, t.y, m & q[3][1]);
      z2 = xor3(s2, t.z, m & q[3][2]);
      z3 = xor3(s3, t.w, m & q[3][3]);
    } else {
      const uint32_t ia = __builtin_amdgcn_ubfe(x[0], b, 1) | (__builtin_amdgcn_ubfe(x[1], b, 1) << 1);
      const uint32_t ib = __builtin_amdgcn_ubfe(x[2], b, 1) | (__builtin_amdgcn_ubfe(x[3], b, 1) << 1);
      const v4u32 ta = lds_u4(la + (ia << 10)), tb4 = lds_u4(la + 4096u + (ib << 10));
      z0 = xor3(s0, r, ta.x) ^ tb4.x;
      z1 = xor3(s1, ta.y, tb4.y);
      z2 = xor3(s2, ta.z, tb4.z);
      z3 = xor3(s3, ta.w, tb4.w);
    }
  }
  z[0] = z0; z[1] = z1; z[2] = z2; z[3] = z3;
}

// ---- multiplying by x^m and squaring (key setup, the single-call kernel's tables) ----
// v <- v * x^m in GF(2^128), be words (gf_mulx_be applied m times), 1 <= m <= 64, m may differ per lane.
// With V the 128-bit number v0:v1:v2:v3 (the coefficient of x^i at bit 127 - i), V * x^m = (V >> m) plus
// the m low bits pushed past x^127: moved to the top as S = V << (128 - m) they stand for s(x) with
// V * x^m's overflow = s(x) * x^128 = s(x) * (1 + x + x^2 + x^7) (the 0xE1 of gf_mulx_be), i.e.
// S ^ S >> 1 ^ S >> 2 ^ S >> 7 -- no second reduction, deg s + 7 < 128.
__host__ __device__ inline void gf_mulxk64(uint32_t (&v)[4], uint32_t m) {
  const uint64_t hi = ((uint64_t)v[0] << 32) | v[1], lo = ((uint64_t)v[2] << 32) | v[3];
  uint64_t rhi, rlo, s;
  if (m >= 64) {
    rhi = 0;
    rlo = hi;
    s = lo;
  } else {
    rhi = hi >> m;
    rlo = (lo >> m) | (hi << (64 - m));
    s = lo << (64 - m);
  }
  rhi ^= s ^ (s >> 1) ^ (s >> 2) ^ (s >> 7);
  rlo ^= (s << 63) ^ (s << 62) ^ (s << 57);
  v[0] = (uint32_t)(rhi >> 32);
  v[1] = (uint32_t)rhi;
  v[2] = (uint32_t)(rlo >> 32);
  v[3] = (uint32_t)rlo;
}

// v <- v * x^m, 0 <= m <= 127.
__host__ __device__ inline void gf_mulxk(uint32_t (&v)[4], uint32_t m) {
  if (m > 64) {
    gf_mulxk64(v, 64);
    m -= 64;
  }
  if (m) gf_mulxk64(v, m);
}

// v <- v^2 in GF(2^128), be words. Squaring is linear: the coefficient of x^i moves to x^(2i), i.e. bit
// b of each 64-bit half to bit 2b+1 of 128 bits; the high half's image stands for O(x) * x^128 =
// O(x) * (1 + x + x^2 + x^7), folded back with the reducing shifts of gf_mulxk64.
__device__ __forceinline__ uint64_t spread32(uint32_t x) {  // bit b -> bit 2b
  uint64_t v = x;
  v = (v | (v << 16)) & 0x0000FFFF0000FFFFull;
  v = (v | (v << 8)) & 0x00FF00FF00FF00FFull;
  v = (v | (v << 4)) & 0x0F0F0F0F0F0F0F0Full;
  v = (v | (v << 2)) & 0x3333333333333333ull;
  v = (v | (v << 1)) & 0x5555555555555555ull;
  return v;
}
__device__ __forceinline__ void gf_square(uint32_t (&v)[4]) {
  // low half x^0..x^63 (words 0, 1) -> x^0..x^126; high half x^64..x^127 (words 2, 3) -> O(x) * x^128
  const uint64_t a_hi = spread32(v[0]) << 1, a_lo = spread32(v[1]) << 1;
  const uint64_t o_hi = spread32(v[2]) << 1, o_lo = spread32(v[3]) << 1;
  uint32_t o[4] = {(uint32_t)(o_hi >> 32), (uint32_t)o_hi, (uint32_t)(o_lo >> 32), (uint32_t)o_lo};
  uint32_t o1[4] = {o[0], o[1], o[2], o[3]}, o2[4] = {o[0], o[1], o[2], o[3]}, o7[4] = {o[0], o[1], o[2], o[3]};
  gf_mulxk64(o1, 1);
  gf_mulxk64(o2, 2);
  gf_mulxk64(o7, 7);
  v[0] = (uint32_t)(a_hi >> 32) ^ o[0] ^ o1[0] ^ o2[0] ^ o7[0];
  v[1] = (uint32_t)a_hi ^ o[1] ^ o1[1] ^ o2[1] ^ o7[1];
  v[2] = (uint32_t)(a_lo >> 32) ^ o[2] ^ o1[2] ^ o2[2] ^ o7[2];
  v[3] = (uint32_t)a_lo ^ o[3] ^ o1[3] ^ o2[3] ^ o7[3];
}

// XOR of x over the wave without the LDS (ds_bpermute) path of __shfl_xor: four DPP steps leave
// every lane with its 16-lane row's XOR (quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror,
// row_mirror), then four v_readlane combine the rows. Wave-uniform result.
__device__ __forceinline__ uint32_t wave_xor(uint32_t x) {
  x ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false);
  x ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, false);
  x ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x141, 0xF, 0xF, false);
  x ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x140, 0xF, 0xF, false);
  return (uint32_t)(__builtin_amdgcn_readlane((int)x, 0) ^ __builtin_amdgcn_readlane((int)x, 16) ^
                    __builtin_amdgcn_readlane((int)x, 32) ^ __builtin_amdgcn_readlane((int)x, 48));
}

// ---- byte helpers for partial / unaligned blocks -------------------------------------------
__device__ __forceinline__ void put_byte(uint32_t w[4], int q, uint32_t v) { w[q >> 2] |= v << (8 * (q & 3)); }
__device__ __forceinline__ uint32_t get_byte(const uint32_t w[4], int q) { return (w[q >> 2] >> (8 * (q & 3))) & 0xffu; }

// Highest non-zero byte index (< valid) of a raw block, or -1.
__device__ __forceinline__ int last_nonzero(const uint32_t w[4], int valid) {
  int r = -1;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    uint32_t x = w[i];
    const int lo = 4 * i;
    if (valid < lo + 4) x &= (valid <= lo) ? 0u : (0xffffffffu >> (8 * (lo + 4 - valid)));
    if (x) r = lo + (31 - __builtin_clz(x)) / 8;
  }
  return r;
}

// Content-type scan of one whole 16-byte plaintext block at byte offset off (record.rs:229-237):
// (off + i) << 8 | byte for its last non-zero byte i, or prev when the block is all zero. Selects
// only (no branch, no indexed register access), so it stays in the fast step's basic block.
__device__ __forceinline__ int64_t block_last_nz(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, uint32_t off,
                                                 int64_t prev) {
  const uint32_t x = w3 ? w3 : w2 ? w2 : w1 ? w1 : w0;
  const uint32_t wi = w3 ? 12u : w2 ? 8u : w1 ? 4u : 0u;
  const uint32_t bi = (31u - (uint32_t)__builtin_clz(x | 1u)) >> 3;  // x != 0 whenever it is used
  const int64_t v = ((int64_t)(off + wi + bi) << 8) | ((x >> (8u * bi)) & 0xffu);
  return x ? v : prev;
}

struct GcmArgs {
  const KeySched* ks;
  const atls_rec* recs;
  uint32_t n;
  const uint8_t* in;
  const uint8_t* aux;
  uint8_t* out;
  uint8_t* tags_out;       // seal
  const uint8_t* tags_in;  // open
  atls_open_result* res;   // open
  const uint32_t* t0;      // 256-entry T-table in global memory
  const uint32_t* idx;     // batch plan (plan.hip): record indices per work list; nullptr: direct
  PlanHdr* plan;
  uint32_t* err;           // direct mode: sticky error word
  uint32_t n_slots;        // direct mode: key-table size
  const uint32_t* gidx;    // direct mode: key groups (plan.hip atls_launch_group), or nullptr
  GroupHdr* ghdr;          // their region sizes and work counters
  uint32_t* done;          // one-record direct launch (the single call): set to done_val when the
  uint32_t done_val;       // record's outputs are visible system-wide (mapped host memory), or nullptr
  uint8_t* tail;           // batch launches: workspace of the deferred last steps (gcm.hip gcm_tail_kernel), or nullptr
};

// The single call's completion flag: after the wave's own stores have left (system-scope release),
// one lane stores done_val into the caller's mapped host memory, where the host spins on it instead
// of waiting for the launch's completion signal (tools/single_call_floor: 6.5 vs 11.9 us).
__device__ __forceinline__ void signal_done(uint32_t* done, uint32_t val, int lane) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // MI355X_MICROARCH.md: the compiler may drop it
  if (lane == 0) __hip_atomic_store(done, val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Open result for one record (record.rs:203-240 decrypt + padding scan). lastnz = (position <<
// 8 | byte) of the last non-zero plaintext byte, -1 if none.
__device__ __forceinline__ void write_open_result(const GcmArgs& A, uint32_t rec_idx, bool tls, uint32_t len, bool ok,
                                                  int64_t lastnz, bool hdr_ok) {
  atls_open_result r;
  r.reserved[0] = r.reserved[1] = 0;
  if (!hdr_ok) {  // WIRE: the header does not frame this record (record.rs:81-102)
    r.status = ATLS_DECODE_ERROR;
    r.content_len = 0;
    r.content_type = 0;
  } else if (!tls) {
    r.status = ok ? ATLS_OK : ATLS_BAD_RECORD_MAC;
    r.content_len = len;
    r.content_type = 0;
  } else if (!ok) {
    r.status = ATLS_DECRYPT_ERROR;
    r.content_len = 0;
    r.content_type = 0;
  } else {
    const uint32_t ty = lastnz >= 0 ? (uint32_t)(lastnz & 0xff) : 0u;
    const bool valid_type = ty == 0 || ty == 20 || ty == 21 || ty == 22 || ty == 23;
    r.status = valid_type ? ATLS_OK : ATLS_DECODE_ERROR;
    r.content_len = (valid_type && lastnz >= 0) ? (uint32_t)(lastnz >> 8) : 0u;
    r.content_type = valid_type ? (uint8_t)ty : 0;
  }
  A.res[rec_idx] = r;
}

}  // namespace atls
