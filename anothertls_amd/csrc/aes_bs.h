// Bitsliced AES for gfx950: 32 blocks per lane, one bit of each block per bit of a 32-bit
// plane, AES rounds as v_bitop3_b32 / v_perm_b32 logic on the VALU (no table lookups).
//
// State: pl[i][j] = plane of state byte i (i = 4*column + row, FIPS-197 order), bit (7 - j):
// j = 0 is the byte's most significant bit (the S-box circuit's U0). Bit k of every plane is
// block k. Round keys enter as the raw little-endian words of the 16 round-key bytes (the
// layout of KeySched::rk, crypto/aes/cipher.rs:216-249 expanded_key); each key bit becomes an
// all-zeros / all-ones plane mask (Key1: one key per lane; Key2: two keys, one per 16 blocks).
//
// Host-compilable (tests/test_aes_bs_emulation.py runs it on the CPU with software versions of
// __builtin_amdgcn_bitop3_b32 and __builtin_amdgcn_perm).
#pragma once
#include <stdint.h>

#include "sbox_bs.h"

// Scheduling fence: keeps the machine scheduler from interleaving independent S-boxes /
// columns, which multiplies live temporaries past the 256-VGPR budget of two waves per SIMD.
#if defined(__HIP_DEVICE_COMPILE__) && defined(ATLS_BS_FENCES)
#define ATLS_BS_FENCE() __builtin_amdgcn_sched_barrier(0)
#else
#define ATLS_BS_FENCE() ((void)0)
#endif

namespace atls_bs {

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
// bit `b` of w -> 0 or 0xffffffff
__device__ __forceinline__ uint32_t bmask(uint32_t w, int b) { return (uint32_t)((int32_t)(w << (31 - b)) >> 31); }

// Round-key masks. Key1: one key for all 32 blocks of the lane. Key2: key `a` for blocks 0-15
// (plane bits 0-15), key `b` for blocks 16-31 -- when a and b are wave-uniform the masks are
// scalar (SALU) values and every AddRoundKey XOR folds into a VALU op's SGPR operand.
struct Key1 {
  uint32_t w[4];
  __device__ __forceinline__ uint32_t mask(int c, int bit) const { return bmask(w[c], bit); }
};
struct Key2 {
  uint32_t a[4], b[4];
  __device__ __forceinline__ uint32_t mask(int c, int bit) const {
    return (bmask(a[c], bit) & 0x0000ffffu) | (bmask(b[c], bit) << 16);  // s_pack_ll_b32_b16
  }
};

__device__ __forceinline__ void sub_bytes(uint32_t (&pl)[16][8]) {
#pragma unroll
  for (int i = 0; i < 16; i++) {
    sbox_bs(pl[i]);
    ATLS_BS_FENCE();
  }
}

// ShiftRows + MixColumns + AddRoundKey. rk[c] = raw word of round-key column c (byte r = row r).
// out_r = xtime(a_r ^ a_{r+1}) ^ a_{r+1} ^ a_{r+2} ^ a_{r+3} (+ key), a_r = ShiftRows input
// byte (row r, column c + r). Planes are MSB-first: significance t lives at index 7 - t.
template <class KM>
__device__ __forceinline__ void shift_mix_ark(uint32_t (&pl)[16][8], const KM& km) {
  uint32_t o[16][8];
#pragma unroll
  for (int c = 0; c < 4; c++) {
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const uint32_t* a0 = pl[4 * ((c + r) & 3) + r];
      const uint32_t* a1 = pl[4 * ((c + r + 1) & 3) + ((r + 1) & 3)];
      const uint32_t* a2 = pl[4 * ((c + r + 2) & 3) + ((r + 2) & 3)];
      const uint32_t* a3 = pl[4 * ((c + r + 3) & 3) + ((r + 3) & 3)];
      uint32_t u[8], v[8];  // indexed by significance t
#pragma unroll
      for (int t = 0; t < 8; t++) {
        u[t] = a0[7 - t] ^ a1[7 - t];
        v[t] = xor3(a1[7 - t], a2[7 - t], a3[7 - t]);
      }
#pragma unroll
      for (int t = 0; t < 8; t++) {
        const uint32_t k = km.mask(c, 8 * r + t);
        uint32_t x;
        if (t == 0) x = xor3(v[0], u[7], k);
        else if (t == 1 || t == 3 || t == 4) x = xor3(xor3(v[t], u[t - 1], u[7]), k, 0u);
        else x = xor3(v[t], u[t - 1], k);
        o[4 * c + r][7 - t] = x;
      }
    }
    ATLS_BS_FENCE();
  }
#pragma unroll
  for (int i = 0; i < 16; i++)
#pragma unroll
    for (int j = 0; j < 8; j++) pl[i][j] = o[i][j];
}

// Final round: ShiftRows + AddRoundKey (no MixColumns).
template <class KM>
__device__ __forceinline__ void shift_ark(uint32_t (&pl)[16][8], const KM& km) {
  uint32_t o[16][8];
#pragma unroll
  for (int c = 0; c < 4; c++)
#pragma unroll
    for (int r = 0; r < 4; r++)
#pragma unroll
      for (int j = 0; j < 8; j++) o[4 * c + r][j] = pl[4 * ((c + r) & 3) + r][j] ^ km.mask(c, 8 * r + 7 - j);
  ATLS_BS_FENCE();
#pragma unroll
  for (int i = 0; i < 16; i++)
#pragma unroll
    for (int j = 0; j < 8; j++) pl[i][j] = o[i][j];
}

template <class KM>
__device__ __forceinline__ void add_round_key(uint32_t (&pl)[16][8], const KM& km) {
#pragma unroll
  for (int i = 0; i < 16; i++)
#pragma unroll
    for (int j = 0; j < 8; j++) pl[i][j] ^= km.mask(i >> 2, 8 * (i & 3) + 7 - j);
}

// Rows i and i + S (i & S == 0) exchange the bit columns selected by ~m and m respectively.
template <int S>
__device__ __forceinline__ void delta_swaps(uint32_t (&x)[32], uint32_t m) {
#pragma unroll
  for (int blk = 0; blk < 32; blk += 2 * S)
#pragma unroll
    for (int i = 0; i < S; i++) {
      const uint32_t a = x[blk + i], b = x[blk + i + S];
      const uint32_t t = ((a >> S) ^ b) & m;
      x[blk + i + S] = b ^ t;
      x[blk + i] = a ^ (t << S);
    }
}

// 32x32 bit transpose: afterwards bit r of x[c] = old bit c of x[r]. Stages 16 and 8 are byte
// moves (v_perm_b32), stages 4, 2, 1 are masked delta swaps.
__device__ __forceinline__ void transpose32(uint32_t (&x)[32]) {
#pragma unroll
  for (int i = 0; i < 16; i++) {  // swap 16-bit halves: rows i and i + 16
    const uint32_t a = x[i], b = x[i + 16];
    x[i] = __builtin_amdgcn_perm(b, a, 0x05040100u);       // {a.lo16, b.lo16}
    x[i + 16] = __builtin_amdgcn_perm(b, a, 0x07060302u);  // {a.hi16, b.hi16}
  }
#pragma unroll
  for (int blk = 0; blk < 32; blk += 16)
#pragma unroll
    for (int i = 0; i < 8; i++) {  // swap bytes: rows i and i + 8
      const uint32_t a = x[blk + i], b = x[blk + i + 8];
      x[blk + i] = __builtin_amdgcn_perm(b, a, 0x06020400u);      // {a.b0, b.b0, a.b2, b.b2}
      x[blk + i + 8] = __builtin_amdgcn_perm(b, a, 0x07030501u);  // {a.b1, b.b1, a.b3, b.b3}
    }
  delta_swaps<4>(x, 0x0f0f0f0fu);
  delta_swaps<2>(x, 0x33333333u);
  delta_swaps<1>(x, 0x55555555u);
}

// Planes -> 32 blocks: blk[w][k] = raw word w (bytes 4w..4w+3, little-endian) of block k.
// Group w's 32 rows are ordered p = 8*byte_in_word + significance, so after the transpose row k
// holds word w of block k. The result overwrites pl (viewed as 4 x 32 words).
__device__ __forceinline__ void planes_to_blocks(uint32_t (&pl)[16][8], uint32_t (&blk)[4][32]) {
#pragma unroll
  for (int w = 0; w < 4; w++) {
    uint32_t x[32];
#pragma unroll
    for (int b = 0; b < 4; b++)
#pragma unroll
      for (int t = 0; t < 8; t++) x[8 * b + t] = pl[4 * w + b][7 - t];
    transpose32(x);
#pragma unroll
    for (int k = 0; k < 32; k++) blk[w][k] = x[k];
    ATLS_BS_FENCE();
  }
}

}  // namespace atls_bs
