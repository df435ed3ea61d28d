// Bitsliced AES for gfx950 (tools only: the microbenchmarks and the CPU emulation tests; the product
// kernel is T-table AES): 8 G blocks per lane, AES rounds as v_bitop3_b32 / v_perm_b32 /
// v_alignbit_b32 logic on the VALU (no table lookups). Measured slower than the T-table kernel both
// as a separate keystream kernel (round 1) and as steps mixed into the record kernel (round 2).
//
// Row-plane layout: st[g][r][j], g = block group (blocks 8g..8g+7), r = state row, j = bit
// significance 7 - j (j = 0 is the MSB, the S-box circuit's U0). Bit 8c + b of a word is bit
// (7 - j) of state byte (row r, column c) -- FIPS-197 byte 4c + r -- of block 8g + b. So
//   * SubBytes is the 94-op circuit (sbox_bs.h) on the 8 words of each (g, r): 32 bytes at once;
//   * ShiftRows rotates row r's words right by 8r bits (one v_alignbit each), in place;
//   * MixColumns combines the four row words of a (g, significance) -- all columns aligned;
//   * AddRoundKey XORs 32 mask words per round (byte c of mask (r, j) = 0xFF where round-key
//     byte (r, c) has bit 7 - j), shared by the four groups; one v_perm_b32 builds a mask from
//     pre-packed key words using v_perm's sign-replicating selectors.
// The layout never renames registers, so a rolled round loop keeps its 128 state words in place.
// Round keys are the raw little-endian words of the 16 round-key bytes (KeySched::rk layout,
// crypto/aes/cipher.rs:216-249 expanded_key): word c = column c, byte r = row r.
//
// Host-compilable (tests/test_aes_bs_emulation.py runs it on the CPU with software versions of
// __builtin_amdgcn_bitop3_b32, __builtin_amdgcn_perm and __builtin_amdgcn_alignbit).
#pragma once
#include <stdint.h>

#include "sbox_bs.h"

namespace atls_bs {

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
// bit `b` of w -> 0 or 0xffffffff
__device__ __forceinline__ uint32_t bmask(uint32_t w, int b) { return (uint32_t)((int32_t)(w << (31 - b)) >> 31); }
__device__ __forceinline__ uint32_t rotr(uint32_t w, int n) { return n ? __builtin_amdgcn_alignbit(w, w, n) : w; }

template <int G>
using StateG = uint32_t[G][4][8];  // [group][row][significance 7 - j]
typedef StateG<4> State;
typedef uint32_t Masks[4][8];     // [row][significance 7 - j]

// Round-key masks from the four raw key words (or any four column words, e.g. a nonce XOR key).
// For bit p = 8r + t: S1 carries bit p of w0 / w1 at bits 15 / 31, S0 bit p of w2 / w3 at bits
// 15 / 31, and v_perm selectors 8..11 replicate exactly those four bits into bytes 0..3.
__device__ __forceinline__ void make_masks(const uint32_t (&w)[4], Masks& m) {
  const uint32_t lo01 = __builtin_amdgcn_perm(w[1], w[0], 0x05040100u);  // {w0.lo16, w1.lo16}
  const uint32_t lo23 = __builtin_amdgcn_perm(w[3], w[2], 0x05040100u);
  const uint32_t hi01 = __builtin_amdgcn_perm(w[1], w[0], 0x07060302u);  // {w0.hi16, w1.hi16}
  const uint32_t hi23 = __builtin_amdgcn_perm(w[3], w[2], 0x07060302u);
#pragma unroll
  for (int r = 0; r < 4; r++)
#pragma unroll
    for (int t = 0; t < 8; t++) {
      const int p = 8 * r + t;
      const uint32_t s1 = p < 16 ? lo01 << (15 - p) : hi01 << (31 - p);
      const uint32_t s0 = p < 16 ? lo23 << (15 - p) : hi23 << (31 - p);
      m[r][7 - t] = __builtin_amdgcn_perm(s0, s1, 0x0b0a0908u);
    }
}

template <int G>
__device__ __forceinline__ void sub_bytes(StateG<G>& st) {
#pragma unroll
  for (int g = 0; g < G; g++)
#pragma unroll
    for (int r = 0; r < 4; r++) sbox_bs(st[g][r]);
}

template <int G>
__device__ __forceinline__ void add_round_key(StateG<G>& st, const Masks& m) {
#pragma unroll
  for (int g = 0; g < G; g++)
#pragma unroll
    for (int r = 0; r < 4; r++)
#pragma unroll
      for (int j = 0; j < 8; j++) st[g][r][j] ^= m[r][j];
}

// ShiftRows + MixColumns + AddRoundKey. After ShiftRows a_r = row r of the column;
// out_r = xtime(a_r ^ a_{r+1}) ^ a_{r+1} ^ a_{r+2} ^ a_{r+3} ^ key. xtime puts bit t-1 of
// u = a_r ^ a_{r+1} at bit t and folds u's bit 7 into bits 0, 1, 3, 4 (0x1b). Significances are
// rewritten in place from 7 down to 0, so each step reads only not-yet-written lower bits; u's
// bit 7 is saved first. Temporaries: 4 + 4 words per group.
template <int G>
__device__ __forceinline__ void shift_mix_ark(StateG<G>& st, const Masks& m) {
#pragma unroll
  for (int g = 0; g < G; g++) {
    uint32_t (&a)[4][8] = st[g];  // a[r][7 - t]
#pragma unroll
    for (int r = 1; r < 4; r++)
#pragma unroll
      for (int j = 0; j < 8; j++) a[r][j] = rotr(a[r][j], 8 * r);
    uint32_t u7[4];
#pragma unroll
    for (int r = 0; r < 4; r++) u7[r] = a[r][0] ^ a[(r + 1) & 3][0];
#pragma unroll
    for (int t = 7; t >= 0; t--) {
      const int j = 7 - t;
      uint32_t o[4];
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const uint32_t v = xor3(a[(r + 1) & 3][j], a[(r + 2) & 3][j], a[(r + 3) & 3][j]);
        const uint32_t k = m[r][j];
        if (t == 0) {
          o[r] = xor3(v, u7[r], k);
        } else {
          const uint32_t u = a[r][j + 1] ^ a[(r + 1) & 3][j + 1];  // bit t - 1 of a_r ^ a_{r+1}
          o[r] = (t == 1 || t == 3 || t == 4) ? xor3(xor3(v, u, u7[r]), k, 0u) : xor3(v, u, k);
        }
      }
#pragma unroll
      for (int r = 0; r < 4; r++) a[r][j] = o[r];
    }
  }
}

// Final round: ShiftRows + AddRoundKey (no MixColumns).
template <int G>
__device__ __forceinline__ void shift_ark(StateG<G>& st, const Masks& m) {
#pragma unroll
  for (int g = 0; g < G; g++)
#pragma unroll
    for (int r = 0; r < 4; r++)
#pragma unroll
      for (int j = 0; j < 8; j++) st[g][r][j] = rotr(st[g][r][j], 8 * r) ^ m[r][j];
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

// Group g's 32 words -> its 8 blocks: rows ordered 8r + t; after the transpose x[8c + b] is raw
// word c (column c, byte r = row r) of block 8g + b.
__device__ __forceinline__ void group_to_blocks(const uint32_t (&grp)[4][8], uint32_t (&x)[32]) {
#pragma unroll
  for (int r = 0; r < 4; r++)
#pragma unroll
    for (int t = 0; t < 8; t++) x[8 * r + t] = grp[r][7 - t];
  transpose32(x);
}

// The inverse (blocks -> planes, for tests): x[8c + b] = raw word c of block 8g + b.
__device__ __forceinline__ void blocks_to_group(uint32_t (&x)[32], uint32_t (&grp)[4][8]) {
  transpose32(x);
#pragma unroll
  for (int r = 0; r < 4; r++)
#pragma unroll
    for (int t = 0; t < 8; t++) grp[r][7 - t] = x[8 * r + t];
}

}  // namespace atls_bs
