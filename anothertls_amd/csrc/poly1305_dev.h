// Poly1305 arithmetic for the ChaCha20-Poly1305 kernels (chacha.hip) and the resident single-call server
// (gcm.hip): p = 2^130 - 5 in five 26-bit limbs, products as 64-bit column sums (v_mad_u64_u32),
// poly1305.rs:19-50 (RFC 8439 §2.5).
#pragma once
#include "plan.h"

namespace atls {

constexpr uint32_t M26 = 0x3ffffffu;

struct P130 { uint32_t l[5]; };

__device__ __forceinline__ P130 p_zero() { P130 z; for (int i = 0; i < 5; i++) z.l[i] = 0; return z; }

// d += h * r (unreduced 64-bit column sums; 2^130 = 5 mod p folds the high columns back with 5 r).
__device__ __forceinline__ void p_mac(uint64_t (&d)[5], const P130& h, const P130& r) {
  const uint32_t s1 = r.l[1] * 5, s2 = r.l[2] * 5, s3 = r.l[3] * 5, s4 = r.l[4] * 5;
  const uint64_t h0 = h.l[0], h1 = h.l[1], h2 = h.l[2], h3 = h.l[3], h4 = h.l[4];
  d[0] += h0 * r.l[0] + h1 * s4 + h2 * s3 + h3 * s2 + h4 * s1;
  d[1] += h0 * r.l[1] + h1 * r.l[0] + h2 * s4 + h3 * s3 + h4 * s2;
  d[2] += h0 * r.l[2] + h1 * r.l[1] + h2 * r.l[0] + h3 * s4 + h4 * s3;
  d[3] += h0 * r.l[3] + h1 * r.l[2] + h2 * r.l[1] + h3 * r.l[0] + h4 * s4;
  d[4] += h0 * r.l[4] + h1 * r.l[3] + h2 * r.l[2] + h3 * r.l[1] + h4 * r.l[0];
}

// Column sums -> limbs (< 2^26, limb 1 < 2^26 + 2^8). The top carry times 5 is formed in 64 bits: with
// up to four products summed (p_sop4) the carry out of column 4 reaches 2^31.
__device__ __forceinline__ P130 p_red(uint64_t (&d)[5]) {
  P130 o;
  uint64_t c;
  c = d[0] >> 26; o.l[0] = (uint32_t)d[0] & M26; d[1] += c;
  c = d[1] >> 26; o.l[1] = (uint32_t)d[1] & M26; d[2] += c;
  c = d[2] >> 26; o.l[2] = (uint32_t)d[2] & M26; d[3] += c;
  c = d[3] >> 26; o.l[3] = (uint32_t)d[3] & M26; d[4] += c;
  c = d[4] >> 26; o.l[4] = (uint32_t)d[4] & M26;
  const uint64_t t = c * 5u + o.l[0];
  o.l[0] = (uint32_t)t & M26;
  o.l[1] += (uint32_t)(t >> 26);
  return o;
}

// h * r mod p, partially reduced (limbs < 2^26 + small). Inputs: limbs < 2^27.
__device__ __forceinline__ P130 p_mul(const P130& h, const P130& r) {
  uint64_t d[5] = {0, 0, 0, 0, 0};
  p_mac(d, h, r);
  return p_red(d);
}

// Add a full 16-byte block (raw LE words) plus 2^128 (poly1305.rs:39-43).
__device__ __forceinline__ void p_add_block(P130& h, uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3) {
  h.l[0] += w0 & M26;
  h.l[1] += ((w0 >> 26) | (w1 << 6)) & M26;
  h.l[2] += ((w1 >> 20) | (w2 << 12)) & M26;
  h.l[3] += ((w2 >> 14) | (w3 << 18)) & M26;
  h.l[4] += (w3 >> 8) | (1u << 24);
}

__device__ __forceinline__ void p_add(P130& a, const P130& b) { for (int i = 0; i < 5; i++) a.l[i] += b.l[i]; }

// A full data slot's MAC in one reduction (SOP): acc' = acc r^(4G) + c0 r^3 + c1 r^2 + c2 r + c3, the
// four products summed as 64-bit column sums before one carry chain, instead of three Horner steps and
// the slot step, each reduced (four carry chains). Column sums stay below 2^59 (p_red). The acc product
// goes last so the data words die as they are folded. Same-box A/B over 3 rounds
// (profiles/r03/ab_c3_w2.log): C3 seal kernel 0.0878 -> 0.0840 ms; with the acc product first it spilled
// 19 VGPRs and measured 12 % slower (profiles/r03/ab_c3_sop_rot16.log).
__device__ __forceinline__ void p_sop4(P130& acc, bool first, const P130& rG, const uint32_t (&X)[16],
                                       const P130& r, const P130& rsq, const P130& rcu) {
  uint64_t d[5];
  P130 c = p_zero();
  p_add_block(c, X[12], X[13], X[14], X[15]);
  for (int i = 0; i < 5; i++) d[i] = c.l[i];
  c = p_zero();
  p_add_block(c, X[0], X[1], X[2], X[3]);
  p_mac(d, c, rcu);
  c = p_zero();
  p_add_block(c, X[4], X[5], X[6], X[7]);
  p_mac(d, c, rsq);
  c = p_zero();
  p_add_block(c, X[8], X[9], X[10], X[11]);
  p_mac(d, c, r);
  if (!first) p_mac(d, acc, rG);
  acc = p_red(d);
}

__device__ __forceinline__ void p_carry(P130& h) {
  uint32_t c;
  c = h.l[0] >> 26; h.l[0] &= M26; h.l[1] += c;
  c = h.l[1] >> 26; h.l[1] &= M26; h.l[2] += c;
  c = h.l[2] >> 26; h.l[2] &= M26; h.l[3] += c;
  c = h.l[3] >> 26; h.l[3] &= M26; h.l[4] += c;
  c = h.l[4] >> 26; h.l[4] &= M26; h.l[0] += c * 5;
  c = h.l[0] >> 26; h.l[0] &= M26; h.l[1] += c;
}

// tag = ((h mod p) + s) mod 2^128 as raw words (poly1305.rs:46-50).
__device__ __forceinline__ void p_finish(P130 h, const uint32_t s[4], uint32_t t[4]) {
  p_carry(h);
  p_carry(h);
  uint32_t g0 = h.l[0] + 5, c = g0 >> 26; g0 &= M26;
  uint32_t g1 = h.l[1] + c; c = g1 >> 26; g1 &= M26;
  uint32_t g2 = h.l[2] + c; c = g2 >> 26; g2 &= M26;
  uint32_t g3 = h.l[3] + c; c = g3 >> 26; g3 &= M26;
  uint32_t g4 = h.l[4] + c - (1u << 26);
  uint32_t mask = (g4 >> 31) - 1u;  // all ones if h >= p
  uint32_t h0 = (h.l[0] & ~mask) | (g0 & mask), h1 = (h.l[1] & ~mask) | (g1 & mask);
  uint32_t h2 = (h.l[2] & ~mask) | (g2 & mask), h3 = (h.l[3] & ~mask) | (g3 & mask);
  uint32_t h4 = (h.l[4] & ~mask) | (g4 & mask);
  uint32_t w0 = h0 | (h1 << 26), w1 = (h1 >> 6) | (h2 << 20), w2 = (h2 >> 12) | (h3 << 14), w3 = (h3 >> 18) | (h4 << 8);
  uint64_t f = (uint64_t)w0 + s[0]; t[0] = (uint32_t)f;
  f = (uint64_t)w1 + s[1] + (f >> 32); t[1] = (uint32_t)f;
  f = (uint64_t)w2 + s[2] + (f >> 32); t[2] = (uint32_t)f;
  f = (uint64_t)w3 + s[3] + (f >> 32); t[3] = (uint32_t)f;
}

template <int G>
__device__ __forceinline__ P130 shfl_p(const P130& v, int src) {
  P130 o;
  for (int i = 0; i < 5; i++) o.l[i] = __shfl(v.l[i], src, G);
  return o;
}

}  // namespace atls
