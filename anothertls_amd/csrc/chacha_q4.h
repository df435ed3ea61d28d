// The one-record ChaCha20-Poly1305 of the single call on a 256-thread workgroup (q4_record), shared by
// chacha.hip (chacha_single_q4) and the resident single-call server (gcm.hip single_resident).
#pragma once
#include "poly1305_dev.h"

namespace atls {

// ---- The single call at four lanes per ChaCha20 block (round 5) ----------------------------
// chacha_single (64 lanes) runs a record's ChaCha20 blocks one per lane -- a 1,537-B record's 26 blocks each
// ~1,300 VALU slots deep on one lane, the four columns as instruction-level parallelism of one wave -- and its
// Poly1305 pieces four per lane (slot Horner, r-power scan, lane combine). Here a 4-wave workgroup gives each
// block a quad of lanes, one state column per lane (the diagonal round takes its b, c, d words from the
// quad's other lanes by DPP quad_perm and hands them back after), so the keystream is ~300 dependent slots
// deep; and each Poly1305 message block gets a thread of its own: thread t holds block t of
// AAD || pad || ciphertext || pad || lengths (poly1305.rs:57-66) and adds m_t r^(Q-t) (the Horner sum
// a = sum m_t r^(Q-t), poly1305.rs:32-45), r^k read from entry k-1 of a 256-thread prefix-product scan.
// Records whose argument block fits (kSingleInline): at most 56 data blocks + the key block (64 quads) and
// Q <= 226 message blocks (256 threads).
#ifndef ATLS_CHACHA_SINGLE_Q4
#define ATLS_CHACHA_SINGLE_Q4 1
#endif
template <int CTRL>
__device__ __forceinline__ uint32_t qperm(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xf, 0xf, false);  // quad_perm
}
#define QRL(a, b, c, d)                     \
  a += b; d = rotl32(d ^ a, 16);            \
  c += d; b = rotl32(b ^ c, 12);            \
  a += b; d = rotl32(d ^ a, 8);             \
  c += d; b = rotl32(b ^ c, 7);

// One RAW record (the Cipher-trait call) by the 256 threads of the workgroup: k its key slot, bytes the
// base d.aux_off / d.in_off index (IV || AAD || input; the received tag at bytes + tag_off on open), outputs
// at out + d.out_off, the tag at tag_out, the open result at *res. The caller releases the stores.
// q4_record's LDS (the caller's: a static array of the single-call kernel, or a piece of the resident server's
// dynamic LDS, whose AES-GCM tables must start at LDS address 0)
struct Q4Lds {
  uint32_t ctw[64 * 16];  // MAC input words (ciphertext, zero past the end)
  uint32_t pw[256][5];    // r^(k+1) at k
  uint32_t rs[8];         // r, s (poly1305.rs:19-26)
  uint32_t part[4][5];
};

template <bool OPEN>
__device__ __forceinline__ void q4_record(const KeySched* k, const atls_rec& d, const uint8_t* bytes, uint32_t tag_off,
                                          uint8_t* out, uint8_t* tag_out, atls_open_result* res, Q4Lds& L) {
  const int t = (int)threadIdx.x, q = t & 3, lane = t & 63, wv = t >> 6;
  const uint32_t blk = (uint32_t)t >> 2;  // ChaCha20 block counter of this quad (0 = Poly1305 key)
  uint32_t* ctw = L.ctw;
  uint32_t(*pw)[5] = L.pw;
  uint32_t* rs = L.rs;
  uint32_t(*part)[5] = L.part;
  const uint32_t n = d.len, aad_len = d.aad_len;
  const uint8_t* iv = bytes + d.aux_off;
  const uint8_t* aadp = iv + 12;
  const uint8_t* src = bytes + d.in_off;
  uint8_t* dst = out + d.out_off;
  const uint32_t na = (aad_len + 15u) / 16u, nct = (n + 15u) / 16u, jmax = (n + 63u) / 64u;
  const uint32_t Q = na + nct + 1u;
  // ---- keystream: column q of block blk (cipher.rs:56-87), every quad (those past jmax idle after) ----
  const uint32_t kq = k->kw[q], kq4 = k->kw[4 + q];
  const uint32_t nq = q ? ((uint32_t)iv[4 * q - 4] | ((uint32_t)iv[4 * q - 3] << 8) | ((uint32_t)iv[4 * q - 2] << 16) |
                           ((uint32_t)iv[4 * q - 1] << 24))
                        : blk;
  const uint32_t c0 = q == 0 ? 0x61707865u : q == 1 ? 0x3320646eu : q == 2 ? 0x79622d32u : 0x6b206574u;
  uint32_t a = c0, b = kq, c = kq4, dd = nq;
#pragma unroll
  for (int i = 0; i < 10; i++) {
    QRL(a, b, c, dd)
    b = qperm<0x39>(b); c = qperm<0x4E>(c); dd = qperm<0x93>(dd);  // diagonal: columns q+1, q+2, q+3
    QRL(a, b, c, dd)
    b = qperm<0x93>(b); c = qperm<0x4E>(c); dd = qperm<0x39>(dd);  // back to column q
  }
  const uint32_t o[4] = {a + c0, b + kq, c + kq4, dd + nq};  // words q, 4 + q, 8 + q, 12 + q of the block
  if (blk == 0 && t < 4) {
    rs[q] = o[0];
    rs[4 + q] = o[1];
  }
  // ---- XOR, store, MAC words: word 4 kk + q of data block blk (bytes 64 (blk - 1) ..) ----
  if (blk >= 1 && blk <= jmax) {
    const uint32_t off = 64u * (blk - 1u), vb = min(64u, n - off);
    const bool skip_xor = (n % 64u) == 0u && blk == jmax;  // cipher.rs:99-102
#pragma unroll
    for (int kk = 0; kk < 4; kk++) {
      const uint32_t p0 = 16u * kk + 4u * (uint32_t)q;
      uint32_t in = 0;
      if (p0 + 4u <= vb) in = ld4(src + off + p0);
      else
        for (uint32_t x = 0; x < 4u; x++)
          if (p0 + x < vb) in |= (uint32_t)src[off + p0 + x] << (8 * x);
      uint32_t ct = skip_xor ? in : in ^ o[kk];
      if (p0 + 4u > vb) ct &= p0 >= vb ? 0u : (0xffffffffu >> (8 * (p0 + 4u - vb)));
      if (p0 + 4u <= vb) st4(dst + off + p0, ct);
      else
        for (uint32_t x = 0; x < 4u; x++)
          if (p0 + x < vb) dst[off + p0 + x] = (uint8_t)(ct >> (8 * x));
      ctw[16u * (blk - 1u) + 4u * kk + (uint32_t)q] = OPEN ? in : ct;  // the MAC runs over the ciphertext
    }
  }
  __syncthreads();
  // ---- r powers: thread t holds r^(t+1) (prefix products, 6 levels per wave, then the wave's (r^64)^w) ----
  const uint32_t r0 = rs[0] & 0x0fffffffu, r1 = rs[1] & 0x0ffffffcu, r2 = rs[2] & 0x0ffffffcu, r3 = rs[3] & 0x0ffffffcu;
  const uint32_t sk[4] = {rs[4], rs[5], rs[6], rs[7]};
  P130 r;
  r.l[0] = r0 & M26;
  r.l[1] = ((r0 >> 26) | (r1 << 6)) & M26;
  r.l[2] = ((r1 >> 20) | (r2 << 12)) & M26;
  r.l[3] = ((r2 >> 14) | (r3 << 18)) & M26;
  r.l[4] = r3 >> 8;
  P130 R = r;
#pragma unroll
  for (int dl = 1; dl < 64; dl <<= 1) {
    if ((uint32_t)dl < Q) {  // uniform: powers past r^Q are not read
      P130 u;
#pragma unroll
      for (int i = 0; i < 5; i++) u.l[i] = __shfl_up(R.l[i], (unsigned)dl, 64);
      const P130 m = p_mul(R, u);
      if (lane >= dl) R = m;
    }
  }
  if (wv >= 1 && Q > 64u * (uint32_t)wv) {  // this wave's entries are r^(64 w + lane + 1)
    const P130 r64 = shfl_p<64>(R, 63);
    P130 f = r64;
    if (wv >= 2) {
      const P130 f2 = p_mul(r64, r64);
      f = wv == 2 ? f2 : p_mul(f2, r64);
    }
    R = p_mul(R, f);
  }
#pragma unroll
  for (int i = 0; i < 5; i++) pw[t][i] = R.l[i];
  __syncthreads();
  // ---- message block t times r^(Q - t), summed ----
  P130 h = p_zero();
  if ((uint32_t)t < Q) {
    uint32_t w[4] = {0, 0, 0, 0};
    if ((uint32_t)t < na) {
#pragma unroll
      for (int x = 0; x < 16; x++)
        if (16u * (uint32_t)t + (uint32_t)x < aad_len) w[x >> 2] |= (uint32_t)aadp[16 * t + x] << (8 * (x & 3));
    } else if ((uint32_t)t < na + nct) {
      const uint32_t pc = (uint32_t)t - na;
#pragma unroll
      for (int x = 0; x < 4; x++) w[x] = ctw[4u * pc + (uint32_t)x];
    } else {  // le64(aad_len) || le64(ct_len) (poly1305.rs:63-64)
      w[0] = aad_len;
      w[2] = n;
    }
    P130 m = p_zero();
    p_add_block(m, w[0], w[1], w[2], w[3]);
    const uint32_t e = Q - (uint32_t)t;  // 1 .. Q
    P130 pe;
#pragma unroll
    for (int i = 0; i < 5; i++) pe.l[i] = pw[e - 1u][i];
    h = p_mul(m, pe);
  }
  for (int off = 32; off >= 1; off >>= 1) {
    if (off == 1) p_carry(h);  // 32 partials summed: limbs < 2^31; carried before the last doubling
    P130 u;
#pragma unroll
    for (int i = 0; i < 5; i++) u.l[i] = __shfl_xor(h.l[i], off, 64);
    p_add(h, u);
  }
  if (lane == 0) {
    p_carry(h);
#pragma unroll
    for (int i = 0; i < 5; i++) part[wv][i] = h.l[i];
  }
  __syncthreads();
  if (t == 0) {
#pragma unroll
    for (int x = 1; x < 4; x++)
#pragma unroll
      for (int i = 0; i < 5; i++) h.l[i] += part[x][i];
    uint32_t tag[4];
    p_finish(h, sk, tag);
    if (!OPEN) {
      st16(tag_out, make_uint4(tag[0], tag[1], tag[2], tag[3]));
    } else {
      const uint4 tg = ld16(bytes + tag_off);
      const bool ok = (tg.x == tag[0]) & (tg.y == tag[1]) & (tg.z == tag[2]) & (tg.w == tag[3]);
      atls_open_result rr;
      rr.reserved[0] = rr.reserved[1] = 0;
      rr.status = ok ? ATLS_OK : ATLS_BAD_RECORD_MAC;  // RAW: Cipher::decrypt (poly1305.rs:91-96)
      rr.content_len = n;
      rr.content_type = 0;
      *res = rr;
    }
  }
}
#undef QRL

}  // namespace atls
