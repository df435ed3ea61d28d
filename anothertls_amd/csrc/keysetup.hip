// Device key setup: one thread per key slot (a connection's write key). Everything the
// record kernels need per key is computed here once, instead of per record as the
// reference does (gcm.rs:52-56 re-expands the key and recomputes H on every call):
//   * AES round keys (crypto/aes/cipher.rs:216-249) as raw words for the T-table rounds;
//   * H = E_K(0^128) (gcm.rs:56), H^1..H^64 (lane-combine multipliers), and
//     x^(4p)*H^64 and x^(4p)*H^32 for p = 0..31 (seeds of the per-record 4-bit GHASH tables);
//   * ChaCha20 key words (chacha20/cipher.rs:29-31).
// Also builds the 256-entry AES T-table T0 used (replicated per LDS bank) by gcm.hip.
#include "aes_sbox.h"
#include "atls_dev.h"

namespace atls {

// T0[x] = {2S, S, S, 3S} little-endian: MixColumns column of S[x] entering at row 0.
__global__ void build_t0_kernel(uint32_t* __restrict__ t0) {
  int x = threadIdx.x;
  uint8_t s = kSbox[x], s2 = xtime(s), s3 = (uint8_t)(s2 ^ s);
  t0[x] = (uint32_t)s2 | ((uint32_t)s << 8) | ((uint32_t)s << 16) | ((uint32_t)s3 << 24);
}

// Byte-oriented AES block encryption for setup only (one block per key: H).
__device__ void aes_encrypt_bytes(const uint8_t* ek, int nr, const uint8_t in[16], uint8_t out[16]) {
  uint8_t s[16];
  for (int i = 0; i < 16; i++) s[i] = in[i] ^ ek[i];
  for (int r = 1; r <= nr; r++) {
    uint8_t t[16];
    for (int c = 0; c < 4; c++)
      for (int row = 0; row < 4; row++) t[4 * c + row] = kSbox[s[4 * ((c + row) & 3) + row]];
    if (r < nr) {
      for (int c = 0; c < 4; c++) {
        uint8_t a0 = t[4 * c], a1 = t[4 * c + 1], a2 = t[4 * c + 2], a3 = t[4 * c + 3];
        uint8_t x = a0 ^ a1 ^ a2 ^ a3;
        t[4 * c] = a0 ^ x ^ xtime(a0 ^ a1);
        t[4 * c + 1] = a1 ^ x ^ xtime(a1 ^ a2);
        t[4 * c + 2] = a2 ^ x ^ xtime(a2 ^ a3);
        t[4 * c + 3] = a3 ^ x ^ xtime(a3 ^ a0);
      }
    }
    for (int i = 0; i < 16; i++) s[i] = t[i] ^ ek[16 * r + i];
  }
  for (int i = 0; i < 16; i++) out[i] = s[i];
}

__global__ void key_setup_kernel(const atls_key* __restrict__ keys, uint32_t n, KeySched* __restrict__ ks) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const atls_key k = keys[i];
  KeySched* o = &ks[i];
  o->suite = k.suite;
  o->key_len = k.key_len;
  o->nr = 0;
  o->valid = 0;
  for (int w = 0; w < 3; w++)
    o->siv[w] = (uint32_t)k.static_iv[4 * w] | ((uint32_t)k.static_iv[4 * w + 1] << 8) |
                ((uint32_t)k.static_iv[4 * w + 2] << 16) | ((uint32_t)k.static_iv[4 * w + 3] << 24);
  o->siv[3] = 0;
  for (int w = 0; w < 8; w++)
    o->kw[w] = (uint32_t)k.key[4 * w] | ((uint32_t)k.key[4 * w + 1] << 8) | ((uint32_t)k.key[4 * w + 2] << 16) |
               ((uint32_t)k.key[4 * w + 3] << 24);
  if (k.suite == kSuiteChacha) {
    o->valid = (k.key_len == 32) ? 1u : 0u;
    return;
  }
  if (k.suite != kSuiteAes128 && k.suite != kSuiteAes256) return;
  if (k.key_len != 16 && k.key_len != 24 && k.key_len != 32) return;  // gcm.rs:49 Blocksize::new
  // FIPS-197 key expansion, crypto/aes/cipher.rs:216-249.
  const int nk = k.key_len / 4, nr = nk + 6;
  uint8_t ek[240];
  const uint8_t rcon[10] = {0x01, 0x02, 0x04, 0x08, 0x10, 0x20, 0x40, 0x80, 0x1B, 0x36};
  for (int j = 0; j < 4 * nk; j++) ek[j] = k.key[j];
  for (int w = nk; w < 4 * (nr + 1); w++) {
    uint8_t t[4] = {ek[4 * (w - 1)], ek[4 * (w - 1) + 1], ek[4 * (w - 1) + 2], ek[4 * (w - 1) + 3]};
    if (w % nk == 0) {
      uint8_t t0 = t[0];
      t[0] = kSbox[t[1]] ^ rcon[w / nk - 1];
      t[1] = kSbox[t[2]];
      t[2] = kSbox[t[3]];
      t[3] = kSbox[t0];
    } else if (nk > 6 && w % nk == 4) {
      for (int b = 0; b < 4; b++) t[b] = kSbox[t[b]];
    }
    for (int b = 0; b < 4; b++) ek[4 * w + b] = ek[4 * (w - nk) + b] ^ t[b];
  }
  for (int w = 0; w < 60; w++)
    o->rk[w] = w < 4 * (nr + 1) ? ((uint32_t)ek[4 * w] | ((uint32_t)ek[4 * w + 1] << 8) |
                                   ((uint32_t)ek[4 * w + 2] << 16) | ((uint32_t)ek[4 * w + 3] << 24))
                                : 0u;
  for (int w = 0; w < 60; w++) o->rkr[w] = (o->rk[w] << 16) | (o->rk[w] >> 16);
  o->nr = (uint32_t)nr;
  // H = E_K(0) (gcm.rs:56) and its powers.
  uint8_t zero[16] = {0}, hb[16];
  aes_encrypt_bytes(ek, nr, zero, hb);
  uint32_t h[4];
  for (int w = 0; w < 4; w++)
    h[w] = ((uint32_t)hb[4 * w] << 24) | ((uint32_t)hb[4 * w + 1] << 16) | ((uint32_t)hb[4 * w + 2] << 8) | hb[4 * w + 3];
  for (int w = 0; w < 4; w++) o->h_be[w] = h[w];
  uint32_t p[4] = {h[0], h[1], h[2], h[3]};
  for (int e = 0; e < 64; e++) {
    for (int w = 0; w < 4; w++) o->hpow_be[e][w] = p[w];
    uint32_t q[4];
    gf_mul_be(p, h, q);
    for (int w = 0; w < 4; w++) p[w] = q[w];
  }
  // p4[j] = x^(4j) * H^64; p4g[t][j] = x^(4j) * H^(8 << t) (records processed in lane groups)
  uint32_t v[4] = {o->hpow_be[63][0], o->hpow_be[63][1], o->hpow_be[63][2], o->hpow_be[63][3]};
  for (int j = 0; j < 32; j++) {
    for (int w = 0; w < 4; w++) o->p4_be[j][w] = v[w];
    gf_mulx_be(v); gf_mulx_be(v); gf_mulx_be(v); gf_mulx_be(v);
  }
  for (int t = 0; t < 3; t++) {
    for (int w = 0; w < 4; w++) v[w] = o->hpow_be[(8 << t) - 1][w];
    for (int j = 0; j < 32; j++) {
      for (int w = 0; w < 4; w++) o->p4g_be[t][j][w] = v[w];
      gf_mulx_be(v); gf_mulx_be(v); gf_mulx_be(v); gf_mulx_be(v);
    }
  }
  o->valid = 1;
}

}  // namespace atls

extern "C" int atls_launch_build_t0(uint32_t* t0, hipStream_t s) {
  hipLaunchKernelGGL(atls::build_t0_kernel, dim3(1), dim3(256), 0, s, t0);
  return hipGetLastError() == hipSuccess ? 0 : ATLS_INTERNAL_ERROR;
}

extern "C" int atls_launch_key_setup(const atls_key* keys, uint32_t n, void* ks, hipStream_t s) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(atls::key_setup_kernel, dim3((n + 63) / 64), dim3(64), 0, s, keys, n,
                     (atls::KeySched*)ks);
  return hipGetLastError() == hipSuccess ? 0 : ATLS_INTERNAL_ERROR;
}
