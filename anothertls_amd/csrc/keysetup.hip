// Device key setup: one thread per key slot (a connection's write key). Everything the
// record kernels need per key is computed here once, instead of per record as the
// reference does (gcm.rs:52-56 re-expands the key and recomputes H on every call):
//   * AES round keys (crypto/aes/cipher.rs:216-249) as raw words for the T-table rounds;
//   * H = E_K(0^128) (gcm.rs:56), H^1..H^64 (lane-combine multipliers), and
//     x^(4p)*H^64 and x^(4p)*H^32 for p = 0..31 (seeds of the per-record 4-bit GHASH tables);
//   * ChaCha20 key words (chacha20/cipher.rs:29-31).
// Also builds the 256-entry AES T-table T0 used (replicated per LDS bank) by gcm.hip.
#include "atls_dev.h"

namespace atls {

// FIPS-197 S-box (the same table as crypto/aes/cipher.rs:7-138).
static __constant__ const uint8_t kSbox[256] = {
    0x63, 0x7c, 0x77, 0x7b, 0xf2, 0x6b, 0x6f, 0xc5, 0x30, 0x01, 0x67, 0x2b, 0xfe, 0xd7, 0xab, 0x76,
    0xca, 0x82, 0xc9, 0x7d, 0xfa, 0x59, 0x47, 0xf0, 0xad, 0xd4, 0xa2, 0xaf, 0x9c, 0xa4, 0x72, 0xc0,
    0xb7, 0xfd, 0x93, 0x26, 0x36, 0x3f, 0xf7, 0xcc, 0x34, 0xa5, 0xe5, 0xf1, 0x71, 0xd8, 0x31, 0x15,
    0x04, 0xc7, 0x23, 0xc3, 0x18, 0x96, 0x05, 0x9a, 0x07, 0x12, 0x80, 0xe2, 0xeb, 0x27, 0xb2, 0x75,
    0x09, 0x83, 0x2c, 0x1a, 0x1b, 0x6e, 0x5a, 0xa0, 0x52, 0x3b, 0xd6, 0xb3, 0x29, 0xe3, 0x2f, 0x84,
    0x53, 0xd1, 0x00, 0xed, 0x20, 0xfc, 0xb1, 0x5b, 0x6a, 0xcb, 0xbe, 0x39, 0x4a, 0x4c, 0x58, 0xcf,
    0xd0, 0xef, 0xaa, 0xfb, 0x43, 0x4d, 0x33, 0x85, 0x45, 0xf9, 0x02, 0x7f, 0x50, 0x3c, 0x9f, 0xa8,
    0x51, 0xa3, 0x40, 0x8f, 0x92, 0x9d, 0x38, 0xf5, 0xbc, 0xb6, 0xda, 0x21, 0x10, 0xff, 0xf3, 0xd2,
    0xcd, 0x0c, 0x13, 0xec, 0x5f, 0x97, 0x44, 0x17, 0xc4, 0xa7, 0x7e, 0x3d, 0x64, 0x5d, 0x19, 0x73,
    0x60, 0x81, 0x4f, 0xdc, 0x22, 0x2a, 0x90, 0x88, 0x46, 0xee, 0xb8, 0x14, 0xde, 0x5e, 0x0b, 0xdb,
    0xe0, 0x32, 0x3a, 0x0a, 0x49, 0x06, 0x24, 0x5c, 0xc2, 0xd3, 0xac, 0x62, 0x91, 0x95, 0xe4, 0x79,
    0xe7, 0xc8, 0x37, 0x6d, 0x8d, 0xd5, 0x4e, 0xa9, 0x6c, 0x56, 0xf4, 0xea, 0x65, 0x7a, 0xae, 0x08,
    0xba, 0x78, 0x25, 0x2e, 0x1c, 0xa6, 0xb4, 0xc6, 0xe8, 0xdd, 0x74, 0x1f, 0x4b, 0xbd, 0x8b, 0x8a,
    0x70, 0x3e, 0xb5, 0x66, 0x48, 0x03, 0xf6, 0x0e, 0x61, 0x35, 0x57, 0xb9, 0x86, 0xc1, 0x1d, 0x9e,
    0xe1, 0xf8, 0x98, 0x11, 0x69, 0xd9, 0x8e, 0x94, 0x9b, 0x1e, 0x87, 0xe9, 0xce, 0x55, 0x28, 0xdf,
    0x8c, 0xa1, 0x89, 0x0d, 0xbf, 0xe6, 0x42, 0x68, 0x41, 0x99, 0x2d, 0x0f, 0xb0, 0x54, 0xbb, 0x16,
};

__device__ inline uint8_t xtime(uint8_t a) { return (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0)); }

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
  // p4[j] = x^(4j) * H^64
  uint32_t v[4] = {o->hpow_be[63][0], o->hpow_be[63][1], o->hpow_be[63][2], o->hpow_be[63][3]};
  for (int j = 0; j < 32; j++) {
    for (int w = 0; w < 4; w++) o->p4_be[j][w] = v[w];
    gf_mulx_be(v); gf_mulx_be(v); gf_mulx_be(v); gf_mulx_be(v);
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
