// Device-side data layout and helpers shared by the gfx950 kernels.
//
// Representation conventions (all kernels):
//  * "raw" words: the 16 bytes of a block as they sit in memory, read as 4 little-endian
//    uint32 (word i = bytes 4i..4i+3). AES state, keystream, ciphertext and the GHASH
//    accumulator live in raw words, so HBM data is never byte-swapped on the hot path.
//  * "be" words: the reference's u128 (utils/bytes.rs:110-121 to_u128_be) split into 4
//    big-endian words, w0 most significant. Used only for GF(2^128) setup math
//    (bit-serial multiply, powers of H) where the reference's bit order matters.
//    raw[i] == bswap(be[i]).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/atls.h"

namespace atls {

// Per key slot device state, built by the key-setup kernel (keysetup.hip). 3648 B, 16-B aligned.
struct alignas(16) KeySched {
  uint32_t suite, nr, key_len, valid;  // nr = AES rounds (10/12/14), 0 for ChaCha
  uint32_t rk[60];                     // AES round keys as raw words (cipher.rs:216-249 expanded_key)
  uint32_t kw[8];                      // ChaCha20 key words, little-endian (chacha20/cipher.rs:29-31)
  uint32_t siv[4];                     // static IV (12 B) as raw words + pad (key_schedule.rs:34)
  uint32_t h_be[4];                    // H = E_K(0^128) (gcm.rs:56)
  uint32_t hpow_be[64][4];             // H^(i+1), i = 0..63: lane-combine multipliers
  uint32_t p4_be[32][4];               // x^(4p) * H^64, p = 0..31: seeds of the 4-bit GHASH tables
  uint32_t rkr[60];                    // rotl16(rk[i]): the T-table rounds' key words (gcm.hip)
  uint32_t pad[4];
  uint32_t p4g_be[3][32][4];           // x^(4p) * H^(8 << t): table seeds of records in lane groups
};
static_assert(sizeof(KeySched) == 3648, "KeySched must be 3648 B");

constexpr int kSuiteAes128 = 0x1301, kSuiteAes256 = 0x1302, kSuiteChacha = 0x1303;

__host__ __device__ inline uint32_t bswap32(uint32_t x) {
  return (x >> 24) | ((x >> 8) & 0xff00u) | ((x << 8) & 0xff0000u) | (x << 24);
}
__host__ __device__ inline uint32_t rotl32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

// 16-byte global load / store at any byte address. The amdhsa ABI runs gfx9+ with unaligned
// access enabled, so these compile to one global_load/store_dwordx4 whatever the alignment:
// records at any offset (wire records put the ciphertext 5 bytes past the header) keep the
// vector path.
__device__ __forceinline__ uint4 ld16(const uint8_t* p) {
  uint4 v;
  __builtin_memcpy(&v, p, 16);
  return v;
}
__device__ __forceinline__ void st16(uint8_t* p, uint4 v) { __builtin_memcpy(p, &v, 16); }
__device__ __forceinline__ uint32_t ld4(const uint8_t* p) {
  uint32_t v;
  __builtin_memcpy(&v, p, 4);
  return v;
}
__device__ __forceinline__ void st4(uint8_t* p, uint32_t v) { __builtin_memcpy(p, &v, 4); }

// RecordType::new (net/record.rs:22-33): Invalid(0), ChangeCipherSpec, Alert, Handshake,
// ApplicationData.
__host__ __device__ inline bool record_type_ok(uint32_t b) { return b == 0 || (b >= 20 && b <= 23); }

// ATLS_MODE_WIRE open: the 5 received header bytes at p (the record's AAD, record.rs:219) as
// raw little-endian words, and whether they frame a record of len ciphertext bytes + 16 B tag
// (Record::from_raw, record.rs:81-102).
__device__ __forceinline__ bool wire_header(const uint8_t* p, uint32_t len, uint32_t& hdr0, uint32_t& hdr1) {
  const uint32_t b0 = p[0], b1 = p[1], b2 = p[2], b3 = p[3], b4 = p[4];
  hdr0 = b0 | (b1 << 8) | (b2 << 16) | (b3 << 24);
  hdr1 = b4;
  return record_type_ok(b0) && ((b3 << 8) | b4) == len + 16u;
}

// GF(2^128) multiply by x in the reference's bit order (be words): right shift, reduce by 0xE1.
__host__ __device__ inline void gf_mulx_be(uint32_t v[4]) {
  uint32_t lsb = v[3] & 1u;
  v[3] = (v[3] >> 1) | (v[2] << 31);
  v[2] = (v[2] >> 1) | (v[1] << 31);
  v[1] = (v[1] >> 1) | (v[0] << 31);
  v[0] = (v[0] >> 1) ^ (lsb ? 0xE1000000u : 0u);
}

// z = x * y in GF(2^128) (be words). Same product as the reference's Gcm::gmult (gcm.rs:21-40):
// that routine bit-reverses both operands and runs a left-shift loop with 0x87; this is the
// NIST SP 800-38D right-shift form of the same field multiplication.
__host__ __device__ inline void gf_mul_be(const uint32_t x[4], const uint32_t y[4], uint32_t z[4]) {
  uint32_t v[4] = {y[0], y[1], y[2], y[3]};
  uint32_t a0 = 0, a1 = 0, a2 = 0, a3 = 0;
  for (int i = 0; i < 128; i++) {
    uint32_t m = 0u - ((x[i >> 5] >> (31 - (i & 31))) & 1u);
    a0 ^= v[0] & m; a1 ^= v[1] & m; a2 ^= v[2] & m; a3 ^= v[3] & m;
    gf_mulx_be(v);
  }
  z[0] = a0; z[1] = a1; z[2] = a2; z[3] = a3;
}

}  // namespace atls
