/*
 * TEST INFRASTRUCTURE ONLY — parity oracle (see ref_restatement.h).
 *
 * Literal CPU restatement of otsmr/AnotherTLS v0.1.3 (reference mounted read-only at
 * /root/reference; paths below are relative to /root/reference/anothertls/src).
 * Every function names the reference lines it restates. Quirks are kept on purpose;
 * SURVEY.md Appendix lists them. Where the reference panics we return a TlsError code
 * instead (documented divergence).
 *
 * Third-party arithmetic: Poly1305 in the reference uses ibig 0.3.6 (unpinned ^0.3.6,
 * not vendored) for (r * a) % p. Restated here as exact 256-bit arithmetic reduced
 * modulo p = 2^130 - 5; pinned by the reference's RFC 8439 KATs (poly1305.rs:112-175).
 */
#include "ref_restatement.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;

/* ---------------------------------------------------------------- AES ---- */
/* crypto/aes/cipher.rs:7-138: FIPS-197 S-box (stored there as [[u8;16];16]). */
static const uint8_t SBOX[256] = {
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
static uint8_t INV_SBOX[256];
static pthread_once_t inv_once = PTHREAD_ONCE_INIT;
static void build_inv_sbox(void) {
  for (int i = 0; i < 256; i++) INV_SBOX[SBOX[i]] = (uint8_t)i;
}

typedef struct {
  int nk, nr;               /* Blocksize B128/B192/B256, cipher.rs:140-160 */
  uint8_t ek[60][4];        /* expanded_key, cipher.rs:163-166 */
  uint8_t state[16];
} aes_t;

/* cipher.rs:251-267 — bitwise GF(2^8) multiply used by MixColumns. */
static uint8_t aes_gmult(uint8_t a, uint8_t b) {
  uint8_t p = 0;
  for (int i = 0; i < 8; i++) {
    if (b & 1) p ^= a;
    uint8_t hbs = a & 0x80;
    a <<= 1;
    if (hbs) a ^= 0x1b;
    b >>= 1;
  }
  return p;
}

/* cipher.rs:216-249 — FIPS-197 key expansion. */
static void aes_expand(const uint8_t* key, int nk, int nr, uint8_t ek[60][4]) {
  static const uint8_t rcon[10] = {0x01, 0x02, 0x04, 0x08, 0x10, 0x20, 0x40, 0x80, 0x1B, 0x36};
  memset(ek, 0, 60 * 4);
  for (int i = 0; i < nk; i++)
    for (int j = 0; j < 4; j++) ek[i][j] = key[i * 4 + j];
  for (int i = nk; i < 4 * (nr + 1); i++) {
    uint8_t t[4];
    memcpy(t, ek[i - 1], 4);
    if (i % nk == 0) {
      uint8_t tmp = t[0]; /* rot_word, cipher.rs:276-282 */
      t[0] = t[1]; t[1] = t[2]; t[2] = t[3]; t[3] = tmp;
      for (int j = 0; j < 4; j++) t[j] = SBOX[t[j]]; /* sub_word, :269-274 */
      t[0] ^= rcon[i / nk - 1];
    } else if (nk > 6 && (i % nk) == 4) {
      for (int j = 0; j < 4; j++) t[j] = SBOX[t[j]];
    }
    for (int j = 0; j < 4; j++) ek[i][j] = ek[i - nk][j] ^ t[j];
  }
}

/* cipher.rs:167-173 AES::init; Blocksize::new(key.len()*8).unwrap() (gcm.rs:49) panics otherwise. */
static int aes_init(aes_t* a, const uint8_t* key, size_t key_len) {
  if (key_len != 16 && key_len != 24 && key_len != 32) return ORA_ILLEGAL_PARAMETER;
  a->nk = (int)key_len / 4;
  a->nr = a->nk + 6;
  aes_expand(key, a->nk, a->nr, a->ek);
  memset(a->state, 0, 16);
  return ORA_OK;
}

static void add_round_key(aes_t* a, int round) { /* cipher.rs:380-386 */
  for (int x = 0; x < 4; x++)
    for (int y = 0; y < 4; y++) a->state[x * 4 + y] ^= a->ek[round * 4 + x][y];
}
static void sub_bytes(aes_t* a) { for (int i = 0; i < 16; i++) a->state[i] = SBOX[a->state[i]]; }
static void inv_sub_bytes(aes_t* a) { for (int i = 0; i < 16; i++) a->state[i] = INV_SBOX[a->state[i]]; }
static void shift_rows(aes_t* a) { /* cipher.rs:298-323 */
  uint8_t* s = a->state;
  uint8_t t = s[1]; s[1] = s[5]; s[5] = s[9]; s[9] = s[13]; s[13] = t;
  t = s[2]; s[2] = s[10]; s[10] = t;
  t = s[6]; s[6] = s[14]; s[14] = t;
  t = s[11]; s[11] = s[7]; s[7] = s[3]; s[3] = s[15]; s[15] = t;
}
static void inv_shift_rows(aes_t* a) { /* cipher.rs:325-351 */
  uint8_t* s = a->state;
  uint8_t t = s[9]; s[9] = s[5]; s[5] = s[1]; s[1] = s[13]; s[13] = t;
  t = s[2]; s[2] = s[10]; s[10] = t;
  t = s[6]; s[6] = s[14]; s[14] = t;
  t = s[3]; s[3] = s[7]; s[7] = s[11]; s[11] = s[15]; s[15] = t;
}
static void mix_columns(aes_t* a, int inverse) { /* cipher.rs:353-378 */
  static const uint8_t fwd[16] = {2, 3, 1, 1, 1, 2, 3, 1, 1, 1, 2, 3, 3, 1, 1, 2};
  static const uint8_t inv[16] = {0xE, 0xB, 0xD, 0x9, 0x9, 0xE, 0xB, 0xD, 0xD, 0x9, 0xE, 0xB, 0xB, 0xD, 0x9, 0xE};
  const uint8_t* m = inverse ? inv : fwd;
  uint8_t tmp[16] = {0};
  for (int c = 0; c < 4; c++)
    for (int r = 0; r < 4; r++)
      for (int mc = 0; mc < 4; mc++) tmp[r + 4 * c] ^= aes_gmult(m[r * 4 + mc], a->state[mc + 4 * c]);
  memcpy(a->state, tmp, 16);
}
/* cipher.rs:175-194 */
static void aes_encrypt(aes_t* a, const uint8_t in[16], uint8_t out[16]) {
  memcpy(a->state, in, 16);
  add_round_key(a, 0);
  for (int round = 1; round <= a->nr; round++) {
    sub_bytes(a);
    shift_rows(a);
    if (round < a->nr) mix_columns(a, 0);
    add_round_key(a, round);
  }
  memcpy(out, a->state, 16);
  memset(a->state, 0, 16);
}
/* cipher.rs:196-215 */
static void aes_decrypt(aes_t* a, const uint8_t in[16], uint8_t out[16]) {
  pthread_once(&inv_once, build_inv_sbox);
  memcpy(a->state, in, 16);
  add_round_key(a, a->nr);
  for (int round = a->nr - 1; round >= 0; round--) {
    inv_shift_rows(a);
    inv_sub_bytes(a);
    add_round_key(a, round);
    if (round >= 1) mix_columns(a, 1);
  }
  memcpy(out, a->state, 16);
  memset(a->state, 0, 16);
}

int ora_aes_encrypt_block(const uint8_t* key, size_t key_len, const uint8_t in[16], uint8_t out[16]) {
  aes_t a;
  int rc = aes_init(&a, key, key_len);
  if (rc) return rc;
  aes_encrypt(&a, in, out);
  return ORA_OK;
}
int ora_aes_decrypt_block(const uint8_t* key, size_t key_len, const uint8_t in[16], uint8_t out[16]) {
  aes_t a;
  int rc = aes_init(&a, key, key_len);
  if (rc) return rc;
  aes_decrypt(&a, in, out);
  return ORA_OK;
}
int ora_aes_expand_key(const uint8_t* key, size_t key_len, uint8_t out[240]) {
  aes_t a;
  int rc = aes_init(&a, key, key_len);
  if (rc) return rc;
  memset(out, 0, 240);
  memcpy(out, a.ek, (size_t)(4 * (a.nr + 1)) * 4);
  return ORA_OK;
}

/* --------------------------------------------------------- bytes.rs ---- */
/* utils/bytes.rs:110-121 to_u128_be: big-endian, zero-fill at the END, truncate to 16. */
static u128 to_u128_be(const uint8_t* b, size_t len) {
  u128 r = 0;
  if (len > 16) len = 16;
  for (size_t i = 0; i < len; i++) r += (u128)b[i] << (120 - 8 * i);
  return r;
}
/* utils/bytes.rs:46-52 */
static void u128_to_bytes_be(u128 v, uint8_t out[16]) {
  for (int i = 0; i < 16; i++) out[i] = (uint8_t)(v >> (120 - 8 * i));
}
static u128 rev128(u128 v) { /* u128::reverse_bits */
  u128 r = 0;
  for (int i = 0; i < 128; i++) {
    r = (r << 1) | (v & 1);
    v >>= 1;
  }
  return r;
}

/* ---------------------------------------------------------------- GCM ---- */
/* crypto/aes/gcm.rs:21-40 — bit-serial GF(2^128) multiply on bit-reversed operands. */
static u128 gcm_gmult(u128 a, u128 b) {
  a = rev128(a);
  b = rev128(b);
  u128 p = 0;
  const u128 hi = (u128)1 << 127;
  for (int i = 0; i < 128; i++) {
    if (b & 1) p ^= a;
    int hbs = (a & hi) != 0;
    a <<= 1;
    if (hbs) a ^= 0x87;
    b >>= 1;
  }
  return rev128(p);
}
void ora_gcm_gmult(const uint8_t a[16], const uint8_t b[16], uint8_t out[16]) {
  u128_to_bytes_be(gcm_gmult(to_u128_be(a, 16), to_u128_be(b, 16)), out);
}

/* crypto/aes/gcm.rs:42-128 Gcm::gcm */
static int gcm_core(const uint8_t* key, size_t key_len, const uint8_t* iv, size_t iv_len,
                    const uint8_t* data, size_t n, const uint8_t* aad, size_t m, int encrypt,
                    uint8_t* out, uint8_t tag[16]) {
  aes_t aes;
  int rc = aes_init(&aes, key, key_len);
  if (rc) return rc;
  u128 counter = 0, X = 0;
  uint8_t blk[16], ek[16];
  memset(blk, 0, 16);
  aes_encrypt(&aes, blk, ek);
  const u128 H = to_u128_be(ek, 16); /* :56 */
  u128 Yi;
  const int is96 = (iv_len * 8 == 96);
  if (!is96) { /* :59-70 — J0 = GHASH(IV || len) */
    u128 N = 0;
    for (size_t i = 0; i < iv_len; i += 16) {
      size_t l = iv_len > i + 16 ? 16 : iv_len - i;
      N = gcm_gmult(N ^ to_u128_be(iv + i, l), H);
    }
    u128 len = (u128)(iv_len * 8);
    Yi = gcm_gmult(N ^ len, H);
  } else { /* :71-74 */
    counter = 1;
    Yi = to_u128_be(iv, iv_len) | 1;
  }
  u128_to_bytes_be(Yi, blk);
  aes_encrypt(&aes, blk, ek);
  u128 auth_tag = to_u128_be(ek, 16); /* :76 */

  for (size_t i = 0; i < m; i += 16) { /* :78-87 */
    size_t l = m > i + 16 ? 16 : m - i;
    X = gcm_gmult(X ^ to_u128_be(aad + i, l), H);
  }
  for (size_t i = 0; i < n; i += 16) { /* :89-119 */
    counter = (counter + 1) % ((u128)1 << 32);
    u128 Y = is96 ? ((Yi & ~(u128)0xFFFFFFFFu) | counter) : (Yi + counter);
    u128_to_bytes_be(Y, blk);
    aes_encrypt(&aes, blk, ek);
    size_t l = n > i + 16 ? 16 : n - i;
    u128 d = to_u128_be(data + i, l);
    unsigned overflow = (unsigned)(16 - l) * 8;
    u128 o = (d ^ to_u128_be(ek, 16));
    o = overflow ? (o >> overflow) : o;
    uint8_t ob[16];
    u128_to_bytes_be(o, ob);
    memcpy(out + i, ob + (16 - l), l);
    if (encrypt) X = gcm_gmult(X ^ (overflow ? (o << overflow) : o), H);
    else X = gcm_gmult(X ^ d, H);
  }
  u128 len = (((u128)m * 8) << 64) | ((u128)n * 8); /* :121 */
  auth_tag ^= gcm_gmult(X ^ len, H);
  u128_to_bytes_be(auth_tag, tag);
  return ORA_OK;
}

int ora_gcm_encrypt(const uint8_t* key, size_t key_len, const uint8_t* iv, size_t iv_len,
                    const uint8_t* pt, size_t n, const uint8_t* aad, size_t m, uint8_t* ct,
                    uint8_t tag[16]) {
  return gcm_core(key, key_len, iv, iv_len, pt, n, aad, m, 1, ct, tag); /* gcm.rs:132-140 */
}
/* gcm.rs:142-157 — decrypt everything, then compare (T != auth_tag -> BadRecordMac). */
int ora_gcm_decrypt(const uint8_t* key, size_t key_len, const uint8_t* iv, size_t iv_len,
                    const uint8_t* ct, size_t n, const uint8_t* aad, size_t m, const uint8_t* tag,
                    size_t tag_len, uint8_t* pt) {
  uint8_t T[16];
  int rc = gcm_core(key, key_len, iv, iv_len, ct, n, aad, m, 0, pt, T);
  if (rc) return rc;
  if (tag_len != 16 || memcmp(T, tag, 16) != 0) return ORA_BAD_RECORD_MAC;
  return ORA_OK;
}

/* ----------------------------------------------------------- ChaCha20 ---- */
static uint32_t u8_to_u32_le(const uint8_t* b) { /* chacha20/cipher.rs:8-10 */
  return (uint32_t)b[0] | (uint32_t)b[1] << 8 | (uint32_t)b[2] << 16 | (uint32_t)b[3] << 24;
}
static uint32_t rotl32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }
#define QR(x, a, b, c, d)                              \
  do {                                                 \
    x[a] += x[b]; x[d] = rotl32(x[d] ^ x[a], 16);      \
    x[c] += x[d]; x[b] = rotl32(x[b] ^ x[c], 12);      \
    x[a] += x[b]; x[d] = rotl32(x[d] ^ x[a], 8);       \
    x[c] += x[d]; x[b] = rotl32(x[b] ^ x[c], 7);       \
  } while (0)

/* cipher.rs:18-37 init + :56-86 get_block (key 32 B, iv 12 B). */
void ora_chacha20_block(const uint8_t key[32], const uint8_t iv[12], uint32_t counter, uint8_t out[64]) {
  uint32_t st[16], x[16];
  st[0] = 0x61707865; st[1] = 0x3320646e; st[2] = 0x79622d32; st[3] = 0x6b206574;
  for (int i = 0; i < 8; i++) st[i + 4] = u8_to_u32_le(key + 4 * i);
  st[12] = counter;
  for (int i = 0; i < 3; i++) st[i + 13] = u8_to_u32_le(iv + 4 * i);
  memcpy(x, st, sizeof x);
  for (int r = 0; r < 10; r++) {
    QR(x, 0, 4, 8, 12); QR(x, 1, 5, 9, 13); QR(x, 2, 6, 10, 14); QR(x, 3, 7, 11, 15);
    QR(x, 0, 5, 10, 15); QR(x, 1, 6, 11, 12); QR(x, 2, 7, 8, 13); QR(x, 3, 4, 9, 14);
  }
  for (int i = 0; i < 16; i++) {
    uint32_t s = x[i] + st[i];
    out[4 * i] = (uint8_t)s; out[4 * i + 1] = (uint8_t)(s >> 8);
    out[4 * i + 2] = (uint8_t)(s >> 16); out[4 * i + 3] = (uint8_t)(s >> 24);
  }
}

/* cipher.rs:91-108 ChaCha20::encrypt. Keeps the F4 quirk: on the last block
 * `count = input.len() % 64`, so when len % 64 == 0 the final 64 bytes are NOT XORed
 * (:99-102). Block count uses f32::ceil (:94). Returns -1 where the reference returns None. */
int ora_chacha20_encrypt(const uint8_t* in, size_t len, const uint8_t* key, size_t key_len,
                         const uint8_t* iv, size_t iv_len, size_t counter, uint8_t* out) {
  if (out != in) memmove(out, in, len);
  const int ok = (key_len == 32 && iv_len == 12);
  size_t blocks_len = (size_t)ceilf((float)len / 64.0f);
  for (size_t j = 0; j < blocks_len; j++) {
    if (!ok) return -1; /* chacha20.clone()? on None */
    uint8_t ks[64];
    ora_chacha20_block(key, iv, (uint32_t)(counter + j), ks);
    size_t count = 64;
    if (j * 64 + 64 >= len) count = len % 64;
    for (size_t i = 0; i < count; i++) out[j * 64 + i] ^= ks[i];
  }
  return 0;
}

/* ----------------------------------------------------------- Poly1305 ---- */
/* 256-bit little-endian limbs, exact arithmetic (restates ibig's IBig ops). */
typedef struct { uint64_t w[5]; } big_t;

static void big_from_le(big_t* r, const uint8_t* b, size_t len) { /* bytes.rs:8-14 */
  memset(r, 0, sizeof *r);
  for (size_t i = 0; i < len; i++) r->w[i / 8] |= (uint64_t)b[i] << (8 * (i % 8));
}
static void big_add(big_t* r, const big_t* a) {
  u128 c = 0;
  for (int i = 0; i < 5; i++) {
    c += (u128)r->w[i] + a->w[i];
    r->w[i] = (uint64_t)c;
    c >>= 64;
  }
}
static int big_ge(const big_t* a, const big_t* b) {
  for (int i = 4; i >= 0; i--) {
    if (a->w[i] != b->w[i]) return a->w[i] > b->w[i];
  }
  return 1;
}
static void big_sub(big_t* r, const big_t* a) {
  uint64_t borrow = 0;
  for (int i = 0; i < 5; i++) {
    u128 d = (u128)r->w[i] - a->w[i] - borrow;
    r->w[i] = (uint64_t)d;
    borrow = (uint64_t)(d >> 64) & 1;
  }
}
/* r = (a * b) mod p, p = 2^130 - 5 (poly1305.rs:44: a = (r * a) % p). Operands < 2^192. */
static void big_mulmod_p(big_t* r, const big_t* a, const big_t* b) {
  uint64_t prod[8] = {0};
  for (int i = 0; i < 3; i++) {
    u128 c = 0;
    for (int j = 0; j < 3; j++) {
      c += (u128)a->w[i] * b->w[j] + prod[i + j];
      prod[i + j] = (uint64_t)c;
      c >>= 64;
    }
    for (int k = i + 3; c && k < 8; k++) {
      c += prod[k];
      prod[k] = (uint64_t)c;
      c >>= 64;
    }
  }
  big_t x;
  memset(&x, 0, sizeof x);
  for (int i = 0; i < 5; i++) x.w[i] = prod[i]; /* < 2^320 fits: products < 2^384 are not possible here */
  /* fold: x = lo + 5*hi while x >= 2^130 */
  for (;;) {
    big_t hi, lo;
    memset(&hi, 0, sizeof hi);
    memset(&lo, 0, sizeof lo);
    lo.w[0] = x.w[0]; lo.w[1] = x.w[1]; lo.w[2] = x.w[2] & 3;
    hi.w[0] = (x.w[2] >> 2) | (x.w[3] << 62);
    hi.w[1] = (x.w[3] >> 2) | (x.w[4] << 62);
    hi.w[2] = x.w[4] >> 2;
    if (!hi.w[0] && !hi.w[1] && !hi.w[2]) break;
    big_t five = hi;
    big_add(&five, &hi); big_add(&five, &hi); big_add(&five, &hi); big_add(&five, &hi);
    x = lo;
    big_add(&x, &five);
  }
  big_t p;
  memset(&p, 0, sizeof p);
  p.w[0] = 0xFFFFFFFFFFFFFFFBull; p.w[1] = 0xFFFFFFFFFFFFFFFFull; p.w[2] = 3;
  while (big_ge(&x, &p)) big_sub(&x, &p);
  *r = x;
}

/* poly1305.rs:24-51 Poly1305::mac */
void ora_poly1305_mac(const uint8_t key[32], const uint8_t* msg, size_t len, uint8_t tag[16]) {
  big_t r, s, a, n;
  big_from_le(&r, key, 16);
  r.w[0] &= 0x0ffffffc0fffffffull; /* clamp 0x0ffffffc0ffffffc0ffffffc0fffffff */
  r.w[1] &= 0x0ffffffc0ffffffcull;
  big_from_le(&s, key + 16, 16);
  memset(&a, 0, sizeof a);
  size_t nb = (size_t)ceilf((float)len / 16.0f); /* :32 f32 ceil */
  for (size_t i = 1; i <= nb; i++) {
    if (i * 16 > len) { /* :33-38 partial block: append 0x01 */
      uint8_t buf[17];
      size_t l = len - (i - 1) * 16;
      memcpy(buf, msg + (i - 1) * 16, l);
      buf[l] = 0x01;
      big_from_le(&n, buf, l + 1);
    } else { /* :39-43 full block + 2^128 */
      big_from_le(&n, msg + (i - 1) * 16, 16);
      n.w[2] += 1;
    }
    big_add(&a, &n);
    big_mulmod_p(&a, &r, &a);
  }
  big_add(&a, &s); /* :46 */
  for (int i = 0; i < 16; i++) tag[i] = (uint8_t)(a.w[i / 8] >> (8 * (i % 8))); /* resize(16) */
}

/* poly1305.rs:19-22 key_gen (ChaCha20Block::init(..).unwrap() panics on bad sizes). */
int ora_poly1305_key_gen(const uint8_t* key, size_t key_len, const uint8_t* iv, size_t iv_len, uint8_t otk[32]) {
  if (key_len != 32 || iv_len != 12) return ORA_ILLEGAL_PARAMETER;
  uint8_t b[64];
  ora_chacha20_block(key, iv, 0, b);
  memcpy(otk, b, 32);
  return ORA_OK;
}

/* poly1305.rs:52-66 pad16 + get_mac_data, MAC'd directly. */
static void mac_aead(const uint8_t otk[32], const uint8_t* ct, size_t n, const uint8_t* aad, size_t m,
                     uint8_t tag[16]) {
  size_t pa = (m % 16) ? 16 - m % 16 : 0, pc = (n % 16) ? 16 - n % 16 : 0;
  size_t total = m + pa + n + pc + 16;
  uint8_t* md = (uint8_t*)calloc(total ? total : 1, 1);
  memcpy(md, aad, m);
  memcpy(md + m + pa, ct, n);
  uint64_t al = m, cl = n;
  for (int i = 0; i < 8; i++) {
    md[m + pa + n + pc + i] = (uint8_t)(al >> (8 * i));
    md[m + pa + n + pc + 8 + i] = (uint8_t)(cl >> (8 * i));
  }
  ora_poly1305_mac(otk, md, total, tag);
  free(md);
}

/* poly1305.rs:70-81 encrypt: ct = ChaCha20(ctr=1), otk, tag over ct. */
int ora_chacha_poly_encrypt(const uint8_t* key, size_t key_len, const uint8_t* iv, size_t iv_len,
                            const uint8_t* pt, size_t n, const uint8_t* aad, size_t m, uint8_t* ct,
                            uint8_t tag[16]) {
  if (ora_chacha20_encrypt(pt, n, key, key_len, iv, iv_len, 1, ct) != 0) return ORA_ILLEGAL_PARAMETER;
  uint8_t otk[32];
  if (ora_poly1305_key_gen(key, key_len, iv, iv_len, otk)) return ORA_ILLEGAL_PARAMETER;
  mac_aead(otk, ct, n, aad, m, tag);
  return ORA_OK;
}
/* poly1305.rs:83-99 decrypt: compare first, then decrypt. */
int ora_chacha_poly_decrypt(const uint8_t* key, size_t key_len, const uint8_t* iv, size_t iv_len,
                            const uint8_t* ct, size_t n, const uint8_t* aad, size_t m,
                            const uint8_t* tag, size_t tag_len, uint8_t* pt) {
  uint8_t otk[32], T[16];
  if (ora_poly1305_key_gen(key, key_len, iv, iv_len, otk)) return ORA_ILLEGAL_PARAMETER;
  mac_aead(otk, ct, n, aad, m, T);
  if (tag_len == 16 && memcmp(T, tag, 16) == 0) {
    if (ora_chacha20_encrypt(ct, n, key, key_len, iv, iv_len, 1, pt) == 0) return ORA_OK;
  }
  return ORA_BAD_RECORD_MAC;
}

/* ciphersuite.rs:78-87 get_cipher: 0x1301/0x1302 -> Gcm (AES size from key.len()),
 * 0x1303 -> Poly1305, anything else -> InsufficientSecurity. */
int ora_cipher_encrypt(uint16_t suite, const uint8_t* key, size_t key_len, const uint8_t* iv,
                       size_t iv_len, const uint8_t* pt, size_t n, const uint8_t* aad, size_t m,
                       uint8_t* ct, uint8_t tag[16]) {
  if (suite == 0x1301 || suite == 0x1302) return ora_gcm_encrypt(key, key_len, iv, iv_len, pt, n, aad, m, ct, tag);
  if (suite == 0x1303) return ora_chacha_poly_encrypt(key, key_len, iv, iv_len, pt, n, aad, m, ct, tag);
  return ORA_INSUFFICIENT_SECURITY;
}
int ora_cipher_decrypt(uint16_t suite, const uint8_t* key, size_t key_len, const uint8_t* iv,
                       size_t iv_len, const uint8_t* ct, size_t n, const uint8_t* aad, size_t m,
                       const uint8_t* tag, size_t tag_len, uint8_t* pt) {
  if (suite == 0x1301 || suite == 0x1302)
    return ora_gcm_decrypt(key, key_len, iv, iv_len, ct, n, aad, m, tag, tag_len, pt);
  if (suite == 0x1303) return ora_chacha_poly_decrypt(key, key_len, iv, iv_len, ct, n, aad, m, tag, tag_len, pt);
  return ORA_INSUFFICIENT_SECURITY;
}

/* ------------------------------------------------------------- SHA-2 ---- */
/* hash/sha256.rs:39-192 (length field: only 7 of 8 bytes written, :60-62). */
typedef struct { uint8_t input[64]; size_t input_len; uint32_t state[8]; u128 length; } sha256_t;
static uint32_t rotr32(uint32_t w, int n) { return (w >> n) | (w << ((32 - n) & 31)); }
static void sha256_round(sha256_t* s) {
  static const uint32_t k[64] = {
      0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
      0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
      0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
      0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
      0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
      0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
      0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
      0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
  uint32_t w[64], a = s->state[0], b = s->state[1], c = s->state[2], d = s->state[3], e = s->state[4],
                  f = s->state[5], g = s->state[6], h = s->state[7];
  for (int t = 0; t < 64; t++) {
    if (t < 16) {
      w[t] = (uint32_t)s->input[4 * t] << 24 | (uint32_t)s->input[4 * t + 1] << 16 |
             (uint32_t)s->input[4 * t + 2] << 8 | s->input[4 * t + 3];
    } else {
      uint32_t s1 = rotr32(w[t - 2], 17) ^ rotr32(w[t - 2], 19) ^ (w[t - 2] >> 10);
      uint32_t s0 = rotr32(w[t - 15], 7) ^ rotr32(w[t - 15], 18) ^ (w[t - 15] >> 3);
      w[t] = s1 + w[t - 7] + s0 + w[t - 16];
    }
    uint32_t t1 = h + (rotr32(e, 6) ^ rotr32(e, 11) ^ rotr32(e, 25)) + ((e & f) ^ (~e & g)) + k[t] + w[t];
    uint32_t t2 = (rotr32(a, 2) ^ rotr32(a, 13) ^ rotr32(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
    h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  s->state[0] += a; s->state[1] += b; s->state[2] += c; s->state[3] += d;
  s->state[4] += e; s->state[5] += f; s->state[6] += g; s->state[7] += h;
  s->input_len = 0;
}
static void sha256_init(sha256_t* s) {
  static const uint32_t iv[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  memset(s, 0, sizeof *s);
  memcpy(s->state, iv, sizeof iv);
}
static void sha256_update(sha256_t* s, const uint8_t* buf, size_t len) { /* :142-152 */
  s->length += len;
  for (size_t i = 0; i < len; i++) {
    s->input[s->input_len++] = buf[i];
    if (s->input_len == 64) sha256_round(s);
  }
}
static void sha256_final(const sha256_t* in, uint8_t out[32]) { /* :154-170, padd_input :47-68 */
  sha256_t s = *in;
  u128 input_len = s.length;
  size_t padding_length = 64 - (size_t)(input_len % 64);
  uint8_t padding[64];
  memset(padding, 0, sizeof padding);
  if (padding_length > 0) {
    padding[0] = 0x80;
    if (padding_length < 9) {
      sha256_update(&s, padding, padding_length);
      padding_length = 64;
      padding[0] = 0;
    }
    for (int i = 1; i < 8; i++) padding[padding_length - i] = (uint8_t)((input_len * 8) >> ((i - 1) * 8));
    sha256_update(&s, padding, padding_length);
  }
  for (int i = 0; i < 32; i++) out[i] = (uint8_t)(s.state[i >> 2] >> (8 * (3 - (i & 3))));
}
void ora_sha256(const uint8_t* msg, size_t len, uint8_t out[32]) {
  sha256_t s;
  sha256_init(&s);
  sha256_update(&s, msg, len);
  sha256_final(&s, out);
}

/* hash/sha384.rs:39-206 (length field: 15 of 16 bytes written, :47-65). */
typedef struct { uint8_t input[128]; size_t input_len; uint64_t state[8]; u128 length; } sha384_t;
static uint64_t rotr64(uint64_t w, int n) { return (w >> n) | (w << ((64 - n) & 63)); }
static void sha384_round(sha384_t* s) {
  static const uint64_t k[80] = {
      0x428a2f98d728ae22ull, 0x7137449123ef65cdull, 0xb5c0fbcfec4d3b2full, 0xe9b5dba58189dbbcull,
      0x3956c25bf348b538ull, 0x59f111f1b605d019ull, 0x923f82a4af194f9bull, 0xab1c5ed5da6d8118ull,
      0xd807aa98a3030242ull, 0x12835b0145706fbeull, 0x243185be4ee4b28cull, 0x550c7dc3d5ffb4e2ull,
      0x72be5d74f27b896full, 0x80deb1fe3b1696b1ull, 0x9bdc06a725c71235ull, 0xc19bf174cf692694ull,
      0xe49b69c19ef14ad2ull, 0xefbe4786384f25e3ull, 0x0fc19dc68b8cd5b5ull, 0x240ca1cc77ac9c65ull,
      0x2de92c6f592b0275ull, 0x4a7484aa6ea6e483ull, 0x5cb0a9dcbd41fbd4ull, 0x76f988da831153b5ull,
      0x983e5152ee66dfabull, 0xa831c66d2db43210ull, 0xb00327c898fb213full, 0xbf597fc7beef0ee4ull,
      0xc6e00bf33da88fc2ull, 0xd5a79147930aa725ull, 0x06ca6351e003826full, 0x142929670a0e6e70ull,
      0x27b70a8546d22ffcull, 0x2e1b21385c26c926ull, 0x4d2c6dfc5ac42aedull, 0x53380d139d95b3dfull,
      0x650a73548baf63deull, 0x766a0abb3c77b2a8ull, 0x81c2c92e47edaee6ull, 0x92722c851482353bull,
      0xa2bfe8a14cf10364ull, 0xa81a664bbc423001ull, 0xc24b8b70d0f89791ull, 0xc76c51a30654be30ull,
      0xd192e819d6ef5218ull, 0xd69906245565a910ull, 0xf40e35855771202aull, 0x106aa07032bbd1b8ull,
      0x19a4c116b8d2d0c8ull, 0x1e376c085141ab53ull, 0x2748774cdf8eeb99ull, 0x34b0bcb5e19b48a8ull,
      0x391c0cb3c5c95a63ull, 0x4ed8aa4ae3418acbull, 0x5b9cca4f7763e373ull, 0x682e6ff3d6b2b8a3ull,
      0x748f82ee5defb2fcull, 0x78a5636f43172f60ull, 0x84c87814a1f0ab72ull, 0x8cc702081a6439ecull,
      0x90befffa23631e28ull, 0xa4506cebde82bde9ull, 0xbef9a3f7b2c67915ull, 0xc67178f2e372532bull,
      0xca273eceea26619cull, 0xd186b8c721c0c207ull, 0xeada7dd6cde0eb1eull, 0xf57d4f7fee6ed178ull,
      0x06f067aa72176fbaull, 0x0a637dc5a2c898a6ull, 0x113f9804bef90daeull, 0x1b710b35131c471bull,
      0x28db77f523047d84ull, 0x32caab7b40c72493ull, 0x3c9ebe0a15c9bebcull, 0x431d67c49c100d4cull,
      0x4cc5d4becb3e42b6ull, 0x597f299cfc657e2aull, 0x5fcb6fab3ad6faecull, 0x6c44198c4a475817ull};
  uint64_t w[80], a = s->state[0], b = s->state[1], c = s->state[2], d = s->state[3], e = s->state[4],
                  f = s->state[5], g = s->state[6], h = s->state[7];
  for (int t = 0; t < 80; t++) {
    if (t < 16) {
      uint64_t v = 0;
      for (int j = 0; j < 8; j++) v = (v << 8) | s->input[8 * t + j];
      w[t] = v;
    } else {
      uint64_t s1 = rotr64(w[t - 2], 19) ^ rotr64(w[t - 2], 61) ^ (w[t - 2] >> 6);
      uint64_t s0 = rotr64(w[t - 15], 1) ^ rotr64(w[t - 15], 8) ^ (w[t - 15] >> 7);
      w[t] = s1 + w[t - 7] + s0 + w[t - 16];
    }
    uint64_t t1 = h + (rotr64(e, 14) ^ rotr64(e, 18) ^ rotr64(e, 41)) + ((e & f) ^ (~e & g)) + k[t] + w[t];
    uint64_t t2 = (rotr64(a, 28) ^ rotr64(a, 34) ^ rotr64(a, 39)) + ((a & b) ^ (a & c) ^ (b & c));
    h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  s->state[0] += a; s->state[1] += b; s->state[2] += c; s->state[3] += d;
  s->state[4] += e; s->state[5] += f; s->state[6] += g; s->state[7] += h;
  s->input_len = 0;
}
static void sha384_init(sha384_t* s) {
  static const uint64_t iv[8] = {0xcbbb9d5dc1059ed8ull, 0x629a292a367cd507ull, 0x9159015a3070dd17ull,
                                 0x152fecd8f70e5939ull, 0x67332667ffc00b31ull, 0x8eb44a8768581511ull,
                                 0xdb0c2e0d64f98fa7ull, 0x47b5481dbefa4fa4ull};
  memset(s, 0, sizeof *s);
  memcpy(s->state, iv, sizeof iv);
}
static void sha384_update(sha384_t* s, const uint8_t* buf, size_t len) {
  s->length += len;
  for (size_t i = 0; i < len; i++) {
    s->input[s->input_len++] = buf[i];
    if (s->input_len == 128) sha384_round(s);
  }
}
static void sha384_final(const sha384_t* in, uint8_t out[48]) {
  sha384_t s = *in;
  u128 input_len = s.length;
  size_t padding_length = 128 - (size_t)(input_len % 128);
  uint8_t padding[128];
  memset(padding, 0, sizeof padding);
  if (padding_length > 0) {
    padding[0] = 0x80;
    if (padding_length < 17) {
      sha384_update(&s, padding, padding_length);
      padding_length = 128;
      padding[0] = 0;
    }
    for (int i = 1; i < 16; i++) padding[padding_length - i] = (uint8_t)((input_len * 8) >> ((i - 1) * 8));
    sha384_update(&s, padding, padding_length);
  }
  for (int i = 0; i < 48; i++) out[i] = (uint8_t)(s.state[i >> 3] >> (8 * (7 - (i & 7))));
}
void ora_sha384(const uint8_t* msg, size_t len, uint8_t out[48]) {
  sha384_t s;
  sha384_init(&s);
  sha384_update(&s, msg, len);
  sha384_final(&s, out);
}

static void sha_x(int hash, const uint8_t* m, size_t l, uint8_t* out) { /* hash/mod.rs:37-42 */
  if (hash == ORA_SHA384) ora_sha384(m, l, out);
  else ora_sha256(m, l, out);
}

/* hash/hmac.rs:29-78 — keys longer than 64 bytes are hashed for BOTH hashes (:41-49). */
void ora_hmac(int hash, const uint8_t* key, size_t key_len, const uint8_t* msg, size_t len, uint8_t* out) {
  uint8_t k_ipad[128], k_opad[128], padded[128], hk[48];
  size_t size = (hash == ORA_SHA384) ? 128 : 64;
  memset(padded, 0, sizeof padded);
  if (key_len > 64) {
    sha_x(hash, key, key_len, hk);
    key = hk;
    key_len = (size_t)hash;
  }
  memcpy(padded, key, key_len);
  for (size_t i = 0; i < size; i++) {
    k_opad[i] = padded[i] ^ 0x5C;
    k_ipad[i] = padded[i] ^ 0x36;
  }
  uint8_t* inner = (uint8_t*)malloc(size + len);
  memcpy(inner, k_ipad, size);
  if (len) memcpy(inner + size, msg, len);
  uint8_t ih[48], outer[128 + 48];
  sha_x(hash, inner, size + len, ih);
  free(inner);
  memcpy(outer, k_opad, size);
  memcpy(outer + size, ih, (size_t)hash);
  sha_x(hash, outer, size + (size_t)hash, out);
}

/* hash/hkdf.rs:24-32 */
void ora_hkdf_extract(int hash, const uint8_t* salt, size_t salt_len, const uint8_t* ikm, size_t ikm_len, uint8_t* prk) {
  ora_hmac(hash, salt, salt_len, ikm, ikm_len, prk);
}
/* hash/hkdf.rs:35-65 (u8 counter; None when out_len > 255*HashLen -> -1) */
int ora_hkdf_expand(int hash, const uint8_t* prk, size_t prk_len, const uint8_t* info, size_t info_len,
                    uint8_t* okm, size_t out_len) {
  size_t hl = (size_t)hash;
  if (out_len > hl * 255) return -1;
  uint8_t last[48];
  size_t last_len = 0, got = 0;
  uint8_t i = 0;
  uint8_t* buf = (uint8_t*)malloc(hl + info_len + 1);
  while (got < out_len) {
    i += 1;
    memcpy(buf, last, last_len);
    if (info_len) memcpy(buf + last_len, info, info_len);
    buf[last_len + info_len] = i;
    ora_hmac(hash, prk, prk_len, buf, last_len + info_len + 1, last);
    last_len = hl;
    size_t need = (out_len < got + hl ? out_len : got + hl) - got;
    memcpy(okm + got, last, need);
    got += need;
  }
  free(buf);
  return 0;
}

/* ---------------------------------------------------- key schedule ---- */
/* net/key_schedule.rs:20-29 */
size_t ora_hkdf_expand_label(const uint8_t* label, size_t label_len, const uint8_t* ctx, size_t ctx_len,
                             size_t out_len, uint8_t* buf) {
  size_t p = 0;
  buf[p++] = (uint8_t)(out_len >> 8);
  buf[p++] = (uint8_t)out_len;
  buf[p++] = (uint8_t)(6 + label_len);
  memcpy(buf + p, "tls13 ", 6);
  p += 6;
  memcpy(buf + p, label, label_len);
  p += label_len;
  buf[p++] = (uint8_t)ctx_len;
  if (ctx_len) memcpy(buf + p, ctx, ctx_len); /* ctx may be NULL when empty (memcpy UB, UBSan) */
  return p + ctx_len;
}
/* net/key_schedule.rs:40-50 Key::from_hkdf (traffic secret is the PRK). */
int ora_key_from_secret(int hash, const uint8_t* secret, size_t secret_len, size_t key_len, size_t iv_len,
                        uint8_t* key, uint8_t* iv) {
  uint8_t info[300];
  size_t il = ora_hkdf_expand_label((const uint8_t*)"key", 3, NULL, 0, key_len, info);
  if (ora_hkdf_expand(hash, secret, secret_len, info, il, key, key_len)) return ORA_INTERNAL_ERROR;
  il = ora_hkdf_expand_label((const uint8_t*)"iv", 2, NULL, 0, iv_len, info);
  if (ora_hkdf_expand(hash, secret, secret_len, info, il, iv, iv_len)) return ORA_INTERNAL_ERROR;
  return ORA_OK;
}
/* net/key_schedule.rs:170-222 KeySchedule::do_key_schedule (after the X25519 shared secret) and
 * :87-114 WriteKeys::application_keys_from_master_secret. out = 5 secrets of HashLen bytes:
 * client / server handshake traffic secret, master secret (the PRK), client / server application
 * traffic secret 0. handshake_hash may be NULL (the last two are then left untouched). */
int ora_key_schedule(int hash, const uint8_t* shared, size_t shared_len, const uint8_t* hello_hash,
                     const uint8_t* handshake_hash, uint8_t* out) {
  const size_t hl = (size_t)hash;
  uint8_t zeros[48], empty_hash[48], early[48], derived[48], hs[48], info[300];
  memset(zeros, 0, sizeof zeros);
  sha_x(hash, (const uint8_t*)"", 0, empty_hash);
  ora_hkdf_extract(hash, zeros, hl, zeros, hl, early);                 /* Early Secret */
  size_t il = ora_hkdf_expand_label((const uint8_t*)"derived", 7, empty_hash, hl, hl, info);
  if (ora_hkdf_expand(hash, early, hl, info, il, derived, hl)) return ORA_INTERNAL_ERROR;
  ora_hkdf_extract(hash, derived, hl, shared, shared_len, hs);         /* Handshake Secret */
  il = ora_hkdf_expand_label((const uint8_t*)"c hs traffic", 12, hello_hash, hl, hl, info);
  if (ora_hkdf_expand(hash, hs, hl, info, il, out, hl)) return ORA_INTERNAL_ERROR;
  il = ora_hkdf_expand_label((const uint8_t*)"s hs traffic", 12, hello_hash, hl, hl, info);
  if (ora_hkdf_expand(hash, hs, hl, info, il, out + hl, hl)) return ORA_INTERNAL_ERROR;
  il = ora_hkdf_expand_label((const uint8_t*)"derived", 7, empty_hash, hl, hl, info);
  if (ora_hkdf_expand(hash, hs, hl, info, il, derived, hl)) return ORA_INTERNAL_ERROR;
  ora_hkdf_extract(hash, derived, hl, zeros, hl, out + 2 * hl);        /* Master Secret */
  if (handshake_hash) {
    il = ora_hkdf_expand_label((const uint8_t*)"c ap traffic", 12, handshake_hash, hl, hl, info);
    if (ora_hkdf_expand(hash, out + 2 * hl, hl, info, il, out + 3 * hl, hl)) return ORA_INTERNAL_ERROR;
    il = ora_hkdf_expand_label((const uint8_t*)"s ap traffic", 12, handshake_hash, hl, hl, info);
    if (ora_hkdf_expand(hash, out + 2 * hl, hl, info, il, out + 4 * hl, hl)) return ORA_INTERNAL_ERROR;
  }
  return ORA_OK;
}
/* net/key_schedule.rs:51-64 */
void ora_per_record_nonce(const uint8_t iv[12], uint64_t seq, uint8_t out[12]) {
  memcpy(out, iv, 12);
  for (int i = 0; i < 8; i++) out[11 - i] ^= (uint8_t)(seq >> (i * 8));
}

/* ------------------------------------------------------ record layer ---- */
static int valid_record_type(uint8_t b) { /* record.rs:22-33 RecordType::new */
  return b == 0 || b == 20 || b == 21 || b == 22 || b == 23;
}
/* net/record.rs:162-198 RecordPayloadProtection::encrypt */
int ora_record_seal(uint16_t suite, const uint8_t* key, size_t key_len, const uint8_t iv[12], uint64_t seq,
                    uint8_t content_type, const uint8_t* frag, size_t frag_len, uint8_t* wire, size_t* wire_len) {
  size_t n = frag_len + 1;
  size_t len = n + 16;
  wire[0] = 23; wire[1] = 3; wire[2] = 3;
  wire[3] = (uint8_t)(len >> 8); wire[4] = (uint8_t)len; /* u16 truncation, :176-183 */
  uint8_t* inner = (uint8_t*)malloc(n);
  memcpy(inner, frag, frag_len);
  inner[frag_len] = content_type; /* :172-173 */
  uint8_t nonce[12];
  ora_per_record_nonce(iv, seq, nonce);
  int rc = ora_cipher_encrypt(suite, key, key_len, nonce, 12, inner, n, wire, 5, wire + 5, wire + 5 + n);
  free(inner);
  if (rc) return rc;
  *wire_len = 5 + n + 16;
  return ORA_OK;
}
/* net/record.rs:81-102 Record::from_raw + :201-240 decrypt */
int ora_record_open(uint16_t suite, const uint8_t* key, size_t key_len, const uint8_t iv[12], uint64_t seq,
                    const uint8_t* wire, size_t wire_len, uint8_t* content, size_t* content_len,
                    uint8_t* content_type) {
  if (wire_len < 5) return ORA_DECODE_ERROR;
  if (!valid_record_type(wire[0])) return ORA_DECODE_ERROR;
  size_t len = ((size_t)wire[3] << 8) | wire[4];
  if (wire_len < 2 + len) return ORA_DECODE_ERROR;
  if (wire_len < 5 + len) return ORA_DECODE_ERROR; /* divergence: reference slice panics (:88) */
  if (len < 16) return ORA_DECODE_ERROR;           /* divergence: usize underflow panic (:208) */
  const uint8_t* frag = wire + 5;
  size_t n = len - 16;
  uint8_t nonce[12];
  ora_per_record_nonce(iv, seq, nonce);
  uint8_t* pt = (uint8_t*)malloc(n ? n : 1);
  int rc = ora_cipher_decrypt(suite, key, key_len, nonce, 12, frag, n, wire, 5, frag + n, 16, pt);
  if (rc) {
    free(pt);
    return rc == ORA_INSUFFICIENT_SECURITY || rc == ORA_ILLEGAL_PARAMETER ? rc : ORA_DECRYPT_ERROR;
  }
  uint8_t type = 0;
  size_t record_len = 0;
  for (size_t i = n; i-- > 0;) {
    if (pt[i] != 0) {
      if (!valid_record_type(pt[i])) {
        free(pt);
        return ORA_DECODE_ERROR;
      }
      type = pt[i];
      record_len = i;
      break;
    }
  }
  memcpy(content, pt, record_len);
  *content_len = record_len;
  *content_type = type;
  free(pt);
  return ORA_OK;
}

/* ------------------------------------------------------------ batches ---- */
enum { MODE_TLS = 0, MODE_RAW = 1, MODE_WIRE = 2 };

static int seal_one(const ora_key* keys, const ora_rec* r, const uint8_t* in, const uint8_t* aux,
                    uint8_t* out, uint8_t* tag) {
  const ora_key* k = &keys[r->key_slot];
  if (r->mode == MODE_WIRE) { /* record.rs:162-198: header || ct || tag at out_off */
    size_t wl = 0;
    uint8_t* w = out + r->out_off;
    int rc = ora_record_seal(k->suite, k->key, k->key_len, k->static_iv, r->seq, r->content_type, in + r->in_off,
                             r->len, w, &wl);
    if (!rc && tag) memcpy(tag, w + wl - 16, 16);
    return rc;
  }
  if (r->mode == MODE_TLS) {
    size_t n = (size_t)r->len + 1, L = n + 16;
    uint8_t hdr[5] = {23, 3, 3, (uint8_t)(L >> 8), (uint8_t)L};
    uint8_t nonce[12];
    ora_per_record_nonce(k->static_iv, r->seq, nonce);
    uint8_t* inner = (uint8_t*)malloc(n);
    memcpy(inner, in + r->in_off, r->len);
    inner[r->len] = r->content_type;
    int rc = ora_cipher_encrypt(k->suite, k->key, k->key_len, nonce, 12, inner, n, hdr, 5, out + r->out_off, tag);
    free(inner);
    return rc;
  }
  const uint8_t* nonce = aux + r->aux_off;
  return ora_cipher_encrypt(k->suite, k->key, k->key_len, nonce, r->iv_len, in + r->in_off, r->len,
                            nonce + r->iv_len, r->aad_len, out + r->out_off, tag);
}

static int open_one(const ora_key* keys, const ora_rec* r, const uint8_t* in, const uint8_t* aux,
                    const uint8_t* tag, uint8_t* out, ora_open_result* res) {
  const ora_key* k = &keys[r->key_slot];
  memset(res, 0, sizeof *res);
  if (r->mode == MODE_TLS || r->mode == MODE_WIRE) {
    size_t n = r->len, L = n + 16;
    uint8_t hdr[5] = {23, 3, 3, (uint8_t)(L >> 8), (uint8_t)L};
    const uint8_t* ct = in + r->in_off;
    if (r->mode == MODE_WIRE) { /* record.rs:81-102 from_raw, :201-220: received header = AAD */
      const uint8_t* w = in + r->in_off;
      if (!valid_record_type(w[0]) || (((size_t)w[3] << 8) | w[4]) != L) {
        res->status = ORA_DECODE_ERROR;
        return 0;
      }
      memcpy(hdr, w, 5);
      ct = w + 5;
      tag = ct + n;
    }
    uint8_t nonce[12];
    ora_per_record_nonce(k->static_iv, r->seq, nonce);
    uint8_t* pt = out + r->out_off;
    int rc = ora_cipher_decrypt(k->suite, k->key, k->key_len, nonce, 12, ct, n, hdr, 5, tag, 16, pt);
    if (rc) {
      res->status = (rc == ORA_BAD_RECORD_MAC) ? ORA_DECRYPT_ERROR : (uint8_t)rc;
      return 0;
    }
    for (size_t i = n; i-- > 0;) {
      if (pt[i] != 0) {
        if (!valid_record_type(pt[i])) {
          res->status = ORA_DECODE_ERROR;
          return 0;
        }
        res->content_type = pt[i];
        res->content_len = (uint32_t)i;
        break;
      }
    }
    return 0;
  }
  const uint8_t* nonce = aux + r->aux_off;
  int rc = ora_cipher_decrypt(k->suite, k->key, k->key_len, nonce, r->iv_len, in + r->in_off, r->len,
                              nonce + r->iv_len, r->aad_len, tag, 16, out + r->out_off);
  res->status = (uint8_t)rc;
  res->content_len = r->len;
  return 0;
}

typedef struct {
  const ora_key* keys; const ora_rec* recs; const uint8_t* in; const uint8_t* aux;
  uint8_t* out; uint8_t* tags; const uint8_t* itags; ora_open_result* res;
  uint32_t lo, hi; int rc; int open;
} job_t;

static void* run_job(void* p) {
  job_t* j = (job_t*)p;
  for (uint32_t i = j->lo; i < j->hi; i++) {
    int rc = j->open ? open_one(j->keys, &j->recs[i], j->in, j->aux, j->itags ? j->itags + 16 * (size_t)i : NULL, j->out, &j->res[i])
                     : seal_one(j->keys, &j->recs[i], j->in, j->aux, j->out,
                                j->tags ? j->tags + 16 * (size_t)i : NULL);
    if (rc && !j->rc) j->rc = rc;
  }
  return NULL;
}

static int run_batch(job_t proto, uint32_t n, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  if ((uint32_t)nthreads > n) nthreads = n ? (int)n : 1;
  job_t* jobs = (job_t*)calloc((size_t)nthreads, sizeof(job_t));
  pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
  for (int t = 0; t < nthreads; t++) {
    jobs[t] = proto;
    jobs[t].lo = (uint32_t)((uint64_t)n * t / nthreads);
    jobs[t].hi = (uint32_t)((uint64_t)n * (t + 1) / nthreads);
    if (nthreads == 1) run_job(&jobs[t]);
    else pthread_create(&th[t], NULL, run_job, &jobs[t]);
  }
  int rc = 0;
  for (int t = 0; t < nthreads; t++) {
    if (nthreads > 1) pthread_join(th[t], NULL);
    if (jobs[t].rc && !rc) rc = jobs[t].rc;
  }
  free(jobs);
  free(th);
  return rc;
}

int ora_seal_batch(const ora_key* keys, const ora_rec* recs, uint32_t n, const uint8_t* in,
                   const uint8_t* aux, uint8_t* out, uint8_t* tags, int nthreads) {
  job_t p;
  memset(&p, 0, sizeof p);
  p.keys = keys; p.recs = recs; p.in = in; p.aux = aux; p.out = out; p.tags = tags;
  return run_batch(p, n, nthreads);
}
int ora_open_batch(const ora_key* keys, const ora_rec* recs, uint32_t n, const uint8_t* in,
                   const uint8_t* aux, const uint8_t* tags, uint8_t* out, ora_open_result* res,
                   int nthreads) {
  job_t p;
  memset(&p, 0, sizeof p);
  p.keys = keys; p.recs = recs; p.in = in; p.aux = aux; p.out = out; p.itags = tags; p.res = res; p.open = 1;
  return run_batch(p, n, nthreads);
}
