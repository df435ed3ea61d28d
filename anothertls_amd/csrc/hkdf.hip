// The hash side of the path on the device: SHA-256 / SHA-384
// (hash/sha256.rs, sha384.rs), HMAC (hash/hmac.rs:29-78), HKDF extract / expand (hash/hkdf.rs:24-65),
// the TLS 1.3 secret chain (KeySchedule::do_key_schedule, net/key_schedule.rs:170-222, and the
// application secrets, :87-114) and traffic-key derivation (Key::from_hkdf, :40-50) straight
// into atls_key slots for atls_set_keys. One thread per item (connection): this runs a few
// times per connection, not per record.
#include "atls_dev.h"

namespace atls {

__constant__ const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

__constant__ const uint64_t K512[80] = {
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

__device__ inline uint32_t rr32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
__device__ inline uint64_t rr64(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }

__device__ void sha256_block(uint32_t st[8], const uint8_t* p) {
  uint32_t w[64];
  for (int t = 0; t < 16; t++)
    w[t] = ((uint32_t)p[4 * t] << 24) | ((uint32_t)p[4 * t + 1] << 16) | ((uint32_t)p[4 * t + 2] << 8) | p[4 * t + 3];
  for (int t = 16; t < 64; t++) {
    uint32_t s0 = rr32(w[t - 15], 7) ^ rr32(w[t - 15], 18) ^ (w[t - 15] >> 3);
    uint32_t s1 = rr32(w[t - 2], 17) ^ rr32(w[t - 2], 19) ^ (w[t - 2] >> 10);
    w[t] = w[t - 16] + s0 + w[t - 7] + s1;
  }
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
  for (int t = 0; t < 64; t++) {
    uint32_t t1 = h + (rr32(e, 6) ^ rr32(e, 11) ^ rr32(e, 25)) + ((e & f) ^ (~e & g)) + K256[t] + w[t];
    uint32_t t2 = (rr32(a, 2) ^ rr32(a, 13) ^ rr32(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
    h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

__device__ void sha384_block(uint64_t st[8], const uint8_t* p) {
  uint64_t w[80];
  for (int t = 0; t < 16; t++) {
    uint64_t v = 0;
    for (int j = 0; j < 8; j++) v = (v << 8) | p[8 * t + j];
    w[t] = v;
  }
  for (int t = 16; t < 80; t++) {
    uint64_t s0 = rr64(w[t - 15], 1) ^ rr64(w[t - 15], 8) ^ (w[t - 15] >> 7);
    uint64_t s1 = rr64(w[t - 2], 19) ^ rr64(w[t - 2], 61) ^ (w[t - 2] >> 6);
    w[t] = w[t - 16] + s0 + w[t - 7] + s1;
  }
  uint64_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
  for (int t = 0; t < 80; t++) {
    uint64_t t1 = h + (rr64(e, 14) ^ rr64(e, 18) ^ rr64(e, 41)) + ((e & f) ^ (~e & g)) + K512[t] + w[t];
    uint64_t t2 = (rr64(a, 28) ^ rr64(a, 34) ^ rr64(a, 39)) + ((a & b) ^ (a & c) ^ (b & c));
    h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

// ---- streaming SHA-256 / SHA-384 (hash/sha256.rs, hash/sha384.rs) ----------------------------
// One thread per message. The reference pads with 0x80, zeros and the bit length written into only
// 7 (SHA-256, sha256.rs:60-62) or 15 (SHA-384) of the 8 / 16 length bytes; below 2^56 bits that is
// the standard length field, which is what this writes.
struct ShaCtx {
  int hl;  // 32 (SHA-256) or 48 (SHA-384)
  uint32_t s32[8];
  uint64_t s64[8];
  uint8_t buf[128];
  uint32_t blen;
  uint64_t total;
};

__device__ void sha_init(ShaCtx& c, int hl) {
  c.hl = hl;
  c.blen = 0;
  c.total = 0;
  if (hl == 32) {
    const uint32_t iv[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    for (int i = 0; i < 8; i++) c.s32[i] = iv[i];
  } else {
    const uint64_t iv[8] = {0xcbbb9d5dc1059ed8ull, 0x629a292a367cd507ull, 0x9159015a3070dd17ull, 0x152fecd8f70e5939ull,
                            0x67332667ffc00b31ull, 0x8eb44a8768581511ull, 0xdb0c2e0d64f98fa7ull, 0x47b5481dbefa4fa4ull};
    for (int i = 0; i < 8; i++) c.s64[i] = iv[i];
  }
}

__device__ void sha_update(ShaCtx& c, const uint8_t* p, uint64_t n) {
  const uint32_t bs = c.hl == 48 ? 128u : 64u;
  c.total += n;
  for (uint64_t i = 0; i < n; i++) {
    c.buf[c.blen++] = p[i];
    if (c.blen == bs) {
      if (c.hl == 32) sha256_block(c.s32, c.buf);
      else sha384_block(c.s64, c.buf);
      c.blen = 0;
    }
  }
}

__device__ void sha_final(ShaCtx& c, uint8_t* out) {
  const uint32_t bs = c.hl == 48 ? 128u : 64u, lb = bs == 128 ? 16u : 8u;
  const uint64_t bits = c.total * 8;
  uint8_t pad[144];
  const uint32_t used = c.blen;
  const uint32_t padn = (used + 1 + lb <= bs) ? bs - used : 2 * bs - used;
  for (uint32_t i = 0; i < padn; i++) pad[i] = 0;
  pad[0] = 0x80;
  for (int i = 0; i < 8; i++) pad[padn - 1 - i] = (uint8_t)(bits >> (8 * i));
  const uint64_t keep = c.total;
  sha_update(c, pad, padn);
  c.total = keep;
  if (c.hl == 32) {
    for (int i = 0; i < 32; i++) out[i] = (uint8_t)(c.s32[i >> 2] >> (8 * (3 - (i & 3))));
  } else {
    for (int i = 0; i < 48; i++) out[i] = (uint8_t)(c.s64[i >> 3] >> (8 * (7 - (i & 7))));
  }
}

__device__ void sha_x(int hl, const uint8_t* m, uint64_t len, uint8_t* out) {  // hash/mod.rs:37-42
  ShaCtx c;
  sha_init(c, hl);
  sha_update(c, m, len);
  sha_final(c, out);
}

// HMAC (hash/hmac.rs:29-78) over the concatenation of up to three message parts. Keys longer than
// 64 bytes are hashed first for BOTH hashes (hmac.rs:41-49), which differs from RFC 2104 for
// SHA-384 keys of 65..128 bytes; the padded key is 64 (SHA-256) or 128 (SHA-384) bytes.
__device__ void hmac_parts(int hl, const uint8_t* key, uint64_t klen, const uint8_t* m0, uint64_t l0, const uint8_t* m1,
                           uint64_t l1, const uint8_t* m2, uint64_t l2, uint8_t* out) {
  const uint32_t size = hl == 48 ? 128u : 64u;
  uint8_t kb[128], hk[48];
  if (klen > 64) {
    sha_x(hl, key, klen, hk);
    key = hk;
    klen = (uint64_t)hl;
  }
  for (uint32_t i = 0; i < size; i++) kb[i] = (i < klen ? key[i] : 0) ^ 0x36;
  ShaCtx c;
  sha_init(c, hl);
  sha_update(c, kb, size);
  sha_update(c, m0, l0);
  sha_update(c, m1, l1);
  sha_update(c, m2, l2);
  uint8_t inner[48];
  sha_final(c, inner);
  for (uint32_t i = 0; i < size; i++) kb[i] ^= 0x36 ^ 0x5c;
  sha_init(c, hl);
  sha_update(c, kb, size);
  sha_update(c, inner, (uint64_t)hl);
  sha_final(c, out);
}

// HKDF-Expand (hash/hkdf.rs:35-65): T(i) = HMAC(PRK, T(i-1) || info || i) with a u8 counter,
// out_len <= 255 * HashLen (checked by the caller).
__device__ void hkdf_expand(int hl, const uint8_t* prk, uint64_t prk_len, const uint8_t* info, uint64_t info_len,
                            uint8_t* out, uint32_t out_len) {
  uint8_t t[48];
  uint32_t got = 0, tl = 0;
  uint8_t i = 0;
  while (got < out_len) {
    i++;
    hmac_parts(hl, prk, prk_len, t, tl, info, info_len, &i, 1, t);
    tl = (uint32_t)hl;
    const uint32_t need = min(out_len - got, (uint32_t)hl);
    for (uint32_t j = 0; j < need; j++) out[got + j] = t[j];
    got += need;
  }
}

// get_hkdf_expand_label (net/key_schedule.rs:20-29): {len_hi, len_lo, 6 + |label|, "tls13 " label,
// |ctx|, ctx}. Returns the length.
__device__ uint32_t expand_label_info(const char* label, uint32_t llen, const uint8_t* ctx, uint32_t clen, uint32_t L,
                                      uint8_t* info) {
  uint32_t p = 0;
  info[p++] = (uint8_t)(L >> 8);
  info[p++] = (uint8_t)L;
  info[p++] = (uint8_t)(6 + llen);
  const char* pre = "tls13 ";
  for (int i = 0; i < 6; i++) info[p++] = (uint8_t)pre[i];
  for (uint32_t i = 0; i < llen; i++) info[p++] = (uint8_t)label[i];
  info[p++] = (uint8_t)clen;
  for (uint32_t i = 0; i < clen; i++) info[p++] = ctx[i];
  return p;
}

__device__ void expand_label(int hl, const uint8_t* secret, const char* label, uint32_t llen, const uint8_t* ctx,
                             uint32_t clen, uint32_t L, uint8_t* out) {
  uint8_t info[128];
  const uint32_t il = expand_label_info(label, llen, ctx, clen, L, info);
  hkdf_expand(hl, secret, (uint64_t)hl, info, il, out, L);
}

__global__ void derive_kernel(uint16_t suite, const uint8_t* __restrict__ secrets, uint32_t hl, uint32_t n,
                              atls_key* __restrict__ out) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint8_t* sec = secrets + (size_t)i * hl;
  atls_key k;
  for (int b = 0; b < (int)sizeof(k); b++) reinterpret_cast<uint8_t*>(&k)[b] = 0;
  k.suite = suite;
  k.key_len = suite == kSuiteAes128 ? 16 : 32;  // CipherSuite::get_key_and_iv_len, ciphersuite.rs:69-77
  k.iv_len = 12;
  expand_label((int)hl, sec, "key", 3, nullptr, 0, k.key_len, k.key);  // Key::from_hkdf, key_schedule.rs:40-50
  expand_label((int)hl, sec, "iv", 2, nullptr, 0, 12, k.static_iv);
  out[i] = k;
}

// Batched hashing primitives (include/atls.h atls_hash_batch): item i hashes data + msg[i] (and
// keys with data + key[i]); output at out + i * out_len.
__global__ void hash_kernel(int op, uint32_t hl, const uint8_t* __restrict__ data, const atls_span* __restrict__ keys,
                            const atls_span* __restrict__ msgs, uint32_t n, uint32_t out_len, uint8_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const atls_span m = msgs[i];
  uint8_t* o = out + (size_t)i * out_len;
  if (op == ATLS_HASH_SHA) {
    sha_x((int)hl, data + m.off, m.len, o);
    return;
  }
  const atls_span k = keys[i];
  if (op == ATLS_HASH_HKDF_EXPAND) {
    hkdf_expand((int)hl, data + k.off, k.len, data + m.off, m.len, o, out_len);
    return;
  }
  // HMAC(key, msg); HKDF-Extract(salt, ikm) = HMAC(salt, ikm) (hash/hkdf.rs:24-32)
  hmac_parts((int)hl, data + k.off, k.len, data + m.off, m.len, nullptr, 0, nullptr, 0, o);
}

// KeySchedule::do_key_schedule (net/key_schedule.rs:170-222) from the (EC)DHE shared secret and
// the ClientHello..ServerHello transcript hash, then the application traffic secrets
// (WriteKeys::application_keys_from_master_secret, :87-114) from the ..server Finished hash. One
// thread per connection; out = {c hs, s hs, master, c ap, s ap} traffic secrets, HashLen each.
__global__ void key_schedule_kernel(uint32_t hl, const uint8_t* __restrict__ shared, uint32_t shared_len,
                                    const uint8_t* __restrict__ hello, const uint8_t* __restrict__ fin, uint32_t n,
                                    uint8_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int h = (int)hl;
  uint8_t zeros[48], empty_hash[48], early[48], derived[48], hs[48];
  for (int j = 0; j < 48; j++) zeros[j] = 0;
  sha_x(h, zeros, 0, empty_hash);
  uint8_t* o = out + (size_t)i * 5 * hl;
  hmac_parts(h, zeros, hl, zeros, hl, nullptr, 0, nullptr, 0, early);                 // Early Secret
  expand_label(h, early, "derived", 7, empty_hash, hl, hl, derived);
  hmac_parts(h, derived, hl, shared + (size_t)i * shared_len, shared_len, nullptr, 0, nullptr, 0, hs);  // Handshake
  const uint8_t* hh = hello + (size_t)i * hl;
  expand_label(h, hs, "c hs traffic", 12, hh, hl, hl, o);
  expand_label(h, hs, "s hs traffic", 12, hh, hl, hl, o + hl);
  expand_label(h, hs, "derived", 7, empty_hash, hl, hl, derived);
  hmac_parts(h, derived, hl, zeros, hl, nullptr, 0, nullptr, 0, o + 2 * hl);          // Master Secret
  if (fin) {
    const uint8_t* fh = fin + (size_t)i * hl;
    expand_label(h, o + 2 * hl, "c ap traffic", 12, fh, hl, hl, o + 3 * hl);
    expand_label(h, o + 2 * hl, "s ap traffic", 12, fh, hl, hl, o + 4 * hl);
  }
}

}  // namespace atls

extern "C" int atls_launch_hash(int op, uint32_t hl, const uint8_t* data, const atls_span* keys, const atls_span* msgs,
                                uint32_t n, uint32_t out_len, uint8_t* out, hipStream_t s) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(atls::hash_kernel, dim3((n + 63) / 64), dim3(64), 0, s, op, hl, data, keys, msgs, n, out_len, out);
  return hipGetLastError() == hipSuccess ? 0 : ATLS_INTERNAL_ERROR;
}

extern "C" int atls_launch_key_schedule(uint32_t hl, const uint8_t* shared, uint32_t shared_len, const uint8_t* hello,
                                        const uint8_t* fin, uint32_t n, uint8_t* out, hipStream_t s) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(atls::key_schedule_kernel, dim3((n + 63) / 64), dim3(64), 0, s, hl, shared, shared_len, hello, fin,
                     n, out);
  return hipGetLastError() == hipSuccess ? 0 : ATLS_INTERNAL_ERROR;
}

extern "C" int atls_launch_derive(uint16_t suite, const uint8_t* secrets, uint32_t secret_len, uint32_t n,
                                  atls_key* out, hipStream_t s) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(atls::derive_kernel, dim3((n + 63) / 64), dim3(64), 0, s, suite, secrets, secret_len, n, out);
  return hipGetLastError() == hipSuccess ? 0 : ATLS_INTERNAL_ERROR;
}
