// TEST INFRASTRUCTURE ONLY: an independent cross-check of whole TLS-mode batches against
// OpenSSL 3 libcrypto (EVP AEADs), multithreaded so that full BASELINE batches (1-2 GiB) can be
// compared record by record in seconds. Never linked into the product.
//
// Record semantics are those of net/record.rs:162-198 (RecordPayloadProtection::encrypt) with the
// engine's TLS-mode descriptors (include/atls.h atls_rec):
//   inner = content (len B) || content_type, AAD = [0x17, 3, 3, (len+17) >> 8, (len+17) & 255],
//   nonce = static_iv ^ (0^4 || be64(seq))  (key_schedule.rs:51-64),
//   ciphertext (len + 1 B) at out + out_off, tag at tags + 16 * i.
// OpenSSL is a valid oracle for AES-GCM with 96-bit IVs and for ChaCha20-Poly1305
// only where the reference's last-block quirk does not fire (AEAD length % 64 != 0):
// such records are reported in `skipped` (1) and must be checked against the oracle instead.
#include <openssl/evp.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {  // = atls_key
  uint16_t suite;
  uint8_t key_len, iv_len;
  uint8_t key[32];
  uint8_t static_iv[12];
  uint8_t reserved[16];
} xc_key;

typedef struct {  // = atls_rec
  uint64_t in_off, out_off, aux_off, seq;
  uint32_t len, key_slot;
  uint16_t aad_len;
  uint8_t content_type, mode, iv_len, reserved[3];
} xc_rec;

typedef struct {
  const xc_key* keys;
  const xc_rec* recs;
  uint32_t lo, hi;
  const uint8_t* in;
  uint8_t* out;
  uint8_t* tags;
  uint8_t* skipped;
  int rc;
} job;

static const EVP_CIPHER* pick(const xc_key* k) {
  if (k->suite == 0x1303) return EVP_chacha20_poly1305();
  return k->key_len == 16 ? EVP_aes_128_gcm() : k->key_len == 24 ? EVP_aes_192_gcm() : EVP_aes_256_gcm();
}

static int seal_one(EVP_CIPHER_CTX* ctx, const xc_key* k, const xc_rec* r, const uint8_t* in, uint8_t* out,
                    uint8_t* tag) {
  uint8_t nonce[12];
  memcpy(nonce, k->static_iv, 12);
  for (int i = 0; i < 8; i++) nonce[4 + i] ^= (uint8_t)(r->seq >> (56 - 8 * i));
  const uint32_t L = r->len + 1u + 16u;
  const uint8_t aad[5] = {0x17, 3, 3, (uint8_t)(L >> 8), (uint8_t)L};
  int outl = 0;
  if (EVP_EncryptInit_ex(ctx, pick(k), NULL, NULL, NULL) != 1) return -1;
  if (EVP_CIPHER_CTX_ctrl(ctx, EVP_CTRL_AEAD_SET_IVLEN, 12, NULL) != 1) return -1;
  if (EVP_EncryptInit_ex(ctx, NULL, NULL, k->key, nonce) != 1) return -1;
  if (EVP_EncryptUpdate(ctx, NULL, &outl, aad, 5) != 1) return -1;
  if (r->len && EVP_EncryptUpdate(ctx, out, &outl, in, (int)r->len) != 1) return -1;
  int o2 = 0;
  if (EVP_EncryptUpdate(ctx, out + r->len, &o2, &r->content_type, 1) != 1) return -1;
  if (EVP_EncryptFinal_ex(ctx, out + r->len + 1, &o2) != 1) return -1;
  return EVP_CIPHER_CTX_ctrl(ctx, EVP_CTRL_AEAD_GET_TAG, 16, tag) == 1 ? 0 : -1;
}

static void* run(void* p) {
  job* j = (job*)p;
  EVP_CIPHER_CTX* ctx = EVP_CIPHER_CTX_new();
  j->rc = ctx ? 0 : -1;
  for (uint32_t i = j->lo; i < j->hi && !j->rc; i++) {
    const xc_rec* r = &j->recs[i];
    const xc_key* k = &j->keys[r->key_slot];
    const int quirk = k->suite == 0x1303 && (r->len + 1u) % 64u == 0u;  // chacha20/cipher.rs:99-102
    j->skipped[i] = (uint8_t)quirk;
    if (quirk) continue;
    j->rc = seal_one(ctx, k, r, j->in + r->in_off, j->out + r->out_off, j->tags + 16ull * i);
  }
  if (ctx) EVP_CIPHER_CTX_free(ctx);
  return NULL;
}

// Seal n TLS-mode records with OpenSSL. Returns 0, or -1 if OpenSSL failed.
int xc_seal_tls_batch(const xc_key* keys, const xc_rec* recs, uint32_t n, const uint8_t* in, uint8_t* out,
                      uint8_t* tags, uint8_t* skipped, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  if ((uint32_t)nthreads > n) nthreads = n ? (int)n : 1;
  job* jobs = (job*)calloc((size_t)nthreads, sizeof(job));
  pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
  if (!jobs || !th) return -1;
  for (int t = 0; t < nthreads; t++) {
    jobs[t] = (job){keys, recs, (uint32_t)((uint64_t)n * t / nthreads), (uint32_t)((uint64_t)n * (t + 1) / nthreads),
                    in, out, tags, skipped, 0};
    pthread_create(&th[t], NULL, run, &jobs[t]);
  }
  int rc = 0;
  for (int t = 0; t < nthreads; t++) {
    pthread_join(th[t], NULL);
    rc |= jobs[t].rc;
  }
  free(jobs);
  free(th);
  return rc;
}
