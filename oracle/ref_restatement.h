/*
 * TEST INFRASTRUCTURE ONLY — the parity oracle for anothertls_amd.
 *
 * A literal CPU restatement (plain C) of otsmr/AnotherTLS v0.1.3's record-layer
 * AEAD path, quirks included. Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library; the product path (anothertls_amd/libatls.so)
 * never links, loads or calls it.
 *
 * Pinned by the reference's own known-answer tests (tests/golden/reference_kats.json,
 * transcribed from the #[cfg(test)] modules cited there) and cross-checked against
 * OpenSSL 3 libcrypto where the reference is standard.
 *
 * The reference (Rust, + ibig 0.3.6 for Poly1305 bignums) cannot be compiled in this
 * image (no cargo/rustc), so oracle/_ref is not built; see DESIGN.md §Oracle.
 */
#ifndef ATLS_REF_RESTATEMENT_H
#define ATLS_REF_RESTATEMENT_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* TlsError codes, anothertls/src/net/alert.rs:18-45 */
enum {
  ORA_OK = 0,
  ORA_BAD_RECORD_MAC = 20,
  ORA_ILLEGAL_PARAMETER = 47, /* documented divergence: the reference panics */
  ORA_DECRYPT_ERROR = 50,
  ORA_DECODE_ERROR = 51,
  ORA_INSUFFICIENT_SECURITY = 71,
  ORA_INTERNAL_ERROR = 80,
};

enum { ORA_SHA256 = 32, ORA_SHA384 = 48 }; /* hash/mod.rs:18-21 */

/* crypto/aes/cipher.rs */
int ora_aes_encrypt_block(const uint8_t* key, size_t key_len, const uint8_t in[16], uint8_t out[16]);
int ora_aes_decrypt_block(const uint8_t* key, size_t key_len, const uint8_t in[16], uint8_t out[16]);
int ora_aes_expand_key(const uint8_t* key, size_t key_len, uint8_t out[240]);

/* crypto/aes/gcm.rs */
int ora_gcm_encrypt(const uint8_t* key, size_t key_len, const uint8_t* iv, size_t iv_len,
                    const uint8_t* pt, size_t n, const uint8_t* aad, size_t m,
                    uint8_t* ct, uint8_t tag[16]);
int ora_gcm_decrypt(const uint8_t* key, size_t key_len, const uint8_t* iv, size_t iv_len,
                    const uint8_t* ct, size_t n, const uint8_t* aad, size_t m,
                    const uint8_t* tag, size_t tag_len, uint8_t* pt);
void ora_gcm_gmult(const uint8_t a[16], const uint8_t b[16], uint8_t out[16]);

/* crypto/chacha20/cipher.rs */
void ora_chacha20_block(const uint8_t key[32], const uint8_t iv[12], uint32_t counter, uint8_t out[64]);
int ora_chacha20_encrypt(const uint8_t* in, size_t len, const uint8_t* key, size_t key_len,
                         const uint8_t* iv, size_t iv_len, size_t counter, uint8_t* out);

/* crypto/chacha20/poly1305.rs */
void ora_poly1305_mac(const uint8_t key[32], const uint8_t* msg, size_t len, uint8_t tag[16]);
int ora_poly1305_key_gen(const uint8_t* key, size_t key_len, const uint8_t* iv, size_t iv_len, uint8_t otk[32]);
int ora_chacha_poly_encrypt(const uint8_t* key, size_t key_len, const uint8_t* iv, size_t iv_len,
                            const uint8_t* pt, size_t n, const uint8_t* aad, size_t m,
                            uint8_t* ct, uint8_t tag[16]);
int ora_chacha_poly_decrypt(const uint8_t* key, size_t key_len, const uint8_t* iv, size_t iv_len,
                            const uint8_t* ct, size_t n, const uint8_t* aad, size_t m,
                            const uint8_t* tag, size_t tag_len, uint8_t* pt);

/* crypto/ciphersuite.rs: Cipher::encrypt / decrypt through get_cipher() */
int ora_cipher_encrypt(uint16_t suite, const uint8_t* key, size_t key_len, const uint8_t* iv,
                       size_t iv_len, const uint8_t* pt, size_t n, const uint8_t* aad, size_t m,
                       uint8_t* ct, uint8_t tag[16]);
int ora_cipher_decrypt(uint16_t suite, const uint8_t* key, size_t key_len, const uint8_t* iv,
                       size_t iv_len, const uint8_t* ct, size_t n, const uint8_t* aad, size_t m,
                       const uint8_t* tag, size_t tag_len, uint8_t* pt);

/* hash/ */
void ora_sha256(const uint8_t* msg, size_t len, uint8_t out[32]);
void ora_sha384(const uint8_t* msg, size_t len, uint8_t out[48]);
void ora_hmac(int hash, const uint8_t* key, size_t key_len, const uint8_t* msg, size_t len, uint8_t* out);
void ora_hkdf_extract(int hash, const uint8_t* salt, size_t salt_len, const uint8_t* ikm, size_t ikm_len, uint8_t* prk);
int ora_hkdf_expand(int hash, const uint8_t* prk, size_t prk_len, const uint8_t* info, size_t info_len,
                    uint8_t* okm, size_t out_len);

/* net/key_schedule.rs */
size_t ora_hkdf_expand_label(const uint8_t* label, size_t label_len, const uint8_t* ctx, size_t ctx_len,
                             size_t out_len, uint8_t* buf);
int ora_key_from_secret(int hash, const uint8_t* secret, size_t secret_len, size_t key_len, size_t iv_len,
                        uint8_t* key, uint8_t* iv);
int ora_key_schedule(int hash, const uint8_t* shared, size_t shared_len, const uint8_t* hello_hash,
                     const uint8_t* handshake_hash, uint8_t* out);
void ora_per_record_nonce(const uint8_t iv[12], uint64_t seq, uint8_t out[12]);

/* net/record.rs: RecordPayloadProtection::encrypt / decrypt for one record */
int ora_record_seal(uint16_t suite, const uint8_t* key, size_t key_len, const uint8_t iv[12], uint64_t seq,
                    uint8_t content_type, const uint8_t* frag, size_t frag_len, uint8_t* wire, size_t* wire_len);
int ora_record_open(uint16_t suite, const uint8_t* key, size_t key_len, const uint8_t iv[12], uint64_t seq,
                    const uint8_t* wire, size_t wire_len, uint8_t* content, size_t* content_len,
                    uint8_t* content_type);

/* Batch form used by the parity tests and the CPU baseline: the same descriptors the
 * engine takes (include/atls.h), sealed one record at a time through the literal
 * restatement. nthreads > 1 splits records over pthreads. */
typedef struct {
  uint16_t suite;
  uint8_t key_len;
  uint8_t iv_len;
  uint8_t key[32];
  uint8_t static_iv[12];
  uint8_t reserved[16];
} ora_key;

typedef struct {
  uint64_t in_off;
  uint64_t out_off;
  uint64_t aux_off;
  uint64_t seq;
  uint32_t len;
  uint32_t key_slot;
  uint16_t aad_len;
  uint8_t content_type;
  uint8_t mode; /* 0 TLS, 1 RAW, 2 WIRE (TLS with header || ct || tag framed in the buffer) */
  uint8_t iv_len;
  uint8_t reserved[3];
} ora_rec;

int ora_seal_batch(const ora_key* keys, const ora_rec* recs, uint32_t n, const uint8_t* in,
                   const uint8_t* aux, uint8_t* out, uint8_t* tags, int nthreads);
typedef struct {
  uint32_t content_len; /* TLS mode: record_len after the zero-padding scan (record.rs:229-237) */
  uint8_t status;       /* 0, or TlsError code */
  uint8_t content_type; /* TLS mode: inner content type (0 = RecordType::Invalid) */
  uint8_t reserved[2];
} ora_open_result;

int ora_open_batch(const ora_key* keys, const ora_rec* recs, uint32_t n, const uint8_t* in,
                   const uint8_t* aux, const uint8_t* tags, uint8_t* out, ora_open_result* res,
                   int nthreads);

#ifdef __cplusplus
}
#endif
#endif
