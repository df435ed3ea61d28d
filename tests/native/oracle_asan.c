/* TEST INFRASTRUCTURE ONLY: the oracle (oracle/ref_restatement.c) exercised under ASan / UBSan on
 * the CPU: every entry point over edge and random lengths (ChaCha20 last-block quirk lengths,
 * non-96-bit GCM IVs, AES-192, HMAC keys around 64 / 128 bytes, HKDF up to 255 * HashLen, record
 * seal / open with tampered bytes, threaded batches). Round trips are asserted; memory and UB
 * errors abort through the sanitizers. Exit 0 = clean. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../oracle/ref_restatement.h"

static unsigned long long rng = 0x9E3779B97F4A7C15ull;
static unsigned rnd(void) {
  rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17;
  return (unsigned)(rng >> 11);
}
static void fill(uint8_t* p, size_t n) { for (size_t i = 0; i < n; i++) p[i] = (uint8_t)rnd(); }
#define CHECK(c) do { if (!(c)) { fprintf(stderr, "check failed %s:%d %s\n", __FILE__, __LINE__, #c); return 1; } } while (0)

int main(void) {
  static const size_t lens[] = {0, 1, 15, 16, 17, 63, 64, 65, 127, 128, 129, 1535, 1536, 1537, 4096, 16383, 16384, 16385};
  uint8_t key[32], iv[64], aad[40], tag[16], tag2[16];
  uint8_t *pt = malloc(16400), *ct = malloc(16400), *back = malloc(16400);
  for (size_t li = 0; li < sizeof lens / sizeof lens[0]; li++) {
    const size_t n = lens[li];
    fill(pt, n); fill(key, 32); fill(iv, 64); fill(aad, 40);
    const size_t kls[3] = {16, 24, 32}, ivls[4] = {12, 1, 8, 60};
    for (int k = 0; k < 3; k++) for (int v = 0; v < 4; v++) {
      const size_t al = rnd() % 41;
      CHECK(ora_gcm_encrypt(key, kls[k], iv, ivls[v], pt, n, aad, al, ct, tag) == 0);
      CHECK(ora_gcm_decrypt(key, kls[k], iv, ivls[v], ct, n, aad, al, tag, 16, back) == 0);
      CHECK(n == 0 || memcmp(back, pt, n) == 0);
      memcpy(tag2, tag, 16); tag2[3] ^= 1;
      CHECK(ora_gcm_decrypt(key, kls[k], iv, ivls[v], ct, n, aad, al, tag2, 16, back) != 0);
    }
    CHECK(ora_chacha_poly_encrypt(key, 32, iv, 12, pt, n, aad, 13, ct, tag) == 0);
    CHECK(ora_chacha_poly_decrypt(key, 32, iv, 12, ct, n, aad, 13, tag, 16, back) == 0);
    CHECK(n == 0 || memcmp(back, pt, n) == 0);
    CHECK(ora_chacha_poly_decrypt(key, 32, iv, 12, ct, n, aad, 13, tag, 15, back) != 0);  /* short tag */
    for (int suite = 0x1301; suite <= 0x1303; suite++) {
      uint8_t* wire = malloc(n + 1 + 5 + 16);
      uint8_t* content = malloc(n + 1 + 16);
      size_t wl = 0, cl = 0;
      uint8_t ctype = 0;
      const size_t kl = suite == 0x1301 ? 16 : 32;
      CHECK(ora_record_seal((uint16_t)suite, key, kl, iv, 77, 23, pt, n, wire, &wl) == 0);
      CHECK(ora_record_open((uint16_t)suite, key, kl, iv, 77, wire, wl, content, &cl, &ctype) == 0);
      wire[5 + rnd() % (wl - 5)] ^= 0x40;
      (void)ora_record_open((uint16_t)suite, key, kl, iv, 77, wire, wl, content, &cl, &ctype);
      (void)ora_record_open((uint16_t)suite, key, kl, iv, 77, wire, rnd() % (wl + 1), content, &cl, &ctype);
      free(wire); free(content);
    }
  }
  /* hashes: message lengths around block sizes, HMAC keys around 64 / 128, HKDF lengths */
  uint8_t msg[300], out[48 * 255], prk[48];
  for (int hl = 32; hl <= 48; hl += 16)
    for (size_t m = 0; m < 300; m += 7) {
      fill(msg, m);
      ora_sha256(msg, m, out); ora_sha384(msg, m, out);
      ora_hmac(hl, msg, m, msg, 300 - m, out);
      ora_hkdf_extract(hl, msg, m % 130, msg, m, prk);
      CHECK(ora_hkdf_expand(hl, prk, (size_t)hl, msg, m % 100, out, (size_t)hl * (m % 256)) == ((m % 256) > 255 ? -1 : 0));
    }
  CHECK(ora_hkdf_expand(32, prk, 32, msg, 10, out, 32 * 256) == -1);
  uint8_t secrets[5 * 48], kk[32], kiv[12];
  CHECK(ora_key_schedule(48, msg, 32, msg + 32, msg + 80, secrets) == 0);
  CHECK(ora_key_from_secret(48, secrets, 48, 32, 12, kk, kiv) == 0);
  /* threaded batch over mixed suites and lengths */
  enum { N = 64 };
  ora_key keys[3];
  memset(keys, 0, sizeof keys);
  for (int i = 0; i < 3; i++) {
    keys[i].suite = (uint16_t)(0x1301 + i); keys[i].key_len = i == 0 ? 16 : 32; keys[i].iv_len = 12;
    fill(keys[i].key, 32); fill(keys[i].static_iv, 12);
  }
  ora_rec recs[N];
  memset(recs, 0, sizeof recs);
  size_t io = 0, oo = 0;
  for (int i = 0; i < N; i++) {
    recs[i].len = rnd() % 3000; recs[i].key_slot = (uint32_t)(i % 3); recs[i].seq = (uint64_t)i; recs[i].content_type = 23;
    recs[i].in_off = io; recs[i].out_off = oo; io += recs[i].len + 16; oo += recs[i].len + 17;
  }
  uint8_t *in = malloc(io + 16), *bo = malloc(oo + 16), *tags = malloc(16 * N), *pt2 = malloc(oo + 16);
  fill(in, io);
  CHECK(ora_seal_batch(keys, recs, N, in, aad, bo, tags, 4) == 0);
  ora_rec orecs[N];
  memcpy(orecs, recs, sizeof recs);
  for (int i = 0; i < N; i++) { orecs[i].in_off = recs[i].out_off; orecs[i].len = recs[i].len + 1; }
  ora_open_result res[N];
  CHECK(ora_open_batch(keys, orecs, N, bo, aad, tags, pt2, res, 4) == 0);
  for (int i = 0; i < N; i++) CHECK(res[i].status == 0 && res[i].content_len == recs[i].len);
  free(in); free(bo); free(tags); free(pt2); free(pt); free(ct); free(back);
  printf("oracle under sanitizers: OK\n");
  return 0;
}
