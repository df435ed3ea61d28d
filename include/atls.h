/*
 * anothertls_amd — MI355X-native TLS 1.3 record-layer AEAD engine. C ABI.
 *
 * This is the drop-in boundary for otsmr/AnotherTLS's per-record bulk AEAD path
 * (paths relative to /root/reference/anothertls/src):
 *
 *   trait Cipher { encrypt(&self,key,iv,plaintext,aad) -> Result<(Vec<u8>,[u8;16]),TlsError>;
 *                  decrypt(&self,key,iv,ciphertext,aad,auth_tag) -> Result<Vec<u8>,TlsError>; }
 *     crypto/ciphersuite.rs:12-31, produced by CipherSuite::get_cipher() :78-87 and called only from
 *     RecordPayloadProtection::encrypt / decrypt (net/record.rs:191-193, :217-220).
 *
 * atls_seal / atls_open replace Cipher::encrypt / Cipher::decrypt one call at a time.
 * The engine API (atls_engine_*, atls_*_batch) is the batched form a record layer uses to put
 * many records (one connection's fragments, or many connections) into one device launch:
 * TLS mode derives the inner plaintext (content || content_type, record.rs:172-173), the
 * 5-byte AAD header (record.rs:175-183) and the per-record nonce (key_schedule.rs:51-64)
 * on the device; RAW mode takes nonce and AAD verbatim (the Cipher trait's contract).
 *
 * Rules: plain C types only; caller-owned buffers; nothing unwinds across this boundary;
 * every entry point returns 0 or a TlsError code (net/alert.rs:18-45). Where the reference
 * panics (bad key/IV sizes, short fragments) we return ATLS_ILLEGAL_PARAMETER or
 * ATLS_DECODE_ERROR instead (documented divergence).
 * All computation runs on the GPU (gfx950); without a usable HIP device every compute
 * entry point returns ATLS_INTERNAL_ERROR (there is no CPU fallback).
 */
#ifndef ANOTHERTLS_AMD_ATLS_H
#define ANOTHERTLS_AMD_ATLS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ATLS_ABI_VERSION 1

/* Status codes = TlsError discriminants, net/alert.rs:18-45. */
enum {
  ATLS_OK = 0,
  ATLS_BAD_RECORD_MAC = 20,       /* tag mismatch in Cipher::decrypt (gcm.rs:150-154, poly1305.rs:93-98) */
  ATLS_ILLEGAL_PARAMETER = 47,    /* bad key / IV length (reference panics: gcm.rs:49, poly1305.rs:20) */
  ATLS_DECRYPT_ERROR = 50,        /* record layer's mapping of any cipher error (record.rs:222) */
  ATLS_DECODE_ERROR = 51,         /* bad inner content type (record.rs:232) / short record */
  ATLS_INSUFFICIENT_SECURITY = 71,/* unknown suite (ciphersuite.rs:50, :84) */
  ATLS_INTERNAL_ERROR = 80        /* no device, allocation or launch failure */
};

/* CipherSuite, crypto/ciphersuite.rs:33-40. 0x1301 and 0x1302 both map to AES-GCM whose key
 * size (128/192/256) is taken from key_len exactly as Gcm::gcm does (gcm.rs:49). */
enum {
  ATLS_TLS_AES_128_GCM_SHA256 = 0x1301,
  ATLS_TLS_AES_256_GCM_SHA384 = 0x1302,
  ATLS_TLS_CHACHA20_POLY1305_SHA256 = 0x1303
};

/* Record modes for the batch API. */
enum {
  ATLS_MODE_TLS = 0, /* seal: in = content (len B); AEAD input = content||content_type (len+1 B);
                        open: in = ciphertext (len B); AAD = [0x17,3,3,(len+16)>>8,(len+16)] for
                        both; nonce = static_iv ^ be64(seq). Open scans for the content type. */
  ATLS_MODE_RAW = 1, /* AEAD over len bytes; nonce (iv_len B) then AAD (aad_len B) read from
                        aux + aux_off; no framing. */
  ATLS_MODE_WIRE = 2 /* TLS mode with the record framing done on the device.
                        seal (RecordPayloadProtection::encrypt, record.rs:162-198): in = content
                        (len B); out + out_off receives the whole wire record, header || ct || tag
                        (5 + len + 1 + 16 B), header = [0x17,3,3,(len+17)>>8,(len+17)].
                        open (Record::from_raw + decrypt, record.rs:81-102, :201-240): in + in_off
                        is a wire record (5 + len + 16 B, len = ciphertext bytes); the received
                        header is the AAD verbatim and the tag is read from the record. A header
                        whose type is not a RecordType (record.rs:22-33) or whose length is not
                        len + 16 gives ATLS_DECODE_ERROR. out + out_off receives len B of inner
                        plaintext, scanned for the content type as in TLS mode.
                        The tags array is written on seal (a copy of the inline tag) and not read
                        on open; it may be NULL when every record of the batch is WIRE. */
};

/* Batch flags. */
enum {
  ATLS_FLAG_DEVICE_PTRS = 1u, /* in/aux/out/tags/results are device pointers (else host memory,
                                 staged through pinned buffers with async copies) */
  ATLS_FLAG_DEVICE_RECS = 2u, /* recs is a device pointer (keeps descriptors resident) */
  ATLS_FLAG_NO_SYNC = 4u,     /* return after enqueueing; call atls_engine_sync() before reading.
                                 A descriptor the device refuses (DEVICE_RECS) is then reported
                                 as ATLS_ILLEGAL_PARAMETER by that atls_engine_sync, or by any
                                 later synchronous call on the engine (the error word is sticky
                                 until a synchronous call reads it). */
  ATLS_FLAG_LAZY_JOIN = 8u    /* honoured only with NO_SYNC, DEVICE_PTRS, DEVICE_RECS and a caller tags
                                 array (the side kernel then reads no engine-owned buffer); otherwise the
                                 batch joins as usual. A mixed-suite batch's ChaCha20-Poly1305 kernel
                                 (second stream) is not joined back into the engine stream at the end of
                                 the batch; the next batch's plan and AES-GCM kernel may start beside it.
                                 The engine stream covers it again after atls_engine_join /
                                 atls_engine_sync, a batch without this flag, or a key-table update.
                                 Batches of one engine stay ordered per record kernel. */
};

/* One connection's write key (a "key slot"). 64 bytes. suite + key + static IV as produced by
 * Key::from_hkdf (key_schedule.rs:40-50). iv_len must be 12 (key_schedule.rs:44). */
typedef struct {
  uint16_t suite;
  uint8_t key_len;
  uint8_t iv_len;
  uint8_t key[32];
  uint8_t static_iv[12];
  uint8_t reserved[16];
} atls_key;

/* One record descriptor. 48 bytes. Offsets are byte offsets into the in/out/aux buffers;
 * the tag of record i lives at tags + 16*i. out may alias in (in-place). */
typedef struct {
  uint64_t in_off;
  uint64_t out_off;
  uint64_t aux_off;
  uint64_t seq; /* TLS mode: per-record sequence number (key_schedule.rs:51-64) */
  uint32_t len;
  uint32_t key_slot;
  uint16_t aad_len;      /* RAW mode */
  uint8_t content_type;  /* TLS seal: inner content type (record.rs:173) */
  uint8_t mode;          /* ATLS_MODE_* */
  uint8_t iv_len;        /* RAW mode nonce length (GCM accepts any length, gcm.rs:59-70) */
  uint8_t reserved[3];
} atls_rec;

/* Per-record open result. 8 bytes. */
typedef struct {
  uint32_t content_len; /* TLS: bytes before the content-type byte (record.rs:229-237); RAW: len */
  uint8_t status;       /* ATLS_OK, or TlsError code (TLS: 50 on tag failure, 51 bad type; RAW: 20) */
  uint8_t content_type; /* TLS: inner content type (0 = RecordType::Invalid, all-zero plaintext) */
  uint8_t reserved[2];
} atls_open_result;

typedef struct atls_engine atls_engine;

/* ---- Cipher-trait drop-in (crypto/ciphersuite.rs:12-31) ---------------------------------
 * atls_seal  <- Cipher::encrypt: out = ciphertext (len B), tag = 16 B.
 * atls_open  <- Cipher::decrypt: out = plaintext (len B) or ATLS_BAD_RECORD_MAC (a tag of the
 *               wrong length is a mismatch, as `T != auth_tag` is in the reference).
 * Host pointers; device 0 or $ATLS_DEVICE. Reentrant and concurrent (Cipher is Send + Sync): a call
 * leases one of at most $ATLS_SINGLE_CONTEXTS (8) call contexts -- engines, streams, a mapped pinned
 * block the kernel reads and writes in place -- and callers beyond that wait for one; a context keeps
 * the device key schedules of its last 16 keys per key size, so repeated keys cost no key setup.
 * $ATLS_SINGLE_RESIDENT=1 (opt-in): ChaCha20-Poly1305 calls whose IV || AAD || input fit 3,584 B go to one
 * workgroup that stays on the GPU and answers through a doorbell in mapped memory (no launch per call); =2:
 * AES-GCM calls too. The server leaves after $ATLS_SINGLE_RESIDENT_IDLE_MS (20) without a call, and the
 * process stops it before each launch of its own (a running kernel holds a hardware queue). */
int atls_seal(uint16_t suite, const uint8_t* key, size_t key_len, const uint8_t* iv, size_t iv_len,
              const uint8_t* aad, size_t aad_len, const uint8_t* in, size_t len, uint8_t* out,
              uint8_t tag[16]);
int atls_open(uint16_t suite, const uint8_t* key, size_t key_len, const uint8_t* iv, size_t iv_len,
              const uint8_t* aad, size_t aad_len, const uint8_t* in, size_t len, const uint8_t* tag,
              size_t tag_len, uint8_t* out);

/* ---- Engine ---------------------------------------------------------------------------- */
atls_engine* atls_engine_create(int device); /* NULL if the device is unusable */
void atls_engine_destroy(atls_engine* e);
/* Wait until everything enqueued on the engine has finished; reports a descriptor a NO_SYNC batch refused.
 * Waits on a completion flag a one-lane kernel writes into mapped memory after a system-scope release (which
 * also writes back the L2 lines the batch's kernels left, host-mapped outputs of DEVICE_PTRS batches
 * included), spinning for at most 100 us and then blocking in a stream synchronisation (env
 * ATLS_SYNC_FLAG=0: a stream synchronisation only). Synchronous batches return the same way; batches that
 * copy into host memory, or read and write page-locked host buffers in place (ATLS_ZERO_COPY), synchronise
 * the stream. */
int atls_engine_sync(atls_engine* e);
/* HIP stream the engine launches on (hipStream_t as void*), for callers that time or order work.
 * Work of ATLS_FLAG_LAZY_JOIN batches is on it only after atls_engine_join. */
void* atls_engine_stream(atls_engine* e);
/* Order the engine stream after every kernel of the batches issued so far (joins the side stream
 * of ATLS_FLAG_LAZY_JOIN batches; no host wait). */
int atls_engine_join(atls_engine* e);

/* Install n key slots (host array). Runs the device key-setup kernel: AES round keys, H = E_K(0),
 * H^1..H^64 and the GHASH table seeds; ChaCha keys are used as given. Replaces previous slots.
 * Up to 4 keys travel in the kernel's launch arguments and the call returns without waiting for the
 * kernel (every later batch of the engine is ordered after it); a fault of that kernel is then reported
 * by the next synchronous call or atls_engine_sync. More keys are staged by a copy and waited for. */
int atls_set_keys(atls_engine* e, const atls_key* keys, uint32_t n);
/* Install n key slots at [first, first + n) without touching the others (connections come and go);
 * first <= the current slot count (slots stay contiguous; the table grows as needed). Waits as
 * atls_set_keys does. */
int atls_update_keys(atls_engine* e, uint32_t first, const atls_key* keys, uint32_t n);

/* Seal / open n records. */
int atls_seal_batch(atls_engine* e, const atls_rec* recs, uint32_t n, const void* in, const void* aux,
                    void* out, uint8_t* tags, uint32_t flags);
int atls_open_batch(atls_engine* e, const atls_rec* recs, uint32_t n, const void* in, const void* aux,
                    const uint8_t* tags, void* out, atls_open_result* results, uint32_t flags);

/* Traffic-key derivation, Key::from_hkdf (key_schedule.rs:40-50): for each of n traffic
 * secrets (secret_len = 32 for SHA-256 suites, 48 for SHA-384), key = HKDF-Expand-Label(secret,
 * "key", "", key_len) and iv = HKDF-Expand-Label(secret, "iv", "", 12), written as atls_key
 * slots (suite, key_len from the suite: 0x1301 -> 16, 0x1302/0x1303 -> 32). Runs on the device. */
int atls_derive_keys(atls_engine* e, uint16_t suite, const uint8_t* secrets, size_t secret_len, uint32_t n,
                     atls_key* out_keys);

/* ---- Hashes on the device (hash/sha256.rs .. hkdf.rs; per connection, not per record) ------------------------
 * One batch item per message: item i reads data + msg[i].off (msg[i].len bytes) and, for the keyed
 * ops, data + key[i].off; its output goes to out + i * out_len. hash_len 32 = SHA-256, 48 = SHA-384.
 *   ATLS_HASH_SHA           sha256 / sha384 (hash/sha256.rs:188-192, sha384.rs:202-206); out_len = hash_len
 *   ATLS_HASH_HMAC          Hmac::new(hash, key).update(msg).result() (hash/hmac.rs:29-78); keys longer
 *                           than 64 bytes are hashed first for both hashes, as the reference does
 *   ATLS_HASH_HKDF_EXTRACT  Hkdf::extract(hash, salt = key, ikm = msg) (hash/hkdf.rs:24-32)
 *   ATLS_HASH_HKDF_EXPAND   Hkdf::expand(info = msg, out_len) with PRK = key (hash/hkdf.rs:35-65);
 *                           out_len > 255 * hash_len is ATLS_ILLEGAL_PARAMETER (the reference's None)
 * data / key / msg / out are host memory. */
typedef struct {
  uint64_t off;
  uint32_t len;
  uint32_t reserved;
} atls_span;
enum { ATLS_HASH_SHA = 0, ATLS_HASH_HMAC = 1, ATLS_HASH_HKDF_EXTRACT = 2, ATLS_HASH_HKDF_EXPAND = 3 };
int atls_hash_batch(atls_engine* e, int op, uint32_t hash_len, const uint8_t* data, size_t data_len,
                    const atls_span* keys, const atls_span* msgs, uint32_t n, uint32_t out_len, uint8_t* out);
/* The TLS 1.3 secret chain of n connections (KeySchedule::do_key_schedule, net/key_schedule.rs:170-222,
 * then WriteKeys::application_keys_from_master_secret, :87-114): from each (EC)DHE shared secret
 * (shared_len bytes) and ClientHello..ServerHello transcript hash (hash_len), out receives per
 * connection 5 secrets of hash_len bytes: client / server handshake traffic secret, master secret,
 * client / server application traffic secret 0 (from the ..server Finished transcript hash in
 * handshake_hashes; NULL leaves those two zero). Feed the traffic secrets to atls_derive_keys. */
int atls_key_schedule(atls_engine* e, uint32_t hash_len, const uint8_t* shared, size_t shared_len,
                      const uint8_t* hello_hashes, const uint8_t* handshake_hashes, uint32_t n, uint8_t* out);

/* The AES block cipher, AES::init + AES::encrypt / AES::decrypt (crypto/aes/cipher.rs:167-215),
 * over nblocks independent 16-byte blocks (ECB) under key slot key_slot of the engine's table
 * (an AES suite slot; otherwise ATLS_ILLEGAL_PARAMETER). Not on the record path -- GCM only
 * encrypts -- but the reference's AES API, on the device. flags: ATLS_FLAG_DEVICE_PTRS and
 * ATLS_FLAG_NO_SYNC as for the batches. */
int atls_aes_blocks(atls_engine* e, int decrypt, uint32_t key_slot, const void* in, void* out, size_t nblocks,
                    uint32_t flags);
/* One block with a raw key (16/24/32 B) on the calling thread's engine (as atls_seal). */
int atls_aes_block(int decrypt, const uint8_t* key, size_t key_len, const uint8_t in[16], uint8_t out[16]);

/* ---- Multi-GPU batches (one process, several devices), SURVEY.md §8(b)/(e) ----------------
 * Records are independent (the nonce is (static_iv, seq), key_schedule.rs:51-64), so a batch
 * splits into contiguous record ranges balanced by cumulative bytes, one per device, each sealed
 * or opened by that device's engine with rebased descriptors; outputs, tags and open results land
 * in the caller's buffers exactly as one engine would write them.
 * devices[0] is the root: with ATLS_FLAG_DEVICE_PTRS the buffers live on it and the other ranges
 * are scattered / gathered over RCCL (grouped send/recv over xGMI) when all devices are distinct,
 * or by device-to-device copies when the list repeats a device. Host buffers: every device stages
 * its own range over its own link. Descriptors are host arrays whose in/out ranges increase with
 * the record index (else ATLS_ILLEGAL_PARAMETER); ATLS_FLAG_DEVICE_RECS / ATLS_FLAG_NO_SYNC are not
 * accepted. Key slots are installed on every device. */
typedef struct atls_multi atls_multi;
atls_multi* atls_multi_create(const int* devices, int n_devices); /* NULL if a device or RCCL fails */
void atls_multi_destroy(atls_multi* m);
int atls_multi_devices(const atls_multi* m);
int atls_multi_uses_rccl(const atls_multi* m); /* 1: RCCL transport, 0: device copies / single device */
/* The RCCL actually loaded (ncclGetVersion, e.g. 22606 = 2.26.6; 0 without RCCL) and the largest
 * point-to-point message the multi engine sends (ranges go in pieces of at most this many bytes;
 * env ATLS_MULTI_CHUNK_MB, default 1 GiB: RCCL 2.26.6 corrupts self messages past 2^30 bytes).
 * The version and the cap are also printed to stderr once per process. */
int atls_multi_rccl_version(const atls_multi* m);
size_t atls_multi_max_message(const atls_multi* m);
int atls_multi_set_keys(atls_multi* m, const atls_key* keys, uint32_t n);
int atls_multi_seal_batch(atls_multi* m, const atls_rec* recs, uint32_t n, const void* in, const void* aux, void* out,
                          uint8_t* tags, uint32_t flags);
int atls_multi_open_batch(atls_multi* m, const atls_rec* recs, uint32_t n, const void* in, const void* aux,
                          const uint8_t* tags, void* out, atls_open_result* results, uint32_t flags);
/* The split both use: first[p] .. first[p+1]-1 are part p's records (first[parts] = n), cut where
 * the cumulative cost (bytes read + bytes written + 16-byte tag per record) crosses p/parts of
 * the total. Host-only, no device needed. */
void atls_partition(const atls_rec* recs, uint32_t n, int open, uint32_t parts, uint32_t* first);

/* ---- Batched record streams (TlsStream::tls_write / tls_read, net/stream.rs:32-150) -------
 * Many connections over one engine: atls_sb_write queues a connection's records (fragmented at
 * 2^14 bytes, RFC 8446 §5.1; the data is copied once, into the batch's page-locked input), atls_sb_flush
 * seals the queued records of every connection in ATLS_MODE_WIRE batches of consecutive records (a quarter of
 * the flush each, 8 .. 64 MiB of wire bytes, one sealed while the previous one is sent) and send()s each
 * connection's wire bytes in order; received bytes (atls_sb_recv / atls_sb_recv_all from the sockets, or atls_sb_feed) are
 * split into whole records (Record::from_raw, record.rs:81-102), atls_sb_open_pending opens every
 * connection's complete records in one batch, atls_sb_read returns the next application-data record of a
 * connection (blocking: receives and opens as needed; UnexpectedMessage (10) for other content types,
 * stream.rs:112-116; BrokenPipe (254) at end of stream). Each connection has a write key and a read key
 * with their own sequence numbers (key_schedule.rs:51-64); a record that fails ends its connection with
 * the record layer's error (50 / 51), which its reader gets after the records before it. Functions
 * returning long give a count (>= 0) or minus a TlsError code.
 * Threads: atls_sb_set_threads(sb, T) (1..64, default 1) spreads flush's sends, atls_sb_recv_all's
 * receives and open_pending's gather / hand-over over T threads (by connection). Calls on one batch
 * are serialised, except atls_sb_read_ready (and the copy-out of atls_sb_read), which take only the
 * connection's own lock: readers of different connections copy out in parallel; and atls_sb_flush, which
 * holds the batch lock only while it takes the queued records (and their input arena: later writes go to a
 * second one), so atls_sb_write on other threads proceeds while it seals and sends (one flush at a time).
 * If the engine fails part-way through a flush, the connections whose records were not sent end with its
 * error. */
typedef struct atls_stream_batch atls_stream_batch;
/* atls_sb_read_ready: no opened record yet. Outside the u8 range of TlsError (alert.rs:18-45, where 253 is
 * GotAlert), so no error code can be mistaken for it. */
enum { ATLS_WOULD_BLOCK = 0x100 };
atls_stream_batch* atls_sb_create(atls_engine* e);
void atls_sb_destroy(atls_stream_batch* sb);
int atls_sb_set_threads(atls_stream_batch* sb, int threads);
/* fd: a connected stream socket; returns the connection id (>= 0) or -code. */
int atls_sb_add_connection(atls_stream_batch* sb, int fd, const atls_key* write_key, const atls_key* read_key);
int atls_sb_write(atls_stream_batch* sb, int conn, uint8_t content_type, const uint8_t* data, size_t len);
long atls_sb_flush(atls_stream_batch* sb);                       /* records sealed and sent */
int atls_sb_feed(atls_stream_batch* sb, int conn, const uint8_t* data, size_t len);
long atls_sb_recv(atls_stream_batch* sb, int conn, size_t max_bytes); /* bytes read; 0 at EOF */
/* Every connection's socket drained without blocking (T threads), straight into its receive buffer;
 * when nothing at all arrived, waits up to timeout_ms for any connection and drains once more. Returns
 * the bytes received. */
long atls_sb_recv_all(atls_stream_batch* sb, int timeout_ms);
long atls_sb_open_pending(atls_stream_batch* sb);                /* records opened */
int atls_sb_read(atls_stream_batch* sb, int conn, uint8_t* buf, size_t cap, size_t* out_len);
/* As atls_sb_read without receiving or opening: an opened record, the connection's error once its
 * opened records are read, or ATLS_WOULD_BLOCK. */
int atls_sb_read_ready(atls_stream_batch* sb, int conn, uint8_t* buf, size_t cap, size_t* out_len);

/* Diagnostic (no reference counterpart): the shader clock the device runs at under the current load, for
 * rooflines counted in cycles. Enqueues wgs (1..1024) one-wave workgroups on `stream`
 * (hipStream_t as void*; NULL = the engine's stream). Each sleeps delay_us microseconds of the 100 MHz
 * constant clock, then writes {shader-clock ticks, constant-clock ticks} over spin_us more to out[2w],
 * out[2w+1] (device memory, 16 B per workgroup): SCLK = 100 MHz x out[2w] / out[2w+1]. The probe uses no
 * LDS, so on a second stream it runs beside a batch's kernels and samples their clock. delay_us and
 * spin_us are each at most 10,000,000 (else ATLS_ILLEGAL_PARAMETER). No host wait. */
int atls_clock_probe(atls_engine* e, void* stream, uint32_t wgs, uint32_t delay_us, uint32_t spin_us, uint64_t* out);

/* Library info: ABI version and the device arch the code objects were built for ("gfx950"). */
int atls_abi_version(void);
const char* atls_device_arch(void);
/* Compile-time experiment switches of this build (bit set, 0 for a product build). Timing
 * experiments that drop work (ATLS_DBG_*) give wrong results; tests assert this is 0. */
enum {
  ATLS_BUILD_DBG_SKIP = 1u, ATLS_BUILD_DBG_SHARED_GHASH = 2u, ATLS_BUILD_GHASH_W = 4u /* retired, never set */,
  ATLS_BUILD_NO_CTR_CACHE = 8u, ATLS_BUILD_GHASH_ROT = 16u, ATLS_BUILD_TT_STAMPS = 32u,
  ATLS_BUILD_CLK_STAMPS = 64u
};
unsigned atls_build_flags(void);

#ifdef __cplusplus
}
#endif
#endif
