// Host engine + C ABI (include/atls.h). C++ on the HIP runtime; no torch types.
//
// The engine owns one HIP device and two streams, the device key-slot table (KeySched, built
// by the key-setup kernel), the AES T-table, and staging buffers for callers that hand over
// host memory. A batch is first planned on the device (plan.hip: validation, one work list per
// kernel, longest records first), then the AES-GCM kernel (engine stream) and the
// ChaCha20-Poly1305 kernel (second stream, joined back) run concurrently over their lists, so
// descriptors may stay device-resident (ATLS_FLAG_DEVICE_RECS) with no host-side partitioning.
//
// atls_seal / atls_open are the Cipher-trait drop-ins (crypto/ciphersuite.rs:12-31): one RAW
// record on the calling thread's engine (key cache, pinned staging), with the same argument
// meaning and error codes.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <chrono>
#include <mutex>
#include <new>
#include <vector>

#include "../../include/atls.h"
#include "atls_dev.h"
#include "engine_internal.h"
#include "plan.h"

extern "C" int atls_launch_build_t0(uint32_t* t0, hipStream_t s);
extern "C" int atls_launch_aes_blocks(int decrypt, const void* ks, const uint8_t* in, uint8_t* out, uint64_t nblocks,
                                      uint32_t* err, int grid, hipStream_t s);
extern "C" int atls_launch_key_setup(const atls_key* keys, const atls_key* host_keys, uint32_t n, void* ks,
                                     const uint32_t* t0, hipStream_t s);
extern "C" int atls_key_setup_inline_max(void);
extern "C" int atls_launch_plan(int open, const void* ks, const atls_rec* recs, uint32_t n, uint32_t n_slots,
                                atls_open_result* res, uint32_t* err, void* P, uint8_t* keys, uint32_t* idx,
                                uint32_t* wg, int cus, hipStream_t s);
extern "C" int atls_launch_gcm(int open, const void* ks, const atls_rec* recs, uint32_t n, const uint8_t* in,
                               const uint8_t* aux, uint8_t* out, uint8_t* tags_out, const uint8_t* tags_in,
                               atls_open_result* res, const uint32_t* t0, const uint32_t* idx, void* plan,
                               uint32_t* err, uint32_t n_slots, int nr_mask, const uint32_t* gidx,
                               const uint32_t* ghdr, int grid, hipStream_t s, uint32_t* done, uint32_t done_val,
                               uint8_t* tail_ws);
extern "C" size_t atls_group_hdr_offset(uint32_t n_slots);
extern "C" size_t atls_gcm_tail_bytes(uint32_t n);
extern "C" int atls_launch_single_resident(uint8_t* blk, uint32_t idle_us, int gcm, hipStream_t s);
extern "C" int atls_launch_clock_probe(uint32_t wgs, uint32_t delay_us, uint32_t spin_us, uint64_t* out, hipStream_t s);
extern "C" int atls_launch_sync_flag(const uint32_t* err, uint32_t* out, uint32_t val, hipStream_t s);
extern "C" int atls_launch_gcm_single(int open, int nr, const void* ks, uint32_t n_slots, const atls_rec* d,
                                      const uint8_t* bytes, uint32_t nbytes, uint32_t tag_off, uint8_t* out,
                                      uint8_t* tags_out, atls_open_result* res, const uint32_t* t0, uint32_t* err,
                                      uint32_t* done, uint32_t done_val, hipStream_t s);
extern "C" int atls_launch_chacha_single(int open, const void* ks, uint32_t n_slots, const atls_rec* d,
                                         const uint8_t* bytes, uint32_t nbytes, uint32_t tag_off, uint8_t* out,
                                         uint8_t* tags_out, atls_open_result* res, uint32_t* err, uint32_t* done,
                                         uint32_t done_val, hipStream_t s);
extern "C" int atls_launch_group(const atls_rec* recs, uint32_t n, uint32_t n_slots, uint32_t* cnt, void* aux,
                                 uint32_t* gidx, int cus, hipStream_t s);
extern "C" int atls_launch_chacha(int open, const void* ks, const atls_rec* recs, uint32_t n, const uint8_t* in,
                                  const uint8_t* aux, uint8_t* out, uint8_t* tags_out, const uint8_t* tags_in,
                                  atls_open_result* res, const uint32_t* idx, void* plan, uint32_t* err,
                                  uint32_t n_slots, int grid, hipStream_t s, uint32_t* done, uint32_t done_val,
                                  int cus);
extern "C" int atls_launch_hash(int op, uint32_t hl, const uint8_t* data, const atls_span* keys, const atls_span* msgs,
                                uint32_t n, uint32_t out_len, uint8_t* out, hipStream_t s);
extern "C" int atls_launch_key_schedule(uint32_t hl, const uint8_t* shared, uint32_t shared_len, const uint8_t* hello,
                                        const uint8_t* fin, uint32_t n, uint8_t* out, hipStream_t s);
extern "C" int atls_launch_derive(uint16_t suite, const uint8_t* secrets, uint32_t secret_len, uint32_t n,
                                  atls_key* out, hipStream_t s);

namespace {

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  bool reserve(size_t n) {
    if (n <= cap) return true;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    size_t want = std::max<size_t>(n, 4096);
    if (hipMalloc(&p, want) != hipSuccess) return false;
    cap = want;
    return true;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

}  // namespace

#ifndef ATLS_SYNC_FLAG_DEFAULT
#define ATLS_SYNC_FLAG_DEFAULT 1  // synchronous returns wait on the sync-flag kernel (finish); env ATLS_SYNC_FLAG=0: stream sync
#endif
struct atls_engine {
  int device = 0;
  hipStream_t stream = nullptr;
  hipStream_t stream2 = nullptr;             // ChaCha20-Poly1305 kernel, concurrent with AES-GCM
  hipEvent_t ev_plan = nullptr, ev_side = nullptr;
  int cus = 256;
  uint32_t n_slots = 0;
  std::vector<atls_key> keys;                // host copy of the installed slots (suite flags below)
  bool has_aes = false, has_chacha = false;  // suites present in the key table: skip idle kernels
  int aes_nr_mask = 0;                       // bit 0/1/2: AES slots with 10/12/14 rounds
  DevBuf ks, t0, err, keys_stage, recs, in, out, aux, tags, res, secrets, dkeys;
  // Batch plans (plan.hip), two sets used by alternate planned batches: with ATLS_FLAG_LAZY_JOIN a
  // batch's side kernel may still read its set while the next batch is planned into the other.
  struct PlanSet {
    DevBuf plan, keys, idx, wg;
    hipEvent_t side_done = nullptr;  // the side (ChaCha20-Poly1305) kernel that read this set ended
    bool pending = false;            // side_done recorded, not yet joined into the engine stream
  } ps[2];
  int par = 0, last_par = 0;  // set of the next / the last planned batch
  DevBuf grp_cnt, grp_aux, grp_idx;          // key groups of direct AES-GCM batches (plan.hip)
  DevBuf tail;                               // deferred last steps of AES-GCM batch records (gcm.hip ATLS_GCM_TAIL)
  bool tail_on = true;                       // ATLS_GCM_TAIL_ON=0: every record runs its own last step
  uint32_t group_min = 2048;                 // ATLS_GCM_GROUP_MIN: smallest batch to group (0: never)
  int chacha_wgs = 8;                        // ATLS_CHACHA_WGS: ChaCha20-Poly1305 workgroups per CU
  // ATLS_CHACHA_W2: direct ChaCha20-Poly1305 batches take the 2-wave kernel always (2, the default), only when
  // they fit in two waves per SIMD (1), never (0). Batches of 2x and 4x C3's records: 2-wave seal 0.180 /
  // 0.369 ms against 0.202 / 0.391 for the 3-wave kernel, opens 0.186 / 0.381 against 0.202 / 0.390
  // (profiles/r03/ab_c3_big_batches.log).
  int chacha_w2 = 2;
  bool force_plan = false;                   // ATLS_FORCE_PLAN=1: plan every batch (tests)
  bool no_pipeline = false;                  // ATLS_NO_PIPELINE=1: stage host batches in one piece
  // Host-memory batches (run_host_pipelined): an upload and a download stream beside the engine stream,
  // created on the first such batch, and two events per chunk.
  hipStream_t up = nullptr, down = nullptr;
  std::vector<hipEvent_t> pev;
  int zero_copy = 0;  // ATLS_ZERO_COPY: 1 = kernels read and write pinned host buffers in place, 2 = write only
  // Synchronous returns (finish): a mapped word pair the sync-flag kernel writes -- [0] completion value,
  // [1] the sticky error word -- instead of hipStreamSynchronize + a copy (ATLS_SYNC_FLAG=0: the old way)
  uint32_t* sync_h = nullptr;
  uint32_t* sync_d = nullptr;
  uint32_t sync_val = 0;
  int sync_flag = ATLS_SYNC_FLAG_DEFAULT;
  std::mutex mu;
};

namespace {

bool set_dev(atls_engine* e) { return hipSetDevice(e->device) == hipSuccess; }

// The sticky error word (a kernel sets it for a descriptor it refuses) collects every batch
// since the last synchronisation; it is read here and cleared only when set, so no batch pays
// a memset launch and a NO_SYNC batch's refusal is reported by the next atls_engine_sync.
int take_err(atls_engine* e, uint32_t err) {
  if (!err) return ATLS_OK;
  const uint32_t zero = 0;
  if (hipMemcpy(e->err.p, &zero, 4, hipMemcpyHostToDevice) != hipSuccess) return ATLS_INTERNAL_ERROR;
  return ATLS_ILLEGAL_PARAMETER;
}

// The engine stream waits for every side kernel not yet joined (ATLS_FLAG_LAZY_JOIN batches).
int join_pending(atls_engine* e) {
  for (auto& q : e->ps) {
    if (!q.pending) continue;
    if (hipStreamWaitEvent(e->stream, q.side_done, 0) != hipSuccess) return ATLS_INTERNAL_ERROR;
    q.pending = false;
  }
  return ATLS_OK;
}

// The sync-flag block (mapped, page-locked), allocated on first use; false: use the stream sync.
bool sync_flag_ready(atls_engine* e) {
  if (!e->sync_flag) return false;
  if (e->sync_h) return true;
  void* p = nullptr;
  void* pd = nullptr;
  if (hipHostMalloc(&p, 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
    e->sync_flag = 0;
    return false;
  }
  if (hipHostGetDevicePointer(&pd, p, 0) != hipSuccess) {
    (void)hipHostFree(p);
    e->sync_flag = 0;
    return false;
  }
  std::memset(p, 0, 64);
  e->sync_h = (uint32_t*)p;
  e->sync_d = (uint32_t*)pd;
  return true;
}

// host_copies: the stream holds copies into the caller's host memory, which may be pageable -- the runtime
// finishes those on the host after the device is done with them, so only a stream synchronisation covers them.
int finish(atls_engine* e, uint32_t flags, bool host_copies = false) {
  if (flags & ATLS_FLAG_NO_SYNC) return ATLS_OK;
  if (join_pending(e)) return ATLS_INTERNAL_ERROR;
  uint32_t err = 0;
  if (!host_copies && sync_flag_ready(e)) {
    // everything before it on the engine stream has finished once the flag reads v. The host spins for at
    // most kSpinUs (the small-call latency win), then blocks in hipStreamSynchronize, so a long
    // batch does not hold a core; a stream that ends without the flag (a fault) is reported by
    // hipStreamQuery, checked every few thousand spins, or by the synchronisation
    constexpr int64_t kSpinUs = 100;
    const uint32_t v = ++e->sync_val;
    __atomic_store_n(&e->sync_h[0], v - 1u, __ATOMIC_RELEASE);
    if (atls_launch_sync_flag((const uint32_t*)e->err.p, e->sync_d, v, e->stream)) return ATLS_INTERNAL_ERROR;
    const auto t0 = std::chrono::steady_clock::now();
    for (uint64_t i = 1;; i++) {
      if (__atomic_load_n(&e->sync_h[0], __ATOMIC_ACQUIRE) == v) break;
      if ((i & 255) == 0 && std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0)
                                    .count() > kSpinUs) {
        if (hipStreamSynchronize(e->stream) != hipSuccess) return ATLS_INTERNAL_ERROR;
        if (__atomic_load_n(&e->sync_h[0], __ATOMIC_ACQUIRE) != v) return ATLS_INTERNAL_ERROR;
        break;
      }
      if ((i & 4095) == 0) {
        const hipError_t q = hipStreamQuery(e->stream);
        if (q == hipSuccess) {
          if (__atomic_load_n(&e->sync_h[0], __ATOMIC_ACQUIRE) == v) break;
          return ATLS_INTERNAL_ERROR;
        }
        if (q != hipErrorNotReady) return ATLS_INTERNAL_ERROR;
      }
      __builtin_ia32_pause();
    }
    err = __atomic_load_n(&e->sync_h[1], __ATOMIC_ACQUIRE);
  } else {
    if (hipStreamSynchronize(e->stream) != hipSuccess) return ATLS_INTERNAL_ERROR;
    if (hipMemcpy(&err, e->err.p, 4, hipMemcpyDeviceToHost) != hipSuccess) return ATLS_INTERNAL_ERROR;
  }
  return take_err(e, err);
}

// Bytes a record reads at in_off and writes at out_off. TLS seal: content + type byte out;
// WIRE seal: header || ct || tag out; WIRE open: header || ct || tag in.
size_t rec_in_len(const atls_rec& r, bool open) {
  return (r.mode == ATLS_MODE_WIRE && open) ? (size_t)r.len + 21 : (size_t)r.len;
}
size_t rec_out_len(const atls_rec& r, bool open) {
  if (open || r.mode == ATLS_MODE_RAW) return r.len;
  return r.mode == ATLS_MODE_WIRE ? (size_t)r.len + 22 : (size_t)r.len + 1;
}

// Largest byte extent touched by the descriptors (host-memory mode only).
// The device address of a page-locked, device-mapped host range [p, p + len) (hipHostMalloc /
// hipHostRegister memory, e.g. torch pin_memory), or nullptr for pageable memory.
void* host_alias(const void* p, size_t len) {
  if (!p || !len) return nullptr;
  hipPointerAttribute_t a, b;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  if (a.type != hipMemoryTypeHost || !a.devicePointer) return nullptr;
  const uint8_t* last = (const uint8_t*)p + len - 1;
  if (hipPointerGetAttributes(&b, last) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  if (b.type != hipMemoryTypeHost || (uint8_t*)b.devicePointer != (uint8_t*)a.devicePointer + (len - 1)) return nullptr;
  return a.devicePointer;
}

void extents(const atls_rec* recs, uint32_t n, bool open, size_t* in_end, size_t* out_end, size_t* aux_end) {
  size_t a = 0, b = 0, c = 0;
  for (uint32_t i = 0; i < n; i++) {
    const atls_rec& r = recs[i];
    a = std::max(a, (size_t)r.in_off + rec_in_len(r, open));
    b = std::max(b, (size_t)r.out_off + rec_out_len(r, open));
    if (r.mode == ATLS_MODE_RAW) c = std::max(c, (size_t)r.aux_off + r.iv_len + r.aad_len);
  }
  *in_end = a;
  *out_end = b;
  *aux_end = c;
}

// The tail workspace of an AES-GCM batch of n records (gcm.hip ATLS_GCM_TAIL), its counters zero; nullptr (no record
// deferred) when the build or ATLS_GCM_TAIL_ON=0 turns deferral off or the buffer cannot grow.
uint8_t* tail_ws(atls_engine* e, uint32_t n, hipStream_t s) {
  const size_t need = atls_gcm_tail_bytes(n);
  if (!need || !e->tail_on) return nullptr;
  const size_t cap = e->tail.cap;
  if (!e->tail.reserve(need)) return nullptr;
  // the tail kernel zeroes the counters after each batch: a new buffer once
  if (e->tail.cap != cap && hipMemsetAsync(e->tail.p, 0, 16, s) != hipSuccess) return nullptr;
  return (uint8_t*)e->tail.p;
}

// The CU count atls_launch_chacha sizes its 2-wave choice by: 0 never takes it, a huge count always does.
int w2_cus(const atls_engine* e) { return e->chacha_w2 == 0 ? 0 : e->chacha_w2 == 2 ? (1 << 26) : e->cus; }

int launch_records(atls_engine* e, bool open, const atls_rec* d_recs, uint32_t n, const uint8_t* d_in,
                   const uint8_t* d_aux, uint8_t* d_out, uint8_t* d_tags_out, const uint8_t* d_tags_in,
                   atls_open_result* d_res, hipStream_t s, uint32_t* done = nullptr, uint32_t done_val = 0) {
  // direct batches only (one record kernel in the key table)
  if (e->has_chacha)
    return atls_launch_chacha(open, e->ks.p, d_recs, n, d_in, d_aux, d_out, d_tags_out, d_tags_in, d_res, nullptr,
                              nullptr, (uint32_t*)e->err.p, e->n_slots, e->cus * e->chacha_wgs, s, done, done_val,
                              w2_cus(e));
  return atls_launch_gcm(open, e->ks.p, d_recs, n, d_in, d_aux, d_out, d_tags_out, d_tags_in, d_res,
                         (const uint32_t*)e->t0.p, nullptr, nullptr, (uint32_t*)e->err.p, e->n_slots,
                         e->aes_nr_mask, nullptr, nullptr, e->cus, s, done, done_val,
                         done ? nullptr : tail_ws(e, n, s));
}

// Host-memory batch in record-aligned chunks over three streams: every chunk's input goes up on the
// upload stream, its kernel runs on the engine stream once that copy is done, and its output comes back
// on the download stream once the kernel is done. Each direction of the link then has one stream that is
// never idle while chunks remain, so uploads of later chunks run beside downloads of earlier ones the
// whole time. tools/ubench/pcie_probe.hip (profiles/r03/pcie_probe.log): PCIe Gen5 gives 57 GB/s one way
// and 48.5 GB/s per direction both ways at once; chunked copies on the round-2 scheme (chunk k's upload,
// kernel and download on one of two streams in turn) reach 40.4 without any kernel. Measured C2 from
// pinned memory: 37.1 GiB/s (round 2 scheme) -> 37.96 (this one, 32 MiB chunks); 16 MiB chunks 32.1,
// 8 MiB 26.6 -- a fixed cost per chunk, not the link, sets the rate at small chunks.
// A fixed-pitch output layout (all records the same stride, the C2/C4 case) comes back with
// hipMemcpy2DAsync, so the bytes between records are never read or written; other layouts stage each
// chunk's output range in and out. Returns -1 when the records are not in ascending order (the caller
// stages the batch in one piece).
int run_host_pipelined(atls_engine* e, bool open, const atls_rec* recs, uint32_t n, const void* in, const void* aux,
                       void* out, uint8_t* tags_out, const uint8_t* tags_in, atls_open_result* res,
                       size_t in_end, size_t out_end, size_t aux_end) {
  static const size_t kChunkBytes = [] {  // ATLS_CHUNK_MB overrides (tuning)
    const char* v = std::getenv("ATLS_CHUNK_MB");
    const long mb = v ? std::atol(v) : 32;
    return (size_t)(mb > 0 ? mb : 32) << 20;
  }();
  // The pipeline fills with small chunks and drains with small chunks: the first chunk's upload and the
  // last chunk's download overlap nothing, so chunk k holds at most kFirst << k bytes on the way up and at
  // most half of what is left on the way down (never below kFirst). ATLS_CHUNK_FIRST_MB overrides; 0 = flat.
  static const size_t kFirst = [] {
    const char* v = std::getenv("ATLS_CHUNK_FIRST_MB");
    const long mb = v ? std::atol(v) : 4;
    return (size_t)(mb > 0 ? mb : 0) << 20;
  }();
  const size_t in_total = n ? recs[n - 1].in_off + rec_in_len(recs[n - 1], open) : 0;
  auto chunk_limit = [&](size_t k, size_t from) {
    if (!kFirst) return kChunkBytes;
    size_t lim = k < 16 ? std::min(kChunkBytes, kFirst << k) : kChunkBytes;
    const size_t rem = in_total > from ? in_total - from : 0;
    return std::min(lim, std::max(kFirst, rem / 2));
  };
  auto ilen = [&](const atls_rec& r) { return rec_in_len(r, open); };
  auto olen = [&](const atls_rec& r) { return rec_out_len(r, open); };
  for (uint32_t i = 1; i < n; i++)
    if (recs[i].in_off < recs[i - 1].in_off + ilen(recs[i - 1]) || recs[i].out_off < recs[i - 1].out_off + olen(recs[i - 1]))
      return -1;
  // each stream on its own: a failed creation of one leaves it null and is retried by the next batch
  if (!e->up && hipStreamCreateWithFlags(&e->up, hipStreamNonBlocking) != hipSuccess) {
    e->up = nullptr;
    return ATLS_INTERNAL_ERROR;
  }
  if (!e->down && hipStreamCreateWithFlags(&e->down, hipStreamNonBlocking) != hipSuccess) {
    e->down = nullptr;
    return ATLS_INTERNAL_ERROR;
  }
  // Output layouts: gapless (every record's output starts where the previous one's ends -- WIRE seals
  // packed back to back, the socket path's case) comes back as one linear copy per chunk, with nothing
  // staged in; a fixed pitch with gaps (TLS seals in 16-byte slots, C2 / C4) by a 2-D copy that skips the
  // gaps -- when the pitch is a multiple of 16: a 2-D copy of 16,406-byte rows ran at 1.7 GB/s against 32
  // for the same bytes linear (tools/host_batch_probe.py, profiles/r05/host_batch_probe*.log); anything
  // else stages the chunk's output range in and out.
  bool gapless = true;
  for (uint32_t i = 1; i < n && gapless; i++) gapless = recs[i].out_off == recs[i - 1].out_off + olen(recs[i - 1]);
  const size_t pitch = n > 1 ? (size_t)(recs[1].out_off - recs[0].out_off) : 0, width = olen(recs[0]);
  bool pitched = n > 1 && !gapless && pitch % 16 == 0;
  for (uint32_t i = 1; i < n && pitched; i++)
    pitched = olen(recs[i]) == width && recs[i].out_off == recs[0].out_off + i * pitch;
  hipStream_t ks = e->stream, up = e->up, down = e->down;
  // A failure after work is queued returns only once the queued copies and kernels are done with the
  // caller's buffers (nothing may write them after the call returns).
  auto fail = [&](int rc) {
    (void)hipStreamSynchronize(up);
    (void)hipStreamSynchronize(ks);
    (void)hipStreamSynchronize(down);
    return rc;
  };
  // ATLS_ZERO_COPY=2: the kernels write their output (records, tags, open results) straight into the
  // page-locked host buffers, so nothing comes back through the download stream and nothing of `out`
  // is staged in (only record bytes are written); the inputs still go up in chunks.
  uint8_t* z_out = nullptr;
  uint8_t* z_tags = nullptr;
  atls_open_result* z_res = nullptr;
  if (e->zero_copy == 2 && out_end) {
    z_out = (uint8_t*)host_alias(out, out_end);
    const uint8_t* tp = open ? nullptr : tags_out;
    z_tags = tp ? (uint8_t*)host_alias(tp, 16 * (size_t)n) : nullptr;
    z_res = open ? (atls_open_result*)host_alias(res, sizeof(atls_open_result) * (size_t)n) : nullptr;
    if (!z_out || (tp && !z_tags) || (open && !z_res)) z_out = z_tags = nullptr, z_res = nullptr;
  }
  const bool zo = z_out != nullptr;
  // the batch's descriptors and aux are in place, and the engine's earlier batches (which used the same
  // staging buffers) are done, before the first upload
  if (aux_end && hipMemcpyAsync(e->aux.p, aux, aux_end, hipMemcpyHostToDevice, ks) != hipSuccess) return fail(ATLS_INTERNAL_ERROR);
  if (hipEventRecord(e->ev_plan, ks) != hipSuccess || hipStreamWaitEvent(up, e->ev_plan, 0) != hipSuccess)
    return fail(ATLS_INTERNAL_ERROR);
  const auto* d_recs = (const atls_rec*)e->recs.p;
  auto* d_in = (uint8_t*)e->in.p;
  auto* d_out = (uint8_t*)e->out.p;
  auto* d_tags = (uint8_t*)e->tags.p;
  auto* d_res = (atls_open_result*)e->res.p;
  (void)in_end;
  (void)out_end;
  size_t k = 0;
  for (uint32_t a = 0; a < n; k++) {
    uint32_t b = a + 1;
    const size_t lim = chunk_limit(k, recs[a].in_off);
    while (b < n && recs[b].in_off + ilen(recs[b]) - recs[a].in_off <= lim) b++;
    while (e->pev.size() < 2 * (k + 1)) {
      hipEvent_t ev;
      if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) return fail(ATLS_INTERNAL_ERROR);
      e->pev.push_back(ev);
    }
    hipEvent_t uploaded = e->pev[2 * k], sealed = e->pev[2 * k + 1];
    const size_t in_lo = recs[a].in_off, in_hi = recs[b - 1].in_off + ilen(recs[b - 1]);
    const size_t out_lo = recs[a].out_off, out_hi = recs[b - 1].out_off + olen(recs[b - 1]);
    const uint32_t cnt = b - a;
    if (in_hi > in_lo &&
        hipMemcpyAsync(d_in + in_lo, (const uint8_t*)in + in_lo, in_hi - in_lo, hipMemcpyHostToDevice, up) != hipSuccess)
      return fail(ATLS_INTERNAL_ERROR);
    if (open && tags_in && hipMemcpyAsync(d_tags + 16 * (size_t)a, tags_in + 16 * (size_t)a, 16 * (size_t)cnt,
                               hipMemcpyHostToDevice, up) != hipSuccess)
      return fail(ATLS_INTERNAL_ERROR);
    if (!zo && !pitched && !gapless && out_hi > out_lo &&
        hipMemcpyAsync(d_out + out_lo, (uint8_t*)out + out_lo, out_hi - out_lo, hipMemcpyHostToDevice, up) != hipSuccess)
      return fail(ATLS_INTERNAL_ERROR);
    if (hipEventRecord(uploaded, up) != hipSuccess || hipStreamWaitEvent(ks, uploaded, 0) != hipSuccess)
      return fail(ATLS_INTERNAL_ERROR);
    uint8_t* k_tags_out = d_tags + 16 * (size_t)a;
    if (zo && !open) k_tags_out = z_tags ? z_tags + 16 * (size_t)a : k_tags_out;
    int rc = launch_records(e, open, d_recs + a, cnt, d_in, (const uint8_t*)e->aux.p, zo ? z_out : d_out, k_tags_out,
                            d_tags + 16 * (size_t)a, zo && open ? z_res + a : d_res + a, ks);
    if (rc) return fail(rc);
    const uint32_t a0 = a;
    a = b;
    if (zo) continue;  // written in place
    if (hipEventRecord(sealed, ks) != hipSuccess || hipStreamWaitEvent(down, sealed, 0) != hipSuccess)
      return fail(ATLS_INTERNAL_ERROR);
    if (pitched) {
      if (width && hipMemcpy2DAsync((uint8_t*)out + out_lo, pitch, d_out + out_lo, pitch, width, cnt,
                                    hipMemcpyDeviceToHost, down) != hipSuccess)
        return fail(ATLS_INTERNAL_ERROR);
    } else if (out_hi > out_lo &&
               hipMemcpyAsync((uint8_t*)out + out_lo, d_out + out_lo, out_hi - out_lo, hipMemcpyDeviceToHost, down) != hipSuccess) {
      return fail(ATLS_INTERNAL_ERROR);
    }
    if (!open && tags_out && hipMemcpyAsync(tags_out + 16 * (size_t)a0, d_tags + 16 * (size_t)a0, 16 * (size_t)cnt,
                                hipMemcpyDeviceToHost, down) != hipSuccess)
      return fail(ATLS_INTERNAL_ERROR);
    if (open && hipMemcpyAsync(res + a0, d_res + a0, sizeof(atls_open_result) * (size_t)cnt, hipMemcpyDeviceToHost, down) !=
                    hipSuccess)
      return fail(ATLS_INTERNAL_ERROR);
  }
  // the engine stream is ordered after the last download (finish synchronises it)
  if (!zo && (hipEventRecord(e->ev_side, down) != hipSuccess || hipStreamWaitEvent(ks, e->ev_side, 0) != hipSuccess))
    return fail(ATLS_INTERNAL_ERROR);
  return finish(e, 0, true);
}

using atls::ResidentHold;  // engine_internal.h; defined below, with the resident single-call server

unsigned long long g_host_unpipelined = 0;  // host batches staged in one piece: records out of order (diagnostic)

int run_batch(atls_engine* e, bool open, const atls_rec* recs, uint32_t n, const void* in, const void* aux,
              void* out, uint8_t* tags_out, const uint8_t* tags_in, atls_open_result* res, uint32_t flags) {
  if (!e) return ATLS_INTERNAL_ERROR;
  if (n == 0) return ATLS_OK;
  ResidentHold hold;
  std::lock_guard<std::mutex> lk(e->mu);
  if (!set_dev(e)) return ATLS_INTERNAL_ERROR;
  if (e->n_slots == 0) return ATLS_ILLEGAL_PARAMETER;
  hipStream_t s = e->stream;
  const bool dev_ptrs = flags & ATLS_FLAG_DEVICE_PTRS;
  const bool dev_recs = flags & ATLS_FLAG_DEVICE_RECS;
  // No tags array: every record must carry its tag in the wire record (ATLS_MODE_WIRE). The
  // kernels then get the engine's scratch array, so a device-resident non-WIRE descriptor cannot
  // fault (it seals into scratch, or fails authentication on open).
  const bool no_tags = open ? !tags_in : !tags_out;
  // A lazy batch leaves its side kernel running into the next batch, so it may use no engine buffer
  // that the next batch rewrites or reallocates: the descriptors must be the caller's (DEVICE_RECS,
  // not the engine's staging copy) and so must the tags (not the engine's scratch array). Any other
  // batch joins the side kernels of earlier lazy batches first.
  const bool lazy = (flags & ATLS_FLAG_LAZY_JOIN) && (flags & ATLS_FLAG_NO_SYNC) && dev_ptrs && dev_recs && !no_tags;
  if (!lazy && join_pending(e)) return ATLS_INTERNAL_ERROR;  // a batch without the flag starts after all
  if (!dev_ptrs && dev_recs) return ATLS_ILLEGAL_PARAMETER;  // host buffers need host-visible descriptors

  if (no_tags && !e->tags.reserve(16 * (size_t)n)) return ATLS_INTERNAL_ERROR;
  const atls_rec* d_recs = recs;
  if (!dev_recs) {
    for (uint32_t i = 0; i < n; i++)
      if (recs[i].key_slot >= e->n_slots || recs[i].mode > ATLS_MODE_WIRE || (no_tags && recs[i].mode != ATLS_MODE_WIRE))
        return ATLS_ILLEGAL_PARAMETER;
    if (!e->recs.reserve(sizeof(atls_rec) * (size_t)n)) return ATLS_INTERNAL_ERROR;
    if (hipMemcpyAsync(e->recs.p, recs, sizeof(atls_rec) * (size_t)n, hipMemcpyHostToDevice, s) != hipSuccess)
      return ATLS_INTERNAL_ERROR;
    d_recs = (const atls_rec*)e->recs.p;
  }
  const uint8_t* d_in = (const uint8_t*)in;
  const uint8_t* d_aux = (const uint8_t*)aux;
  uint8_t* d_out = (uint8_t*)out;
  uint8_t* d_tags_out = no_tags ? (uint8_t*)e->tags.p : tags_out;
  const uint8_t* d_tags_in = no_tags ? (const uint8_t*)e->tags.p : tags_in;
  atls_open_result* d_res = res;
  size_t in_end = 0, out_end = 0, aux_end = 0;
  // A key table holding one record kernel's suite and round count gives a direct batch: that
  // kernel walks the descriptors itself. Otherwise the batch is planned (plan.hip): ~30 us of
  // small launches that sort records into per-kernel lists, longest first.
  const int kinds = (e->has_chacha ? 1 : 0) + __builtin_popcount((unsigned)e->aes_nr_mask);
  const bool planned = kinds > 1 || e->force_plan;
  bool zc = false;
  if (!dev_ptrs) {
    extents(recs, n, open, &in_end, &out_end, &aux_end);
    // Zero copy (opt-in, ATLS_ZERO_COPY=1): every host buffer of the batch is page-locked and mapped, so
    // the kernels read the records from host memory and write their output there in place, over PCIe,
    // with no staging copies. C2 from pinned memory, same box (profiles/r03/bench_c2_pcie_modes_*.log):
    // staged 38.2 GiB/s, zero copy 33.9, output-only zero copy (=2, run_host_pipelined) 38.6: the lane
    // groups' 128-B runs of 8 records 16 KiB apart touch many host pages at once, where a copy engine
    // streams.
    if (e->zero_copy == 1) {
      // a buffer the batch does not touch (extent 0, e.g. aux in TLS / WIRE batches) gets a placeholder the
      // kernels never dereference: the engine's error word, which always exists (the engine's
      // staging buffers are null on a fresh engine, which made the first call fall back to staging)
      void* ph = e->err.p;
      const void* zi = in_end ? host_alias(in, in_end) : ph;
      void* zo = out_end ? host_alias(out, out_end) : ph;
      const void* za = aux_end ? host_alias(aux, aux_end) : ph;
      const void* zt = no_tags ? e->tags.p : host_alias(open ? (const void*)tags_in : (const void*)tags_out, 16 * (size_t)n);
      void* zr = open ? host_alias(res, sizeof(atls_open_result) * (size_t)n) : (void*)res;
      if (zi && zo && za && zt && (zr || !open)) {
        zc = true;
        d_in = (const uint8_t*)zi;
        d_out = (uint8_t*)zo;
        d_aux = (const uint8_t*)za;
        d_tags_out = (uint8_t*)zt;
        d_tags_in = (const uint8_t*)zt;
        d_res = (atls_open_result*)zr;
      }
    }
  }
  if (!dev_ptrs && !zc) {
    if (!e->in.reserve(in_end + 16) || !e->out.reserve(out_end + 16) || !e->aux.reserve(aux_end + 16) ||
        !e->tags.reserve(16 * (size_t)n) || !e->res.reserve(sizeof(atls_open_result) * (size_t)n))
      return ATLS_INTERNAL_ERROR;
    if (!planned && n > 1 && !e->no_pipeline) {
      const int rc = run_host_pipelined(e, open, recs, n, in, aux, out, tags_out, tags_in, res, in_end, out_end, aux_end);
      if (rc != -1) return rc;
      __atomic_fetch_add(&g_host_unpipelined, 1ull, __ATOMIC_RELAXED);
    }
    if (in_end && hipMemcpyAsync(e->in.p, in, in_end, hipMemcpyHostToDevice, s) != hipSuccess) return ATLS_INTERNAL_ERROR;
    if (aux_end && hipMemcpyAsync(e->aux.p, aux, aux_end, hipMemcpyHostToDevice, s) != hipSuccess)
      return ATLS_INTERNAL_ERROR;
    if (open && tags_in && hipMemcpyAsync(e->tags.p, tags_in, 16 * (size_t)n, hipMemcpyHostToDevice, s) != hipSuccess)
      return ATLS_INTERNAL_ERROR;
    // Bytes of `out` outside the records must come back unchanged: stage them in too.
    if (out_end && hipMemcpyAsync(e->out.p, out, out_end, hipMemcpyHostToDevice, s) != hipSuccess)
      return ATLS_INTERNAL_ERROR;
    d_in = (const uint8_t*)e->in.p;
    d_aux = (const uint8_t*)e->aux.p;
    d_out = (uint8_t*)e->out.p;
    d_tags_out = (uint8_t*)e->tags.p;
    d_tags_in = (const uint8_t*)e->tags.p;
    d_res = (atls_open_result*)e->res.p;
  }
  int rc = 0;
  const uint32_t* idx = nullptr;
  void* plan_hdr = nullptr;
  auto& ps = e->ps[e->par];
  if (planned) {
    // this set was last read by the side kernel of the planned batch before the previous one: the
    // plan waits for it on the device, or on the host if a buffer has to grow (a reallocation)
    const size_t wg_bytes = 2 * 4 * (size_t)atls::kPlanKeys * atls::kPlanMaxWG;
    const bool grow = ps.plan.cap < sizeof(atls::PlanHdr) || ps.keys.cap < n || ps.idx.cap < 4 * (size_t)n ||
                      ps.wg.cap < wg_bytes;
    if (ps.pending) {
      if ((grow ? hipEventSynchronize(ps.side_done) : hipStreamWaitEvent(s, ps.side_done, 0)) != hipSuccess)
        return ATLS_INTERNAL_ERROR;
      ps.pending = false;
    }
    if (!ps.plan.reserve(sizeof(atls::PlanHdr)) || !ps.keys.reserve(n) || !ps.idx.reserve(4 * (size_t)n) ||
        !ps.wg.reserve(wg_bytes))
      return ATLS_INTERNAL_ERROR;
    rc = atls_launch_plan(open, e->ks.p, d_recs, n, e->n_slots, d_res, (uint32_t*)e->err.p, ps.plan.p,
                          (uint8_t*)ps.keys.p, (uint32_t*)ps.idx.p, (uint32_t*)ps.wg.p, e->cus, s);
    if (rc) return rc;
    idx = (const uint32_t*)ps.idx.p;
    plan_hdr = ps.plan.p;
    e->last_par = e->par;
    e->par ^= 1;
  }
  // Both suites present: ChaCha20-Poly1305 (VALU-bound) on the second stream beside AES-GCM
  // (LDS-bound), joined back into the engine stream.
  const bool side = e->has_aes && e->has_chacha;
  if (e->has_chacha) {
    hipStream_t cs = s;
    if (side) {
      if (hipEventRecord(e->ev_plan, s) != hipSuccess || hipStreamWaitEvent(e->stream2, e->ev_plan, 0) != hipSuccess)
        return ATLS_INTERNAL_ERROR;
      cs = e->stream2;
    }
    rc = atls_launch_chacha(open, e->ks.p, d_recs, n, d_in, d_aux, d_out, d_tags_out, d_tags_in, d_res, idx,
                            plan_hdr, (uint32_t*)e->err.p, e->n_slots, e->cus * e->chacha_wgs, cs, nullptr, 0,
                            w2_cus(e));
    if (rc) return rc;
    if (side && hipEventRecord(ps.side_done, e->stream2) != hipSuccess) return ATLS_INTERNAL_ERROR;
  }
  if (e->has_aes) {
    // A direct batch large enough: records of one key slot go through the kernel in lane groups
    // (gcm.hip gcm_group), after a counting sort by key slot (three small launches).
    const uint32_t* gidx = nullptr;
    const uint32_t* ghdr = nullptr;
    if (!planned && e->group_min && n >= e->group_min && e->n_slots <= atls::kGroupMaxSlots) {
      const size_t nb = (size_t)e->n_slots + 1, hdr_at = atls_group_hdr_offset(e->n_slots);
      const size_t cnt_cap = e->grp_cnt.cap;
      if (!e->grp_cnt.reserve(8 * nb) || !e->grp_aux.reserve(hdr_at + sizeof(atls::GroupHdr) + 4 * (size_t)n) ||
          !e->grp_idx.reserve(4 * (size_t)n))
        return ATLS_INTERNAL_ERROR;
      // counts and cursors are zero between batches (group_place clears them): zero a new buffer once
      if (e->grp_cnt.cap != cnt_cap && hipMemsetAsync(e->grp_cnt.p, 0, e->grp_cnt.cap, s) != hipSuccess)
        return ATLS_INTERNAL_ERROR;
      rc = atls_launch_group(d_recs, n, e->n_slots, (uint32_t*)e->grp_cnt.p, e->grp_aux.p, (uint32_t*)e->grp_idx.p,
                             e->cus, s);
      if (rc) return rc;
      gidx = (const uint32_t*)e->grp_idx.p;
      ghdr = (const uint32_t*)((const uint8_t*)e->grp_aux.p + hdr_at);
    }
    // bit 3: beside the ChaCha20-Poly1305 kernel (gcm.hip gcm_kernel BESIDE: its seal waves leave room for a ChaCha wave)
    rc = atls_launch_gcm(open, e->ks.p, d_recs, n, d_in, d_aux, d_out, d_tags_out, d_tags_in, d_res,
                         (const uint32_t*)e->t0.p, idx, plan_hdr, (uint32_t*)e->err.p, e->n_slots,
                         e->aes_nr_mask | (side ? 8 : 0),
                         gidx, ghdr, e->cus, s, nullptr, 0, tail_ws(e, n, s));
  }
  if (rc) return rc;
  if (side) {  // join now, or (lazy) when the set is reused / atls_engine_join / a batch without the flag
    if (lazy) ps.pending = true;
    else if (hipStreamWaitEvent(s, ps.side_done, 0) != hipSuccess) return ATLS_INTERNAL_ERROR;
  }
  // host buffers read and written in place: the batch ends before the call returns, by a stream synchronisation
  // (the kernels' stores to page-locked host memory are covered by the stream's completion)
  if (zc) return finish(e, flags & ~ATLS_FLAG_NO_SYNC, true);
  if (!dev_ptrs) {
    if (out_end && hipMemcpyAsync(out, e->out.p, out_end, hipMemcpyDeviceToHost, s) != hipSuccess)
      return ATLS_INTERNAL_ERROR;
    if (!open && tags_out && hipMemcpyAsync(tags_out, e->tags.p, 16 * (size_t)n, hipMemcpyDeviceToHost, s) != hipSuccess)
      return ATLS_INTERNAL_ERROR;
    if (open && hipMemcpyAsync(res, e->res.p, sizeof(atls_open_result) * (size_t)n, hipMemcpyDeviceToHost, s) !=
                    hipSuccess)
      return ATLS_INTERNAL_ERROR;
    return finish(e, flags & ~ATLS_FLAG_NO_SYNC, true);
  }
  return finish(e, flags);
}

int key_status(const atls_key& k) {
  if (k.suite == ATLS_TLS_CHACHA20_POLY1305_SHA256) return k.key_len == 32 ? ATLS_OK : ATLS_ILLEGAL_PARAMETER;
  if (k.suite == ATLS_TLS_AES_128_GCM_SHA256 || k.suite == ATLS_TLS_AES_256_GCM_SHA384)
    return (k.key_len == 16 || k.key_len == 24 || k.key_len == 32) ? ATLS_OK : ATLS_ILLEGAL_PARAMETER;
  return ATLS_INSUFFICIENT_SECURITY;
}

// Key slots [first, first + n) from host keys: the device key-setup kernel writes them in place
// (the table grows, keeping the other slots); replace = the table becomes exactly these n slots.
// Caller holds e->mu.
int install_keys(atls_engine* e, uint32_t first, const atls_key* keys, uint32_t n, bool replace) {
  ResidentHold hold;
  int status = ATLS_OK;
  for (uint32_t i = 0; i < n && status == ATLS_OK; i++) status = key_status(keys[i]);
  if (!set_dev(e)) return ATLS_INTERNAL_ERROR;
  if (join_pending(e)) return ATLS_INTERNAL_ERROR;  // no side kernel reads the table while it changes
  const uint32_t total = replace ? n : std::max(e->n_slots, first + n);
  const size_t need = sizeof(atls::KeySched) * (size_t)std::max<uint32_t>(total, 1);
  if (need > e->ks.cap) {  // grow, keeping the installed slots
    DevBuf grown;
    if (!grown.reserve(std::max(need, 2 * e->ks.cap))) return ATLS_INTERNAL_ERROR;
    if (!replace && e->n_slots &&
        hipMemcpyAsync(grown.p, e->ks.p, sizeof(atls::KeySched) * (size_t)e->n_slots, hipMemcpyDeviceToDevice,
                       e->stream) != hipSuccess)
      return ATLS_INTERNAL_ERROR;
    if (hipStreamSynchronize(e->stream) != hipSuccess) return ATLS_INTERNAL_ERROR;
    e->ks.release();
    e->ks = grown;
    grown.p = nullptr;
    grown.cap = 0;
  }
  // A few keys (a connection's new key, the single call's cache miss) travel in the key-setup kernel's
  // arguments: no staging copy and no host wait -- the kernel is ordered before every later batch by the
  // engine stream, and the other streams start from events recorded on it. More keys are staged by one
  // copy, and the call waits for the kernel (the caller's host array is read by that copy).
  const bool inl = n <= (uint32_t)atls_key_setup_inline_max();
  if (!inl) {
    if (!e->keys_stage.reserve(sizeof(atls_key) * (size_t)n)) return ATLS_INTERNAL_ERROR;
    if (hipMemcpyAsync(e->keys_stage.p, keys, sizeof(atls_key) * (size_t)n, hipMemcpyHostToDevice, e->stream) != hipSuccess)
      return ATLS_INTERNAL_ERROR;
  }
  if (atls_launch_key_setup(inl ? nullptr : (const atls_key*)e->keys_stage.p, keys, n, (atls::KeySched*)e->ks.p + first,
                            (const uint32_t*)e->t0.p, e->stream))
    return ATLS_INTERNAL_ERROR;
  if (!inl && hipStreamSynchronize(e->stream) != hipSuccess) return ATLS_INTERNAL_ERROR;
  if (replace) e->keys.clear();
  if (e->keys.size() < total) e->keys.resize(total);
  std::copy(keys, keys + n, e->keys.begin() + first);
  e->n_slots = total;
  e->has_aes = e->has_chacha = false;
  e->aes_nr_mask = 0;
  for (const atls_key& k : e->keys) {
    if (k.suite == ATLS_TLS_CHACHA20_POLY1305_SHA256) {
      e->has_chacha = true;
      continue;
    }
    e->has_aes = true;  // AES-GCM, or an invalid slot the GCM kernel reports
    if (key_status(k) == ATLS_OK) e->aes_nr_mask |= k.key_len == 16 ? 1 : k.key_len == 24 ? 2 : 4;
  }
  return status;
}

// ---- Cipher-trait calls (atls_seal / atls_open / atls_aes_block) ------------------------------
// The reference's record layer calls Cipher::encrypt / decrypt once per record from any thread
// (Arc<dyn Cipher + Send + Sync>, ciphersuite.rs:78-87, record.rs:191-193). A call leases a context
// from a bounded pool (at most ATLS_SINGLE_CONTEXTS, default 8; further callers wait for one): its
// own engines (one per kind of key: AES-128 / -192 / -256 / ChaCha20, so every call is a direct
// single-kernel batch) with a small key cache, pinned staging and its own streams. Calls of
// different threads run concurrently, a thread gets back the context it used last when it is free
// (its key cache), and a repeated key costs no key setup (the reference re-expands the key and
// recomputes H on every call, gcm.rs:52-56).
constexpr uint32_t kCacheSlots = 16;

struct KindEngine {
  atls_engine* e = nullptr;
  uint64_t stamp[kCacheSlots] = {};  // LRU clock per slot; 0 = free
  uint64_t clock = 0;
};

struct SingleCtx {
  KindEngine kinds[4];  // AES-128, AES-192, AES-256, ChaCha20-Poly1305
  int res_slot = -2;    // slot of the resident single-call server (-2: not asked yet, -1: none left)
  uint32_t res_seq = 0;
  uint8_t* pin = nullptr;  // page-locked, mapped into the device's address space
  uint8_t* pin_dev = nullptr;
  size_t pin_cap = 0;
  uint32_t calls = 0;  // completion-flag value of the last call (the flag word lives in the pinned block)
  bool reserve_pin(size_t n) {
    if (n <= pin_cap) return true;
    if (pin) (void)hipHostFree(pin);
    pin = pin_dev = nullptr;
    pin_cap = 0;
    size_t c = std::max<size_t>(n, size_t(1) << 16);
    void* p = nullptr;
    void* pd = nullptr;
    // fine-grained (coherent): the kernel's reads of the block see the host's latest writes and its
    // writes reach the host without a cache write-back
    if (hipHostMalloc(&p, c, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return false;
    if (hipHostGetDevicePointer(&pd, p, 0) != hipSuccess) {
      (void)hipHostFree(p);
      return false;
    }
    pin = (uint8_t*)p;
    pin_dev = (uint8_t*)pd;
    pin_cap = c;
    return true;
  }
};

struct CtxPool {
  std::mutex mu;
  std::condition_variable cv;
  std::vector<SingleCtx*> free;
  size_t created = 0;
  size_t max = [] {
    const char* v = std::getenv("ATLS_SINGLE_CONTEXTS");
    const long n = v ? std::atol(v) : 8;
    return (size_t)(n > 0 ? n : 8);
  }();
};
CtxPool& ctx_pool() {
  static CtxPool* pool = new CtxPool();  // never destroyed: outlives every thread
  return *pool;
}

// A context for the duration of one call; back to the pool when the lease ends.
struct CtxLease {
  SingleCtx* c = nullptr;
  CtxLease() {
    thread_local SingleCtx* last = nullptr;
    CtxPool& P = ctx_pool();
    std::unique_lock<std::mutex> lk(P.mu);
    for (;;) {
      auto it = std::find(P.free.begin(), P.free.end(), last);
      if (last && it != P.free.end()) {
        c = last;
        P.free.erase(it);
      } else if (!P.free.empty()) {
        c = P.free.back();
        P.free.pop_back();
      } else if (P.created < P.max) {
        c = new (std::nothrow) SingleCtx();
        if (c) P.created++;
      } else {
        P.cv.wait(lk);
        continue;
      }
      break;
    }
    last = c;
  }
  ~CtxLease() {
    if (!c) return;
    CtxPool& P = ctx_pool();
    {
      std::lock_guard<std::mutex> lk(P.mu);
      P.free.push_back(c);
    }
    P.cv.notify_one();
  }
};

int kind_of(uint16_t suite, size_t key_len) {
  if (suite == ATLS_TLS_CHACHA20_POLY1305_SHA256) return 3;
  return key_len == 16 ? 0 : key_len == 24 ? 1 : 2;
}

// Slot of this key in the context's engine of its kind, installing it (LRU eviction) on a miss.
int cached_slot(SingleCtx* c, uint16_t suite, const uint8_t* key, size_t key_len, atls_engine** eng, uint32_t* slot,
                bool* installed = nullptr) {
  if (installed) *installed = false;
  KindEngine& k = c->kinds[kind_of(suite, key_len)];
  if (!k.e) {
    const char* dv = std::getenv("ATLS_DEVICE");
    k.e = atls_engine_create(dv ? std::atoi(dv) : 0);
    if (!k.e) return ATLS_INTERNAL_ERROR;
  }
  *eng = k.e;
  uint32_t victim = 0;
  for (uint32_t i = 0; i < kCacheSlots; i++) {
    if (k.stamp[i] && i < k.e->keys.size() && k.e->keys[i].suite == suite && k.e->keys[i].key_len == key_len &&
        std::memcmp(k.e->keys[i].key, key, key_len) == 0) {
      k.stamp[i] = ++k.clock;
      *slot = i;
      return ATLS_OK;
    }
    if (k.stamp[i] < k.stamp[victim]) victim = i;
  }
  atls_key nk;
  std::memset(&nk, 0, sizeof nk);
  nk.suite = suite;
  nk.key_len = (uint8_t)key_len;
  nk.iv_len = 12;
  std::memcpy(nk.key, key, key_len);
  // slots fill in order, so a new slot never leaves a gap in the table
  const uint32_t s = std::min<uint32_t>(victim, (uint32_t)k.e->keys.size());
  int rc;
  {
    std::lock_guard<std::mutex> lk(k.e->mu);
    rc = install_keys(k.e, s, &nk, 1, false);
  }
  if (rc) return rc;
  k.stamp[s] = ++k.clock;
  *slot = s;
  if (installed) *installed = true;
  return ATLS_OK;
}

// ---- the resident single-call server (opt-in) ----
// ATLS_SINGLE_RESIDENT: 1 = ChaCha20-Poly1305 calls through the server, 2 = AES-GCM calls too (the server with
// the AES-GCM path serves ChaCha20-Poly1305 0-0.3 us slower: profiles/r05/single/resident_modes_noscratch.log)
int resident_mode() {
  static const int v = [] {
    const char* e = std::getenv("ATLS_SINGLE_RESIDENT");
    const int m = e ? std::atoi(e) : 0;
    return m == 1 || m == 2 ? m : 0;
  }();
  return v;
}
bool resident_enabled() { return resident_mode() != 0; }
uint32_t resident_idle_us() {  // ATLS_SINGLE_RESIDENT_IDLE_MS: how long a server waits for the next call (20 ms)
  static const uint32_t v = [] {
    const char* e = std::getenv("ATLS_SINGLE_RESIDENT_IDLE_MS");
    const long ms = e ? std::atol(e) : 20;
    return (uint32_t)std::min<long>(std::max<long>(ms, 1), 1000) * 1000u;
  }();
  return v;
}
// The process's resident single-call server for both suites (ATLS_SINGLE_RESIDENT=1, gcm.hip single_resident): one mapped, coherent block with a slot per call context (doorbell, flag, request, reply)
// and a common area (alive, stop), one stream, one workgroup -- a resident kernel holds a hardware queue,
// so there is one server for the whole process, not one per context.
constexpr int kResSlots = 8;
constexpr size_t kResBell = 0, kResFlag = 64, kResReq = 256, kResTag = 512, kResRes = 528, kResBytes = 1024,
                 kResOut = 8192, kResSlotBytes = 16384, kResCommon = kResSlots * kResSlotBytes, kResAlive = kResCommon,
                 kResStopAt = kResCommon + 64, kResBlock = kResCommon + 4096;
struct ResidentReqH {  // gcm.hip ResidentReq
  const void* ks;
  atls_rec d;
  uint32_t tag_off;
  uint32_t open;
  uint32_t nr;  // 0: ChaCha20-Poly1305; 10 / 12 / 14: AES-GCM
  uint32_t pad0;
  const void* t0;
  void* err;
  uint64_t pad1[5];
};
static_assert(sizeof(ResidentReqH) == 128, "gcm.hip ResidentReq");
struct ResidentServer {
  std::mutex mu;
  uint8_t* h = nullptr;
  uint8_t* d = nullptr;
  hipStream_t s = nullptr;
  int dev = -1;
  int slots_used = 0;
  bool failed = false;
};
ResidentServer& resident_server() {
  static ResidentServer* r = new ResidentServer();  // never destroyed: stopped by stop_resident at exit
  return *r;
}
// At exit the server is told to stop and waited for, before the runtime unmaps the block it polls.
void stop_resident() {
  ResidentServer& S = resident_server();
  std::lock_guard<std::mutex> lk(S.mu);
  if (!S.h) return;
  __atomic_store_n((uint32_t*)(S.h + kResStopAt), 1u, __ATOMIC_SEQ_CST);
  (void)hipSetDevice(S.dev);
  (void)hipStreamSynchronize(S.s);
}

// The context's slot of the server (allocating the server on first use): -1 when every slot is taken,
// the server failed, or the call runs on another device.
int resident_slot(SingleCtx* c, atls_engine* e) {
  if (c->res_slot != -2) return c->res_slot;
  ResidentServer& S = resident_server();
  std::lock_guard<std::mutex> lk(S.mu);
  c->res_slot = -1;
  if (S.failed) return -1;
  if (!S.h) {
    void* p = nullptr;
    void* pd = nullptr;
    if (hipHostMalloc(&p, kResBlock, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
      S.failed = true;
      return -1;
    }
    if (hipHostGetDevicePointer(&pd, p, 0) != hipSuccess || hipStreamCreateWithFlags(&S.s, hipStreamNonBlocking) != hipSuccess) {
      (void)hipHostFree(p);
      S.failed = true;
      return -1;
    }
    std::memset(p, 0, kResBlock);
    S.d = (uint8_t*)pd;
    __atomic_store_n(&S.h, (uint8_t*)p, __ATOMIC_RELEASE);  // ResidentHold reads it without S.mu
    S.dev = e->device;
    std::atexit(stop_resident);
  }
  if (S.dev != e->device || S.slots_used >= kResSlots) return -1;
  c->res_slot = S.slots_used++;
  return c->res_slot;
}

// A running server holds its hardware queue (GPU_MAX_HW_QUEUES is 4 per process), so any other kernel of the
// process whose stream maps to that queue would wait for the server's idle timeout. Every entry point that
// launches work of its own therefore holds a ResidentHold from before its first launch until it returns: the
// hold counts itself in g_res_holds and stops a running server (stop word, wait for alive == 0, clear the word);
// while any hold is live no call relaunches the server (resident_launch_locked refuses, and the call takes the
// launch path instead), so a batch can neither be overtaken by a relaunch between its yield and its own
// launches nor wait behind a server kept alive by other threads' calls. The
// count is raised before S.mu is taken and a relaunch reads it under S.mu, so either the relaunch sees the hold
// or the hold's stop sees the relaunched server.
std::atomic<int> g_res_holds{0};
unsigned long long g_res_fallbacks = 0;  // calls that found the server busy and took the launch path
constexpr int kResidentBusy = -1;  // resident_call: a launch of the process is in flight, use the launch path

void resident_stop(ResidentServer& S) {
  std::lock_guard<std::mutex> lk(S.mu);
  uint32_t* alive = (uint32_t*)(S.h + kResAlive);
  uint32_t* stop = (uint32_t*)(S.h + kResStopAt);
  if (__atomic_load_n(alive, __ATOMIC_SEQ_CST) == 0) return;
  __atomic_store_n(stop, 1u, __ATOMIC_SEQ_CST);
  const auto t0 = std::chrono::steady_clock::now();
  while (__atomic_load_n(alive, __ATOMIC_ACQUIRE) != 0 && std::chrono::steady_clock::now() - t0 < std::chrono::seconds(2))
    __builtin_ia32_pause();
  (void)hipStreamSynchronize(S.s);  // the kernel itself has ended
  __atomic_store_n(alive, 0u, __ATOMIC_SEQ_CST);
  __atomic_store_n(stop, 0u, __ATOMIC_SEQ_CST);
}

// ResidentHold's constructor and destructor (engine_internal.h) use these; they follow the anonymous namespace.
void resident_hold_begin() {
  if (!resident_enabled()) return;
  g_res_holds.fetch_add(1, std::memory_order_seq_cst);
  ResidentServer& S = resident_server();
  if (__atomic_load_n(&S.h, __ATOMIC_ACQUIRE)) resident_stop(S);
}

// Launches the server unless it runs (caller holds S.mu); kResidentBusy while a hold is live. The kernel's last
// store is alive := 0, so a server seen alive == 0 is gone or about to be; a new one on the same stream starts
// after it.
int resident_launch_locked(ResidentServer& S) {
  if (__atomic_load_n((uint32_t*)(S.h + kResAlive), __ATOMIC_SEQ_CST) != 0) return ATLS_OK;
  if (g_res_holds.load(std::memory_order_seq_cst) > 0) return kResidentBusy;
  __atomic_store_n((uint32_t*)(S.h + kResAlive), 1u, __ATOMIC_SEQ_CST);
  return atls_launch_single_resident(S.d, resident_idle_us(), resident_mode() == 2 ? 1 : 0, S.s);
}

// One call through the server: request into the context's slot, doorbell, then the slot's flag. Returns
// ATLS_OK (outputs in the slot), kResidentBusy (not served: take the launch path) or ATLS_INTERNAL_ERROR.
int resident_call(SingleCtx* c, const void* ks, const atls_rec& d, const uint8_t* bytes, uint32_t nbytes, uint32_t tag_off,
                  bool open, uint32_t nr, const void* t0tab, void* err) {
  ResidentServer& S = resident_server();
  uint8_t* h = S.h + (size_t)c->res_slot * kResSlotBytes;
  const ResidentReqH q{ks, d, tag_off, open ? 1u : 0u, nr, 0u, t0tab, err, {0, 0, 0, 0, 0}};
  std::memcpy(h + kResReq, &q, sizeof q);
  std::memcpy(h + kResBytes, bytes, nbytes);
  uint32_t v = ++c->res_seq;
  if (v == 0) v = c->res_seq = 1;
  uint32_t* flag = (uint32_t*)(h + kResFlag);
  const uint32_t* alive = (const uint32_t*)(S.h + kResAlive);
  __atomic_store_n(flag, v - 1u, __ATOMIC_RELEASE);  // pending: doorbell != flag
  __atomic_store_n((uint32_t*)(h + kResBell), v, __ATOMIC_SEQ_CST);
  // A relaunch refused because a launch of the process is in flight: no server runs (alive == 0 and the hold's
  // stop waited for the kernel to end), so the request is withdrawn (flag := doorbell, nothing pending for a
  // later server) and the call goes down the launch path.
  auto relaunch = [&]() -> int {
    const int rc = resident_launch_locked(S);
    if (rc == kResidentBusy) __atomic_store_n(flag, v, __ATOMIC_RELEASE);
    return rc == kResidentBusy ? kResidentBusy : rc ? ATLS_INTERNAL_ERROR : ATLS_OK;
  };
  if (__atomic_load_n(alive, __ATOMIC_SEQ_CST) == 0) {
    std::lock_guard<std::mutex> lk(S.mu);
    if (const int rc = relaunch()) return rc;
  }
  const auto t0 = std::chrono::steady_clock::now();
  for (uint64_t i = 1;; i++) {
    if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == v) return ATLS_OK;
    if ((i & 255) == 0 && __atomic_load_n(alive, __ATOMIC_ACQUIRE) == 0) {
      // the server left (idle) before it saw this call: its flag stores precede alive := 0, so look once more
      if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == v) return ATLS_OK;
      std::lock_guard<std::mutex> lk(S.mu);
      if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == v) return ATLS_OK;
      if (const int rc = relaunch()) return rc;
    }
    if ((i & 4095) == 0) {
      const hipError_t qs = hipStreamQuery(S.s);
      if (qs != hipSuccess && qs != hipErrorNotReady) return ATLS_INTERNAL_ERROR;
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
        std::fprintf(stderr, "anothertls_amd: resident server did not answer in 2 s (slot %d bell %u flag %u alive %u)\n",
                     c->res_slot, v, __atomic_load_n(flag, __ATOMIC_ACQUIRE), __atomic_load_n(alive, __ATOMIC_ACQUIRE));
        return ATLS_INTERNAL_ERROR;
      }
    }
    __builtin_ia32_pause();
  }
}

// Records up to this many bytes are read by the kernel straight from the pinned staging block
// (mapped host memory, no copy); longer ones are staged to the device in one copy. Outputs always
// go straight to the pinned block. Measured (profiles/r03/single_call_latency_zc*.json, median us
// per call): 16,385-B AES-128-GCM seal 54.7 read in place vs 60.3 with the copy, 1,537 B 30 either
// way. ATLS_SINGLE_ZC_MAX overrides (tuning).
size_t single_zero_copy_max() {
  static const size_t v = [] {
    const char* e = std::getenv("ATLS_SINGLE_ZC_MAX");
    return e ? (size_t)std::atol(e) : (size_t)1 << 20;
  }();
  return v;
}

// ATLS_SINGLE_INLINE=0 sends every single call through the pinned-block path (A/B of the argument-block
// path, tests).
bool single_inline() {
  static const bool v = [] {
    const char* e = std::getenv("ATLS_SINGLE_INLINE");
    return !e || std::atoi(e) != 0;
  }();
  return v;
}

// 128-bit canary in the pinned tag slot of a seal: a kernel that refused the record leaves it in
// place. Refusals cannot happen here (the descriptor is built and checked on the host exactly as
// direct_reject checks it); the canary keeps a refusal from passing unnoticed all the same, at a
// false-alarm rate of 2^-128.
constexpr uint32_t kTagCanary[4] = {0x6c1f9a3du, 0xb2e4570cu, 0x93d0e8a1u, 0x0f7b2c56u};

// One Cipher::encrypt / decrypt call as a single RAW record: descriptor, tag, IV, AAD and input
// are written into the context's pinned block, the kernel reads them there (or from one copy of
// the block for long records), writes output, tag and result straight back into it and then a
// completion flag the host spins on (no wait for the launch's completion signal). No other copy
// and no descriptor upload.
int single(bool open, uint16_t suite, const uint8_t* key, size_t key_len, const uint8_t* iv, size_t iv_len,
           const uint8_t* aad, size_t aad_len, const uint8_t* in, size_t len, const uint8_t* tag_in, size_t tag_len,
           uint8_t* out, uint8_t* tag_out) {
  if (suite != ATLS_TLS_AES_128_GCM_SHA256 && suite != ATLS_TLS_AES_256_GCM_SHA384 &&
      suite != ATLS_TLS_CHACHA20_POLY1305_SHA256)
    return ATLS_INSUFFICIENT_SECURITY;  // CipherSuite::get_cipher, ciphersuite.rs:78-87
  if (suite == ATLS_TLS_CHACHA20_POLY1305_SHA256) {
    if (key_len != 32 || iv_len != 12) return ATLS_ILLEGAL_PARAMETER;  // poly1305.rs:20 unwrap
    // ChaCha20::encrypt counts blocks as f32 (chacha20/cipher.rs:94), exact only below 2^24 B:
    // longer inputs are refused rather than sealed differently from the reference
    if (len >= (size_t(1) << 24)) return ATLS_ILLEGAL_PARAMETER;
  } else if (key_len != 16 && key_len != 24 && key_len != 32) {
    return ATLS_ILLEGAL_PARAMETER;  // gcm.rs:49 unwrap
  }
  if (iv_len > 255 || aad_len > 0xffff || len > 0xffffffffull) return ATLS_ILLEGAL_PARAMETER;
  if (open && tag_len != 16) return ATLS_BAD_RECORD_MAC;  // `T != auth_tag` with a wrong-length slice
  CtxLease lease;
  SingleCtx* c = lease.c;
  if (!c) return ATLS_INTERNAL_ERROR;
  atls_engine* e = nullptr;
  uint32_t slot = 0;
  bool installed = false;
  int rc = cached_slot(c, suite, key, key_len, &e, &slot, &installed);
  if (rc) return rc;
  // pinned block: descriptor | tag | open result | completion flag | iv || aad | input | output
  const size_t rec_at = 0, tag_at = 64, res_at = 80, done_at = 88, aux_at = 96;
  const size_t in_at = (aux_at + iv_len + aad_len + 15) & ~size_t(15);
  const size_t out_at = (in_at + len + 15) & ~size_t(15), total = out_at + len + 16;
  if (!c->reserve_pin(total)) return ATLS_INTERNAL_ERROR;
  uint8_t* h = c->pin;
  atls_rec r;
  std::memset(&r, 0, sizeof r);
  r.in_off = in_at;
  r.out_off = out_at;
  r.aux_off = aux_at;
  r.len = (uint32_t)len;
  r.key_slot = slot;
  r.mode = ATLS_MODE_RAW;
  r.iv_len = (uint8_t)iv_len;
  r.aad_len = (uint16_t)aad_len;
  // IV || AAD || input || tag that fit the launch's argument block go there with the descriptor
  // (gcm_single / chacha_single): the kernel makes no dependent reads of mapped host memory before its
  // first round. Longer records: the kernel reads descriptor and data from the pinned block (or a copy).
  const size_t inl_in = (iv_len + aad_len + 15) & ~size_t(15), inl_tag = (inl_in + len + 15) & ~size_t(15);
  const bool inl = single_inline() && inl_tag + (open ? 16 : 0) <= atls::kSingleInline;
  if (open) {
    std::memset(h + res_at, 0xff, sizeof(atls_open_result));  // the kernel writes every field
  } else {
    std::memcpy(h + tag_at, kTagCanary, 16);
  }
  if (!inl) {
    std::memcpy(h + rec_at, &r, sizeof r);
    if (open) std::memcpy(h + tag_at, tag_in, 16);
    if (iv_len) std::memcpy(h + aux_at, iv, iv_len);
    if (aad_len) std::memcpy(h + aux_at + iv_len, aad, aad_len);
    if (len) std::memcpy(h + in_at, in, len);
  }
  std::lock_guard<std::mutex> lk(e->mu);
  if (!set_dev(e)) return ATLS_INTERNAL_ERROR;
  hipStream_t s = e->stream;
  if (inl && resident_enabled() && (suite == ATLS_TLS_CHACHA20_POLY1305_SHA256 || resident_mode() == 2) &&
      resident_slot(c, e) >= 0) {
    // the resident server: no launch per call (the new key's setup, if any, finishes first)
    if (installed && hipStreamSynchronize(s) != hipSuccess) return ATLS_INTERNAL_ERROR;
    uint8_t bytes[atls::kSingleInline];
    if (iv_len) std::memcpy(bytes, iv, iv_len);
    if (aad_len) std::memcpy(bytes + iv_len, aad, aad_len);
    if (len) std::memcpy(bytes + inl_in, in, len);
    if (open) std::memcpy(bytes + inl_tag, tag_in, 16);
    atls_rec d = r;
    d.in_off = inl_in;
    d.aux_off = 0;
    d.out_off = 0;
    uint8_t* rh = resident_server().h + (size_t)c->res_slot * kResSlotBytes;
    if (open) std::memset(rh + kResRes, 0xff, sizeof(atls_open_result));  // the server writes every field
    else std::memcpy(rh + kResTag, kTagCanary, 16);
    const bool chacha = suite == ATLS_TLS_CHACHA20_POLY1305_SHA256;
    rc = resident_call(c, (const atls::KeySched*)e->ks.p + slot, d, bytes, (uint32_t)(inl_tag + (open ? 16 : 0)),
                       (uint32_t)inl_tag, open, chacha ? 0u : (uint32_t)key_len / 4u + 6u, e->t0.p, e->err.p);
    if (rc != kResidentBusy) {
      if (rc) return rc;
      if (!open) {
        if (std::memcmp(rh + kResTag, kTagCanary, 16) == 0) return ATLS_ILLEGAL_PARAMETER;
        if (len) std::memcpy(out, rh + kResOut, len);
        std::memcpy(tag_out, rh + kResTag, 16);
        return ATLS_OK;
      }
      atls_open_result res;
      std::memcpy(&res, rh + kResRes, sizeof res);
      if (res.status != ATLS_OK) {
        if (len) std::memset(out, 0, len);
        return res.status;
      }
      if (len) std::memcpy(out, rh + kResOut, len);
      return ATLS_OK;
    }
    // busy: another thread's launch is in flight (a batch, a key install); this call is launched like it
    __atomic_fetch_add(&g_res_fallbacks, 1ull, __ATOMIC_RELAXED);
  }
  ResidentHold hold;
  uint8_t* hd = c->pin_dev;
  const uint32_t done_val = ++c->calls;
  // the flag word holds anything after a (re)allocation of the block: set it to a value other than
  // done_val, so only this launch's store ends the spin
  __atomic_store_n((uint32_t*)(h + done_at), done_val - 1u, __ATOMIC_RELEASE);
  if (inl) {
    uint8_t bytes[atls::kSingleInline];
    if (iv_len) std::memcpy(bytes, iv, iv_len);
    if (aad_len) std::memcpy(bytes + iv_len, aad, aad_len);
    if (len) std::memcpy(bytes + inl_in, in, len);
    if (open) std::memcpy(bytes + inl_tag, tag_in, 16);
    atls_rec d = r;
    d.in_off = inl_in;
    d.aux_off = 0;
    const uint32_t nbytes = (uint32_t)(inl_tag + (open ? 16 : 0));
    rc = suite == ATLS_TLS_CHACHA20_POLY1305_SHA256
             ? atls_launch_chacha_single(open, e->ks.p, e->n_slots, &d, bytes, nbytes, (uint32_t)inl_tag, hd,
                                         hd + tag_at, (atls_open_result*)(hd + res_at), (uint32_t*)e->err.p,
                                         (uint32_t*)(hd + done_at), done_val, s)
             : atls_launch_gcm_single(open, (int)key_len / 4 + 6, e->ks.p, e->n_slots, &d, bytes, nbytes,
                                      (uint32_t)inl_tag, hd, hd + tag_at, (atls_open_result*)(hd + res_at),
                                      (const uint32_t*)e->t0.p, (uint32_t*)e->err.p, (uint32_t*)(hd + done_at),
                                      done_val, s);
  } else {
    const uint8_t* src = hd;  // descriptor, aux, tag-in and input: read in place ...
    if (len > single_zero_copy_max()) {  // ... or from one copy of the block
      if (!e->in.reserve(out_at) || hipMemcpyAsync(e->in.p, h, out_at, hipMemcpyHostToDevice, s) != hipSuccess)
        return ATLS_INTERNAL_ERROR;
      src = (const uint8_t*)e->in.p;
    }
    rc = launch_records(e, open, (const atls_rec*)(src + rec_at), 1, src, src, hd, hd + tag_at, src + tag_at,
                        (atls_open_result*)(hd + res_at), s, (uint32_t*)(hd + done_at), done_val);
  }
  if (rc) return rc;
  // spin on the kernel's completion flag (visible once every output byte is); a stream that ends
  // without it (a fault) is reported by hipStreamQuery, checked every few thousand spins
  const uint32_t* done = (const uint32_t*)(h + done_at);
  for (uint64_t i = 1;; i++) {
    if (__atomic_load_n(done, __ATOMIC_ACQUIRE) == done_val) break;
    if ((i & 4095) == 0) {
      const hipError_t q = hipStreamQuery(s);
      if (q == hipSuccess) {
        if (__atomic_load_n(done, __ATOMIC_ACQUIRE) == done_val) break;
        return ATLS_INTERNAL_ERROR;  // the launch ended and never signalled
      }
      if (q != hipErrorNotReady) return ATLS_INTERNAL_ERROR;
    }
    __builtin_ia32_pause();
  }
  if (!open) {
    if (std::memcmp(h + tag_at, kTagCanary, 16) == 0) return ATLS_ILLEGAL_PARAMETER;
    if (len) std::memcpy(out, h + out_at, len);
    std::memcpy(tag_out, h + tag_at, 16);
    return ATLS_OK;
  }
  atls_open_result res;
  std::memcpy(&res, h + res_at, sizeof res);
  if (res.status != ATLS_OK) {
    if (len) std::memset(out, 0, len);  // no unauthenticated plaintext leaves (reference returns Err)
    return res.status;
  }
  if (len) std::memcpy(out, h + out_at, len);
  return ATLS_OK;
}

}  // namespace

atls::ResidentHold::ResidentHold() : active(resident_enabled()) {
  if (active) resident_hold_begin();
}
atls::ResidentHold::~ResidentHold() {
  if (active) g_res_holds.fetch_sub(1, std::memory_order_seq_cst);
}

uint32_t atls::engine_slots(atls_engine* e) {
  if (!e) return 0;
  std::lock_guard<std::mutex> lk(e->mu);
  return e->n_slots;
}

extern "C" {

int atls_abi_version(void) { return ATLS_ABI_VERSION; }
const char* atls_device_arch(void) { return "gfx950"; }

atls_engine* atls_engine_create(int device) {
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || device < 0 || device >= count) return nullptr;
  ResidentHold hold;  // the T-table build below is a launch
  atls_engine* e = new (std::nothrow) atls_engine();
  if (!e) return nullptr;
  e->device = device;
  hipDeviceProp_t prop;
  if (hipSetDevice(device) != hipSuccess || hipGetDeviceProperties(&prop, device) != hipSuccess ||
      hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&e->stream2, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&e->ev_plan, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&e->ev_side, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&e->ps[0].side_done, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&e->ps[1].side_done, hipEventDisableTiming) != hipSuccess) {
    for (auto& q : e->ps)
      if (q.side_done) (void)hipEventDestroy(q.side_done);
    if (e->ev_plan) (void)hipEventDestroy(e->ev_plan);
    if (e->ev_side) (void)hipEventDestroy(e->ev_side);
    if (e->stream2) (void)hipStreamDestroy(e->stream2);
    if (e->stream) (void)hipStreamDestroy(e->stream);
    delete e;
    return nullptr;
  }
  e->cus = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
  if (const char* v = std::getenv("ATLS_FORCE_PLAN")) e->force_plan = std::atoi(v) != 0;
  if (const char* v = std::getenv("ATLS_NO_PIPELINE")) e->no_pipeline = std::atoi(v) != 0;
  if (const char* v = std::getenv("ATLS_CHACHA_WGS")) e->chacha_wgs = std::max(1, std::atoi(v));
  if (const char* v = std::getenv("ATLS_CHACHA_W2")) e->chacha_w2 = std::atoi(v);
  if (const char* v = std::getenv("ATLS_ZERO_COPY")) e->zero_copy = std::atoi(v);
  if (const char* v = std::getenv("ATLS_GCM_GROUP_MIN")) e->group_min = (uint32_t)std::max(0, std::atoi(v));
  if (const char* v = std::getenv("ATLS_GCM_TAIL_ON")) e->tail_on = std::atoi(v) != 0;
  if (const char* v = std::getenv("ATLS_SYNC_FLAG")) e->sync_flag = std::atoi(v) != 0;
  if (!e->t0.reserve(256 * 4) || !e->err.reserve(16) || hipMemsetAsync(e->err.p, 0, 16, e->stream) != hipSuccess ||
      atls_launch_build_t0((uint32_t*)e->t0.p, e->stream) ||
      hipStreamSynchronize(e->stream) != hipSuccess) {
    atls_engine_destroy(e);
    return nullptr;
  }
  return e;
}

void atls_engine_destroy(atls_engine* e) {
  if (!e) return;
  ResidentHold hold;  // its streams' last kernels must not sit behind a running server
  (void)hipSetDevice(e->device);
  if (e->stream) (void)hipStreamSynchronize(e->stream);
  if (e->stream2) (void)hipStreamSynchronize(e->stream2);
  for (DevBuf* b : {&e->ks, &e->t0, &e->err, &e->keys_stage, &e->recs, &e->in, &e->out, &e->aux, &e->tags, &e->res,
                    &e->secrets, &e->dkeys, &e->grp_cnt, &e->grp_aux, &e->grp_idx, &e->tail})
    b->release();
  for (auto& q : e->ps) {
    for (DevBuf* b : {&q.plan, &q.keys, &q.idx, &q.wg}) b->release();
    if (q.side_done) (void)hipEventDestroy(q.side_done);
  }
  if (e->ev_plan) (void)hipEventDestroy(e->ev_plan);
  if (e->ev_side) (void)hipEventDestroy(e->ev_side);
  for (hipEvent_t ev : e->pev) (void)hipEventDestroy(ev);
  if (e->up) (void)hipStreamDestroy(e->up);
  if (e->down) (void)hipStreamDestroy(e->down);
  if (e->stream2) (void)hipStreamDestroy(e->stream2);
  if (e->stream) (void)hipStreamDestroy(e->stream);
  if (e->sync_h) (void)hipHostFree(e->sync_h);
  delete e;
}

int atls_engine_sync(atls_engine* e) {
  if (!e) return ATLS_INTERNAL_ERROR;
  ResidentHold hold;  // finish may launch the completion-flag kernel
  std::lock_guard<std::mutex> lk(e->mu);
  if (!set_dev(e)) return ATLS_INTERNAL_ERROR;
  return finish(e, 0);
}

int atls_engine_join(atls_engine* e) {
  if (!e) return ATLS_INTERNAL_ERROR;
  std::lock_guard<std::mutex> lk(e->mu);
  if (!set_dev(e)) return ATLS_INTERNAL_ERROR;
  return join_pending(e);
}

void* atls_engine_stream(atls_engine* e) { return e ? (void*)e->stream : nullptr; }

int atls_set_keys(atls_engine* e, const atls_key* keys, uint32_t n) {
  if (!e || (!keys && n)) return ATLS_INTERNAL_ERROR;
  std::lock_guard<std::mutex> lk(e->mu);
  return install_keys(e, 0, keys, n, true);
}

int atls_update_keys(atls_engine* e, uint32_t first, const atls_key* keys, uint32_t n) {
  if (!e || (!keys && n)) return ATLS_INTERNAL_ERROR;
  std::lock_guard<std::mutex> lk(e->mu);
  if (first > e->n_slots) return ATLS_ILLEGAL_PARAMETER;  // slots stay contiguous
  return install_keys(e, first, keys, n, false);
}

int atls_seal_batch(atls_engine* e, const atls_rec* recs, uint32_t n, const void* in, const void* aux, void* out,
                    uint8_t* tags, uint32_t flags) {
  return run_batch(e, false, recs, n, in, aux, out, tags, nullptr, nullptr, flags);
}

int atls_open_batch(atls_engine* e, const atls_rec* recs, uint32_t n, const void* in, const void* aux,
                    const uint8_t* tags, void* out, atls_open_result* results, uint32_t flags) {
  return run_batch(e, true, recs, n, in, aux, out, nullptr, tags, results, flags);
}

int atls_seal(uint16_t suite, const uint8_t* key, size_t key_len, const uint8_t* iv, size_t iv_len,
              const uint8_t* aad, size_t aad_len, const uint8_t* in, size_t len, uint8_t* out, uint8_t tag[16]) {
  return single(false, suite, key, key_len, iv, iv_len, aad, aad_len, in, len, nullptr, 0, out, tag);
}

int atls_open(uint16_t suite, const uint8_t* key, size_t key_len, const uint8_t* iv, size_t iv_len,
              const uint8_t* aad, size_t aad_len, const uint8_t* in, size_t len, const uint8_t* tag, size_t tag_len,
              uint8_t* out) {
  return single(true, suite, key, key_len, iv, iv_len, aad, aad_len, in, len, tag, tag_len, out, nullptr);
}

int atls_derive_keys(atls_engine* e, uint16_t suite, const uint8_t* secrets, size_t secret_len, uint32_t n,
                     atls_key* out_keys) {
  if (!e) return ATLS_INTERNAL_ERROR;
  ResidentHold hold;
  if (suite != ATLS_TLS_AES_128_GCM_SHA256 && suite != ATLS_TLS_AES_256_GCM_SHA384 &&
      suite != ATLS_TLS_CHACHA20_POLY1305_SHA256)
    return ATLS_INSUFFICIENT_SECURITY;
  const size_t hl = suite == ATLS_TLS_AES_256_GCM_SHA384 ? 48 : 32;  // CipherSuite::get_tshash
  if (secret_len != hl) return ATLS_ILLEGAL_PARAMETER;
  if (n == 0) return ATLS_OK;
  std::lock_guard<std::mutex> lk(e->mu);
  if (!set_dev(e)) return ATLS_INTERNAL_ERROR;
  if (!e->secrets.reserve(secret_len * n) || !e->dkeys.reserve(sizeof(atls_key) * (size_t)n)) return ATLS_INTERNAL_ERROR;
  if (hipMemcpyAsync(e->secrets.p, secrets, secret_len * n, hipMemcpyHostToDevice, e->stream) != hipSuccess)
    return ATLS_INTERNAL_ERROR;
  if (atls_launch_derive(suite, (const uint8_t*)e->secrets.p, (uint32_t)secret_len, n, (atls_key*)e->dkeys.p, e->stream))
    return ATLS_INTERNAL_ERROR;
  if (hipMemcpyAsync(out_keys, e->dkeys.p, sizeof(atls_key) * (size_t)n, hipMemcpyDeviceToHost, e->stream) != hipSuccess)
    return ATLS_INTERNAL_ERROR;
  return hipStreamSynchronize(e->stream) == hipSuccess ? ATLS_OK : ATLS_INTERNAL_ERROR;
}

int atls_hash_batch(atls_engine* e, int op, uint32_t hash_len, const uint8_t* data, size_t data_len,
                    const atls_span* keys, const atls_span* msgs, uint32_t n, uint32_t out_len, uint8_t* out) {
  if (!e) return ATLS_INTERNAL_ERROR;
  ResidentHold hold;
  if ((hash_len != 32 && hash_len != 48) || op < ATLS_HASH_SHA || op > ATLS_HASH_HKDF_EXPAND || !msgs ||
      (op != ATLS_HASH_SHA && !keys))
    return ATLS_ILLEGAL_PARAMETER;
  if (op == ATLS_HASH_HKDF_EXPAND ? out_len > 255u * hash_len : out_len != hash_len)
    return ATLS_ILLEGAL_PARAMETER;  // hkdf.rs:38 returns None past 255 * HashLen
  for (uint32_t i = 0; i < n; i++) {  // every span inside data
    if (msgs[i].off > data_len || msgs[i].len > data_len - msgs[i].off) return ATLS_ILLEGAL_PARAMETER;
    if (op != ATLS_HASH_SHA && (keys[i].off > data_len || keys[i].len > data_len - keys[i].off))
      return ATLS_ILLEGAL_PARAMETER;
  }
  if (n == 0) return ATLS_OK;
  std::lock_guard<std::mutex> lk(e->mu);
  if (!set_dev(e)) return ATLS_INTERNAL_ERROR;
  hipStream_t s = e->stream;
  const size_t span_bytes = sizeof(atls_span) * (size_t)n, out_bytes = (size_t)out_len * n;
  if (!e->secrets.reserve(data_len + 2 * span_bytes + 64) || !e->dkeys.reserve(out_bytes + 16)) return ATLS_INTERNAL_ERROR;
  uint8_t* d = (uint8_t*)e->secrets.p;
  atls_span* dk = (atls_span*)(d + ((data_len + 15) & ~size_t(15)));
  atls_span* dm = dk + n;
  if ((data_len && hipMemcpyAsync(d, data, data_len, hipMemcpyHostToDevice, s) != hipSuccess) ||
      (keys && hipMemcpyAsync(dk, keys, span_bytes, hipMemcpyHostToDevice, s) != hipSuccess) ||
      hipMemcpyAsync(dm, msgs, span_bytes, hipMemcpyHostToDevice, s) != hipSuccess)
    return ATLS_INTERNAL_ERROR;
  if (atls_launch_hash(op, hash_len, d, keys ? dk : nullptr, dm, n, out_len, (uint8_t*)e->dkeys.p, s)) return ATLS_INTERNAL_ERROR;
  if (hipMemcpyAsync(out, e->dkeys.p, out_bytes, hipMemcpyDeviceToHost, s) != hipSuccess) return ATLS_INTERNAL_ERROR;
  return hipStreamSynchronize(s) == hipSuccess ? ATLS_OK : ATLS_INTERNAL_ERROR;
}

int atls_key_schedule(atls_engine* e, uint32_t hash_len, const uint8_t* shared, size_t shared_len,
                      const uint8_t* hello_hashes, const uint8_t* handshake_hashes, uint32_t n, uint8_t* out) {
  if (!e) return ATLS_INTERNAL_ERROR;
  ResidentHold hold;
  if ((hash_len != 32 && hash_len != 48) || !shared || !hello_hashes || shared_len > 1024) return ATLS_ILLEGAL_PARAMETER;
  if (n == 0) return ATLS_OK;
  std::lock_guard<std::mutex> lk(e->mu);
  if (!set_dev(e)) return ATLS_INTERNAL_ERROR;
  hipStream_t s = e->stream;
  const size_t sb = shared_len * n, hb = (size_t)hash_len * n, ob = 5 * (size_t)hash_len * n;
  const size_t a0 = (sb + 15) & ~size_t(15), a1 = a0 + ((hb + 15) & ~size_t(15));
  if (!e->secrets.reserve(a1 + hb + 16) || !e->dkeys.reserve(ob + 16)) return ATLS_INTERNAL_ERROR;
  uint8_t* d = (uint8_t*)e->secrets.p;
  if (hipMemcpyAsync(d, shared, sb, hipMemcpyHostToDevice, s) != hipSuccess ||
      hipMemcpyAsync(d + a0, hello_hashes, hb, hipMemcpyHostToDevice, s) != hipSuccess ||
      (handshake_hashes && hipMemcpyAsync(d + a1, handshake_hashes, hb, hipMemcpyHostToDevice, s) != hipSuccess) ||
      hipMemsetAsync(e->dkeys.p, 0, ob, s) != hipSuccess)
    return ATLS_INTERNAL_ERROR;
  if (atls_launch_key_schedule(hash_len, d, (uint32_t)shared_len, d + a0, handshake_hashes ? d + a1 : nullptr, n,
                               (uint8_t*)e->dkeys.p, s))
    return ATLS_INTERNAL_ERROR;
  if (hipMemcpyAsync(out, e->dkeys.p, ob, hipMemcpyDeviceToHost, s) != hipSuccess) return ATLS_INTERNAL_ERROR;
  return hipStreamSynchronize(s) == hipSuccess ? ATLS_OK : ATLS_INTERNAL_ERROR;
}

int atls_aes_blocks(atls_engine* e, int decrypt, uint32_t key_slot, const void* in, void* out, size_t nblocks,
                    uint32_t flags) {
  if (!e) return ATLS_INTERNAL_ERROR;
  ResidentHold hold;
  if (nblocks == 0) return ATLS_OK;
  std::lock_guard<std::mutex> lk(e->mu);
  if (!set_dev(e)) return ATLS_INTERNAL_ERROR;
  if (key_slot >= e->n_slots) return ATLS_ILLEGAL_PARAMETER;
  hipStream_t s = e->stream;
  const size_t bytes = 16 * nblocks;
  const bool dev = flags & ATLS_FLAG_DEVICE_PTRS;
  const uint8_t* d_in = (const uint8_t*)in;
  uint8_t* d_out = (uint8_t*)out;
  if (!dev) {
    if (!e->in.reserve(bytes) || !e->out.reserve(bytes) ||
        hipMemcpyAsync(e->in.p, in, bytes, hipMemcpyHostToDevice, s) != hipSuccess)
      return ATLS_INTERNAL_ERROR;
    d_in = (const uint8_t*)e->in.p;
    d_out = (uint8_t*)e->out.p;
  }
  if (atls_launch_aes_blocks(decrypt, (const atls::KeySched*)e->ks.p + key_slot, d_in, d_out, nblocks,
                             (uint32_t*)e->err.p, e->cus * 8, s))
    return ATLS_INTERNAL_ERROR;
  if (!dev) {
    if (hipMemcpyAsync(out, e->out.p, bytes, hipMemcpyDeviceToHost, s) != hipSuccess) return ATLS_INTERNAL_ERROR;
    return finish(e, flags & ~ATLS_FLAG_NO_SYNC, true);
  }
  return finish(e, flags);
}

int atls_clock_probe(atls_engine* e, void* stream, uint32_t wgs, uint32_t delay_us, uint32_t spin_us, uint64_t* out) {
  if (!e) return ATLS_INTERNAL_ERROR;
  if (!out || wgs == 0 || wgs > 1024 || delay_us > 10000000u || spin_us > 10000000u) return ATLS_ILLEGAL_PARAMETER;
  if (!set_dev(e)) return ATLS_INTERNAL_ERROR;
  return atls_launch_clock_probe(wgs, delay_us, spin_us, out, stream ? (hipStream_t)stream : e->stream);
}

int atls_aes_block(int decrypt, const uint8_t* key, size_t key_len, const uint8_t in[16], uint8_t out[16]) {
  if (key_len != 16 && key_len != 24 && key_len != 32) return ATLS_ILLEGAL_PARAMETER;  // AES::init key sizes
  CtxLease lease;
  SingleCtx* c = lease.c;
  if (!c) return ATLS_INTERNAL_ERROR;
  atls_engine* e = nullptr;
  uint32_t slot = 0;
  // any AES suite: the slot only carries the key (the thread's engine of this key size)
  const int rc = cached_slot(c, ATLS_TLS_AES_128_GCM_SHA256, key, key_len, &e, &slot);
  return rc ? rc : atls_aes_blocks(e, decrypt, slot, in, out, 1, 0);
}

}  // extern "C"

// Debug: copy key slot `slot`'s device key schedule (atls_dev.h KeySched, 3,648 B) to host, for the tests
// of the key-setup kernel against a host model (tests/test_gpu_keysetup.py). Returns its size or -1.
// Host-memory batches that could not be pipelined because their records were out of order (staged in one piece).
extern "C" unsigned long long atls_debug_host_unpipelined(void) {
  return __atomic_load_n(&g_host_unpipelined, __ATOMIC_RELAXED);
}

// Single calls that found the resident server held by another thread's launch and took the launch path instead
// (tests/helpers/resident_check.py).
extern "C" unsigned long long atls_debug_resident_fallbacks(void) {
  return __atomic_load_n(&g_res_fallbacks, __ATOMIC_RELAXED);
}

extern "C" int atls_debug_key_sched(atls_engine* e, uint32_t slot, void* out, size_t cap) {
  if (!e || !out || cap < sizeof(atls::KeySched)) return -1;
  std::lock_guard<std::mutex> lk(e->mu);
  if (slot >= e->n_slots || !set_dev(e) || hipStreamSynchronize(e->stream) != hipSuccess) return -1;
  if (hipMemcpy(out, (const atls::KeySched*)e->ks.p + slot, sizeof(atls::KeySched), hipMemcpyDeviceToHost) != hipSuccess)
    return -1;
  return (int)sizeof(atls::KeySched);
}

// Debug: copy the last batch plan (PlanHdr words, then the first n_idx record indices) to host.
extern "C" int atls_debug_plan(atls_engine* e, uint32_t* out, uint32_t n_idx) {
  if (!e) return -1;
  std::lock_guard<std::mutex> lk(e->mu);  // before reading last_par / the plan set
  const auto& q = e->ps[e->last_par];
  if (!q.plan.p) return -1;
  if (!set_dev(e) || join_pending(e) || hipStreamSynchronize(e->stream) != hipSuccess) return -1;
  if (hipMemcpy(out, q.plan.p, sizeof(atls::PlanHdr), hipMemcpyDeviceToHost) != hipSuccess) return -1;
  if (n_idx && hipMemcpy(out + sizeof(atls::PlanHdr) / 4, q.idx.p, 4 * (size_t)n_idx, hipMemcpyDeviceToHost) != hipSuccess)
    return -1;
  return 0;
}
