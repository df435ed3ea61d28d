// Multi-GPU batches in one process (include/atls.h atls_multi_*), SURVEY.md §8(b)/(e).
//
// Records are independent: a record's nonce comes from (static_iv, seq) (net/key_schedule.rs:51-64)
// and nothing carries over between records, so a batch splits into contiguous record ranges, one
// per device, balanced by cumulative bytes (atls_partition: each record costs the bytes it reads
// and writes, in + out + 16-byte tag, so a mixed-length batch like C5 splits by work, not by count).
// Each device runs its own engine (engine.cpp) over its range with rebased descriptors.
//
// Device-resident batches live on the root device (devices[0]). The other ranges travel over
// RCCL (grouped ncclSend / ncclRecv, xGMI peer links) when every device of the engine is distinct:
// one group scatters the input ranges (and on open the tags), every device seals / opens its
// range, and one group gathers output ranges, tags and open results back into the caller's
// buffers. A range's output bytes travel both ways (out to the device first), so bytes between
// records come back as the caller had them, as with one engine. The root's own range is processed in place, overlapped with the transfers. RCCL is
// loaded on first use (dlopen, the same librccl.so.1 PyTorch's process may already hold); a
// device list with repeats (several ranges on one GPU: tests on a one-GPU box) uses HIP
// device-to-device copies instead. Host-memory batches need no exchange: each device stages its
// own range over its own PCIe link, one host thread per device.
//
// Descriptors are validated before anything is queued, and a failure after that point waits for
// the queued transfers and kernels (drain) before returning, so the caller's buffers are never
// touched after the call returns. ATLS_MULTI_RCCL_SELF=1 with one device repeated runs the RCCL
// branch as rank-0-to-itself send / recv on a one-rank communicator (the one-GPU test of the
// RCCL binding, tests/test_gpu_dist.py).
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <rccl/rccl.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <thread>
#include <type_traits>
#include <vector>

#include "../../include/atls.h"
#include "engine_internal.h"

namespace {

// ---- the few RCCL entry points we use, resolved at run time ------------------------------
// rccl.h gives the types and the prototypes; the library itself is dlopen'ed (the librccl.so.1
// PyTorch may already hold), and every resolved pointer has exactly the header's type.
struct Rccl {
  decltype(&ncclCommInitAll) comm_init_all = nullptr;
  decltype(&ncclCommDestroy) comm_destroy = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  decltype(&ncclSend) send = nullptr;
  decltype(&ncclRecv) recv = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
  decltype(&ncclGetVersion) get_version = nullptr;
  int version = 0;          // NCCL_VERSION_CODE of the library actually loaded (e.g. 22606 for 2.26.6)
  const char* path = "";    // its file (dladdr)
  bool ok = false;
};
static_assert(std::is_same<decltype(Rccl::send), ncclResult_t (*)(const void*, size_t, ncclDataType_t, int, ncclComm_t,
                                                                  hipStream_t)>::value,
              "ncclSend prototype");
static_assert(std::is_same<decltype(Rccl::recv), ncclResult_t (*)(void*, size_t, ncclDataType_t, int, ncclComm_t,
                                                                  hipStream_t)>::value,
              "ncclRecv prototype");
static_assert(std::is_same<decltype(Rccl::comm_init_all), ncclResult_t (*)(ncclComm_t*, int, const int*)>::value,
              "ncclCommInitAll prototype");
static_assert(ncclSuccess == 0 && ncclUint8 == 1, "rccl.h enums");

template <typename F>
void resolve(void* h, const char* name, F& f) {
  f = reinterpret_cast<F>(dlsym(h, name));
}

const Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
    if (!h) return;
    resolve(h, "ncclCommInitAll", r.comm_init_all);
    resolve(h, "ncclCommDestroy", r.comm_destroy);
    resolve(h, "ncclGroupStart", r.group_start);
    resolve(h, "ncclGroupEnd", r.group_end);
    resolve(h, "ncclSend", r.send);
    resolve(h, "ncclRecv", r.recv);
    resolve(h, "ncclGetErrorString", r.error_string);
    resolve(h, "ncclGetVersion", r.get_version);
    r.ok = r.comm_init_all && r.comm_destroy && r.group_start && r.group_end && r.send && r.recv && r.get_version;
    if (r.ok && r.get_version(&r.version) != ncclSuccess) r.version = 0;
    Dl_info info;
    if (r.ok && dladdr(reinterpret_cast<void*>(r.send), &info) && info.dli_fname) r.path = info.dli_fname;
  });
  return r;
}

struct DevMem {
  int device = 0;
  void* p = nullptr;
  size_t cap = 0;
  bool reserve(size_t n) {
    if (n <= cap) return true;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    if (hipSetDevice(device) != hipSuccess || hipMalloc(&p, std::max<size_t>(n, 256)) != hipSuccess) return false;
    cap = std::max<size_t>(n, 256);
    return true;
  }
  ~DevMem() {
    if (p) {
      (void)hipSetDevice(device);
      (void)hipFree(p);
    }
  }
};

struct Part {
  int device = 0;
  atls_engine* eng = nullptr;
  hipStream_t comm = nullptr;                  // transfers of this device (RCCL or copies)
  hipEvent_t ev_in = nullptr, ev_done = nullptr;
  DevMem in, out, aux, tags, res;              // staging of a non-root range
  std::vector<atls_rec> recs;                  // rebased descriptors (alive until the batch ends)
};

size_t in_len(const atls_rec& r, bool open) { return (r.mode == ATLS_MODE_WIRE && open) ? (size_t)r.len + 21 : r.len; }
size_t out_len(const atls_rec& r, bool open) {
  if (open || r.mode == ATLS_MODE_RAW) return r.len;
  return r.mode == ATLS_MODE_WIRE ? (size_t)r.len + 22 : (size_t)r.len + 1;
}

}  // namespace

struct atls_multi {
  std::vector<Part> parts;
  std::vector<ncclComm_t> comms;  // one per device when all devices are distinct (one in self mode)
  bool use_rccl = false;
  // ATLS_MULTI_RCCL_SELF=1 with one device repeated: a one-rank communicator, and every part's
  // transfers are RCCL send / recv of rank 0 to itself on the root's transfer stream. The batch
  // then goes through exactly the RCCL branch of run_device on a one-GPU box (tests).
  bool rccl_self = false;
  size_t xfer_chunk = ~size_t(0);  // largest RCCL message (multi_xfer_chunk() at creation)
  int rccl_version = 0;            // of the loaded library (0 without RCCL)
  std::mutex mu;
};

namespace {

// Largest RCCL point-to-point message: ATLS_MULTI_CHUNK_MB when the multi engine is created (0 = none),
// else 1024 MiB. RCCL 2.26.6 (the library PyTorch ships, which this process resolves librccl.so.1 to
// once torch is loaded) returns wrong bytes past 2^30 of a self send / recv of 2 GiB
// (profiles/r04/multi_diag.log); tools/rccl_p2p_probe brackets the threshold per library
// (profiles/r05/rccl_p2p_probe_*.log). 1 GiB pieces are what every tested message size
// below the threshold is, for every version seen.
constexpr size_t kRcclSafePiece = size_t(1) << 30;
size_t multi_xfer_chunk(int version) {
  (void)version;  // one cap for every library version measured so far
  const char* e = std::getenv("ATLS_MULTI_CHUNK_MB");
  if (!e) return kRcclSafePiece;
  const long mb = std::atol(e);
  return mb > 0 ? (size_t)mb << 20 : ~size_t(0);
}

// Once per process: which RCCL the multi engines use and the message cap.
void log_rccl(const Rccl& R, size_t cap) {
  static std::once_flag once;
  std::call_once(once, [&] {
    std::fprintf(stderr, "anothertls_amd: RCCL %d.%d.%d (%s), point-to-point messages capped at %zu MiB\n",
                 R.version / 10000, (R.version / 100) % 100, R.version % 100, R.path,
                 cap == ~size_t(0) ? (size_t)0 : cap >> 20);
  });
}

// Wait for everything queued for this batch (engine streams, transfer streams), and clear the
// part engines' sticky error words, so an early return never leaves work that reads or writes
// the caller's buffers, and no refusal of this batch is reported by a later call.
void drain(atls_multi* m) {
  for (Part& q : m->parts) {
    (void)atls_engine_sync(q.eng);
    (void)hipSetDevice(q.device);
    (void)hipStreamSynchronize(q.comm);
  }
}

// Device-resident batch on the root device. first[p] .. first[p+1] = records of part p.
int run_device(atls_multi* m, bool open, const atls_rec* recs, const uint32_t* first, const uint8_t* in,
               const uint8_t* aux, size_t aux_end, uint8_t* out, uint8_t* tags_out, const uint8_t* tags_in,
               atls_open_result* res) {
  const size_t P = m->parts.size();
  Part& root = m->parts[0];
  const uint32_t dflags = ATLS_FLAG_DEVICE_PTRS | ATLS_FLAG_NO_SYNC;
  struct Range {
    size_t in_lo = 0, in_hi = 0, out_lo = 0, out_hi = 0;
    uint32_t a = 0, b = 0;
  };
  std::vector<Range> rg(P);
  for (size_t p = 0; p < P; p++) {
    Range& r = rg[p];
    r.a = first[p];
    r.b = first[p + 1];
    if (r.a == r.b) continue;
    r.in_lo = recs[r.a].in_off;
    r.out_lo = recs[r.a].out_off;
    r.in_hi = recs[r.b - 1].in_off + in_len(recs[r.b - 1], open);
    r.out_hi = recs[r.b - 1].out_off + out_len(recs[r.b - 1], open);
  }
  // Where part p's side of a transfer runs: its own device, comm rank and stream over RCCL between
  // distinct devices; the root's otherwise (device copies, or RCCL self mode).
  const bool own_side = m->use_rccl && !m->rccl_self;
  auto side_stream = [&](size_t p) { return own_side ? m->parts[p].comm : root.comm; };
  auto side_device = [&](size_t p) { return own_side ? m->parts[p].device : root.device; };
  // Root work is ordered after the caller's prior work on the root device (its engine stream).
  if (hipSetDevice(root.device) != hipSuccess || hipEventRecord(root.ev_in, (hipStream_t)atls_engine_stream(root.eng)) != hipSuccess ||
      hipStreamWaitEvent(root.comm, root.ev_in, 0) != hipSuccess)
    return ATLS_INTERNAL_ERROR;
  // ---- staging buffers and rebased descriptors of the non-root parts ----
  for (size_t p = 1; p < P; p++) {
    Part& q = m->parts[p];
    const Range& r = rg[p];
    const uint32_t cnt = r.b - r.a;
    if (!cnt) continue;
    q.recs.assign(recs + r.a, recs + r.b);
    for (atls_rec& d : q.recs) {
      d.in_off -= r.in_lo;
      d.out_off -= r.out_lo;
    }
    if (!q.in.reserve(r.in_hi - r.in_lo + 16) || !q.out.reserve(r.out_hi - r.out_lo + 16) || !q.aux.reserve(aux_end + 16) ||
        !q.tags.reserve(16 * (size_t)cnt) || !q.res.reserve(sizeof(atls_open_result) * (size_t)cnt))
      return ATLS_INTERNAL_ERROR;  // nothing queued yet but the root's event wait
  }
  // ---- scatter: input ranges, aux, (open) tags; gather: output ranges, tags, results ----
  auto xfer = [&](bool to_parts) -> int {
    if (m->use_rccl) {
      const Rccl& R = rccl();
      if (R.group_start() != ncclSuccess) return ATLS_INTERNAL_ERROR;
      ncclResult_t bad = ncclSuccess;
      auto chk = [&](ncclResult_t r) {
        if (r != ncclSuccess && bad == ncclSuccess) bad = r;
      };
      // Every send / recv pair in pieces of at most multi_xfer_chunk() bytes, matched in order on both
      // sides: one C4 range is 2 GiB each way (131,072 x 16 KiB), and a single RCCL point-to-point
      // message of 2^31 bytes or more came back wrong on the one-GPU self exchange
      // (tests/test_gpu_c4_full.py, round 4).
      const size_t piece = m->xfer_chunk;
      auto send = [&](const void* p, size_t bytes, int peer, ncclComm_t c, hipStream_t st) {
        for (size_t o = 0; o < bytes; o += piece)
          chk(R.send((const uint8_t*)p + o, std::min(piece, bytes - o), ncclUint8, peer, c, st));
      };
      auto recv = [&](void* p, size_t bytes, int peer, ncclComm_t c, hipStream_t st) {
        for (size_t o = 0; o < bytes; o += piece)
          chk(R.recv((uint8_t*)p + o, std::min(piece, bytes - o), ncclUint8, peer, c, st));
      };
      for (size_t p = 1; p < P; p++) {
        Part& q = m->parts[p];
        const Range& r = rg[p];
        const uint32_t cnt = r.b - r.a;
        if (!cnt) continue;
        // root = rank 0; part p = rank p, or rank 0 itself in self mode
        const int peer = m->rccl_self ? 0 : (int)p;
        ncclComm_t rc = m->comms[0], qc = m->comms[m->rccl_self ? 0 : p];
        hipStream_t qs = side_stream(p);
        if (to_parts) {
          send(in + r.in_lo, r.in_hi - r.in_lo, peer, rc, root.comm);
          recv(q.in.p, r.in_hi - r.in_lo, 0, qc, qs);
          send(out + r.out_lo, r.out_hi - r.out_lo, peer, rc, root.comm);  // bytes between records
          recv(q.out.p, r.out_hi - r.out_lo, 0, qc, qs);
          if (aux_end) {
            send(aux, aux_end, peer, rc, root.comm);
            recv(q.aux.p, aux_end, 0, qc, qs);
          }
          if (open && tags_in) {
            send(tags_in + 16 * (size_t)r.a, 16 * (size_t)cnt, peer, rc, root.comm);
            recv(q.tags.p, 16 * (size_t)cnt, 0, qc, qs);
          }
        } else {
          send(q.out.p, r.out_hi - r.out_lo, 0, qc, qs);
          recv(out + r.out_lo, r.out_hi - r.out_lo, peer, rc, root.comm);
          if (!open && tags_out) {
            send(q.tags.p, 16 * (size_t)cnt, 0, qc, qs);
            recv(tags_out + 16 * (size_t)r.a, 16 * (size_t)cnt, peer, rc, root.comm);
          }
          if (open) {
            send(q.res.p, sizeof(atls_open_result) * (size_t)cnt, 0, qc, qs);
            recv(res + r.a, sizeof(atls_open_result) * (size_t)cnt, peer, rc, root.comm);
          }
        }
      }
      chk(R.group_end());  // always closes the group, also after a failed call inside it
      return bad == ncclSuccess ? ATLS_OK : ATLS_INTERNAL_ERROR;
    }
    // device-to-device copies (repeated devices): issued on the root's transfer stream
    if (hipSetDevice(root.device) != hipSuccess) return ATLS_INTERNAL_ERROR;
    for (size_t p = 1; p < P; p++) {
      Part& q = m->parts[p];
      const Range& r = rg[p];
      const uint32_t cnt = r.b - r.a;
      if (!cnt) continue;
      const hipMemcpyKind k = hipMemcpyDeviceToDevice;
      bool ok = true;
      if (to_parts) {
        ok = hipMemcpyAsync(q.in.p, in + r.in_lo, r.in_hi - r.in_lo, k, root.comm) == hipSuccess &&
             hipMemcpyAsync(q.out.p, out + r.out_lo, r.out_hi - r.out_lo, k, root.comm) == hipSuccess;
        if (ok && aux_end) ok = hipMemcpyAsync(q.aux.p, aux, aux_end, k, root.comm) == hipSuccess;
        if (ok && open && tags_in)
          ok = hipMemcpyAsync(q.tags.p, tags_in + 16 * (size_t)r.a, 16 * (size_t)cnt, k, root.comm) == hipSuccess;
      } else {
        ok = hipMemcpyAsync(out + r.out_lo, q.out.p, r.out_hi - r.out_lo, k, root.comm) == hipSuccess;
        if (ok && !open && tags_out)
          ok = hipMemcpyAsync(tags_out + 16 * (size_t)r.a, q.tags.p, 16 * (size_t)cnt, k, root.comm) == hipSuccess;
        if (ok && open)
          ok = hipMemcpyAsync(res + r.a, q.res.p, sizeof(atls_open_result) * (size_t)cnt, k, root.comm) == hipSuccess;
      }
      if (!ok) return ATLS_INTERNAL_ERROR;
    }
    return ATLS_OK;
  };
  // From here on work is queued: every failure drains it before returning.
  auto fail = [&](int rc) {
    drain(m);
    return rc;
  };
  int rc = xfer(true);
  if (rc) return fail(rc);
  // inputs in place -> every part's engine stream may start
  for (size_t p = 1; p < P; p++) {
    Part& q = m->parts[p];
    if (rg[p].a == rg[p].b) continue;
    if (hipSetDevice(side_device(p)) != hipSuccess || hipEventRecord(q.ev_in, side_stream(p)) != hipSuccess ||
        hipSetDevice(q.device) != hipSuccess || hipStreamWaitEvent((hipStream_t)atls_engine_stream(q.eng), q.ev_in, 0) != hipSuccess)
      return fail(ATLS_INTERNAL_ERROR);
  }
  // ---- every part seals / opens its range (the root in place, beside the transfers) ----
  for (size_t p = 0; p < P; p++) {
    Part& q = m->parts[p];
    const Range& r = rg[p];
    const uint32_t cnt = r.b - r.a;
    if (!cnt) continue;
    if (p == 0) {
      rc = open ? atls_open_batch(q.eng, recs + r.a, cnt, in, aux, tags_in ? tags_in + 16 * (size_t)r.a : nullptr, out,
                                  res + r.a, dflags)
                : atls_seal_batch(q.eng, recs + r.a, cnt, in, aux, out, tags_out ? tags_out + 16 * (size_t)r.a : nullptr,
                                  dflags);
    } else {
      const bool want_tags = open ? tags_in != nullptr : tags_out != nullptr;
      rc = open ? atls_open_batch(q.eng, q.recs.data(), cnt, q.in.p, q.aux.p, want_tags ? (const uint8_t*)q.tags.p : nullptr,
                                  q.out.p, (atls_open_result*)q.res.p, dflags)
                : atls_seal_batch(q.eng, q.recs.data(), cnt, q.in.p, q.aux.p, q.out.p,
                                  want_tags ? (uint8_t*)q.tags.p : nullptr, dflags);
    }
    if (rc) return fail(rc);
    if (p && (hipSetDevice(q.device) != hipSuccess || hipEventRecord(q.ev_done, (hipStream_t)atls_engine_stream(q.eng)) != hipSuccess))
      return fail(ATLS_INTERNAL_ERROR);
  }
  // ---- gather ----
  for (size_t p = 1; p < P; p++) {
    Part& q = m->parts[p];
    if (rg[p].a == rg[p].b) continue;
    if (hipSetDevice(side_device(p)) != hipSuccess || hipStreamWaitEvent(side_stream(p), q.ev_done, 0) != hipSuccess)
      return fail(ATLS_INTERNAL_ERROR);
  }
  rc = xfer(false);
  if (rc) return fail(rc);
  // every part's status (sticky error words), then the transfer streams
  int status = ATLS_OK;
  for (size_t p = 0; p < P; p++) {
    if (rg[p].a == rg[p].b) continue;
    const int s = atls_engine_sync(m->parts[p].eng);
    if (s && !status) status = s;
  }
  for (size_t p = 0; p < P; p++) {
    if (hipSetDevice(m->parts[p].device) != hipSuccess || hipStreamSynchronize(m->parts[p].comm) != hipSuccess)
      return fail(ATLS_INTERNAL_ERROR);
  }
  return status;
}

// Host-memory batch: every part stages its own range through its engine (own PCIe link).
int run_host(atls_multi* m, bool open, const atls_rec* recs, const uint32_t* first, const uint8_t* in, const uint8_t* aux,
             uint8_t* out, uint8_t* tags_out, const uint8_t* tags_in, atls_open_result* res) {
  const size_t P = m->parts.size();
  std::vector<int> rcs(P, ATLS_OK);
  auto work = [&](size_t p) {
    Part& q = m->parts[p];
    const uint32_t a = first[p], b = first[p + 1];
    if (a == b) return;
    const size_t in_lo = recs[a].in_off, out_lo = recs[a].out_off;
    q.recs.assign(recs + a, recs + b);
    for (atls_rec& d : q.recs) {
      d.in_off -= in_lo;
      d.out_off -= out_lo;
    }
    rcs[p] = open ? atls_open_batch(q.eng, q.recs.data(), b - a, in + in_lo, aux, tags_in ? tags_in + 16 * (size_t)a : nullptr,
                                    out + out_lo, res + a, 0)
                  : atls_seal_batch(q.eng, q.recs.data(), b - a, in + in_lo, aux, out + out_lo,
                                    tags_out ? tags_out + 16 * (size_t)a : nullptr, 0);
  };
  std::vector<std::thread> th;
  for (size_t p = 1; p < P; p++) th.emplace_back(work, p);
  work(0);
  for (auto& t : th) t.join();
  for (int r : rcs)
    if (r) return r;
  return ATLS_OK;
}

int run(atls_multi* m, bool open, const atls_rec* recs, uint32_t n, const void* in, const void* aux, void* out,
        uint8_t* tags_out, const uint8_t* tags_in, atls_open_result* res, uint32_t flags) {
  if (!m) return ATLS_INTERNAL_ERROR;
  if (n == 0) return ATLS_OK;
  if (!recs || (flags & (ATLS_FLAG_DEVICE_RECS | ATLS_FLAG_NO_SYNC))) return ATLS_ILLEGAL_PARAMETER;
  // contiguous ranges must not interleave: offsets increase with the record index
  size_t aux_end = 0;
  for (uint32_t i = 0; i < n; i++) {
    if (i && (recs[i].in_off < recs[i - 1].in_off + in_len(recs[i - 1], open) ||
              recs[i].out_off < recs[i - 1].out_off + out_len(recs[i - 1], open)))
      return ATLS_ILLEGAL_PARAMETER;
    if (recs[i].mode == ATLS_MODE_RAW) aux_end = std::max(aux_end, (size_t)recs[i].aux_off + recs[i].iv_len + recs[i].aad_len);
  }
  // refused descriptors are refused before anything is queued (as run_batch does for one engine)
  const uint32_t n_slots = atls::engine_slots(m->parts[0].eng);  // every part holds the same key table
  const bool no_tags = open ? !tags_in : !tags_out;
  for (uint32_t i = 0; i < n; i++)
    if (recs[i].key_slot >= n_slots || recs[i].mode > ATLS_MODE_WIRE || (no_tags && recs[i].mode != ATLS_MODE_WIRE))
      return ATLS_ILLEGAL_PARAMETER;
  std::lock_guard<std::mutex> lk(m->mu);
  const uint32_t P = (uint32_t)m->parts.size();
  std::vector<uint32_t> first(P + 1);
  atls_partition(recs, n, open ? 1 : 0, P, first.data());
  if (flags & ATLS_FLAG_DEVICE_PTRS)
    return run_device(m, open, recs, first.data(), (const uint8_t*)in, (const uint8_t*)aux, aux_end, (uint8_t*)out, tags_out,
                      tags_in, res);
  return run_host(m, open, recs, first.data(), (const uint8_t*)in, (const uint8_t*)aux, (uint8_t*)out, tags_out, tags_in, res);
}

}  // namespace

extern "C" {

void atls_partition(const atls_rec* recs, uint32_t n, int open, uint32_t parts, uint32_t* first) {
  if (!parts) return;
  uint64_t total = 0;
  for (uint32_t i = 0; i < n; i++) total += in_len(recs[i], open != 0) + out_len(recs[i], open != 0) + 16;
  first[0] = 0;
  uint64_t cum = 0;
  uint32_t i = 0;
  for (uint32_t p = 1; p < parts; p++) {
    // first record whose cumulative cost before it reaches p/parts of the total
    const uint64_t target = (total * p + parts / 2) / parts;
    while (i < n && cum + (in_len(recs[i], open != 0) + out_len(recs[i], open != 0) + 16) / 2 < target) {
      cum += in_len(recs[i], open != 0) + out_len(recs[i], open != 0) + 16;
      i++;
    }
    first[p] = i;
  }
  first[parts] = n;
}

atls_multi* atls_multi_create(const int* devices, int n_devices) {
  if (!devices || n_devices < 1) return nullptr;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess) return nullptr;
  for (int i = 0; i < n_devices; i++)
    if (devices[i] < 0 || devices[i] >= count) return nullptr;
  atls_multi* m = new (std::nothrow) atls_multi();
  if (!m) return nullptr;
  m->parts.resize((size_t)n_devices);
  bool distinct = true;
  for (int i = 0; i < n_devices; i++) {
    Part& q = m->parts[(size_t)i];
    q.device = devices[i];
    q.in.device = q.out.device = q.aux.device = q.tags.device = q.res.device = devices[i];
    for (int j = 0; j < i; j++) distinct = distinct && devices[j] != devices[i];
    q.eng = atls_engine_create(devices[i]);
    if (!q.eng || hipSetDevice(devices[i]) != hipSuccess || hipStreamCreateWithFlags(&q.comm, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&q.ev_in, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&q.ev_done, hipEventDisableTiming) != hipSuccess) {
      atls_multi_destroy(m);
      return nullptr;
    }
  }
  const char* self_env = std::getenv("ATLS_MULTI_RCCL_SELF");
  const bool self = !distinct && self_env && std::atoi(self_env) != 0 &&
                    std::all_of(devices, devices + n_devices, [&](int d) { return d == devices[0]; });
  if ((distinct || self) && n_devices > 1) {
    const Rccl& R = rccl();
    const int ranks = self ? 1 : n_devices;
    m->comms.assign((size_t)ranks, nullptr);
    if (!R.ok || R.comm_init_all(m->comms.data(), ranks, devices) != ncclSuccess) {
      m->comms.clear();
      atls_multi_destroy(m);
      return nullptr;
    }
    m->use_rccl = true;
    m->rccl_self = self;
    m->rccl_version = R.version;
    m->xfer_chunk = multi_xfer_chunk(R.version);
    log_rccl(R, m->xfer_chunk);
  }
  return m;
}

void atls_multi_destroy(atls_multi* m) {
  if (!m) return;
  if (!m->comms.empty() && rccl().ok)
    for (ncclComm_t c : m->comms)
      if (c) rccl().comm_destroy(c);
  for (Part& q : m->parts) {
    (void)hipSetDevice(q.device);
    if (q.comm) (void)hipStreamSynchronize(q.comm);
    if (q.ev_in) (void)hipEventDestroy(q.ev_in);
    if (q.ev_done) (void)hipEventDestroy(q.ev_done);
    if (q.comm) (void)hipStreamDestroy(q.comm);
    if (q.eng) atls_engine_destroy(q.eng);
  }
  delete m;
}

int atls_multi_devices(const atls_multi* m) { return m ? (int)m->parts.size() : 0; }
int atls_multi_uses_rccl(const atls_multi* m) { return m && m->use_rccl ? 1 : 0; }
int atls_multi_rccl_version(const atls_multi* m) { return m && m->use_rccl ? m->rccl_version : 0; }
size_t atls_multi_max_message(const atls_multi* m) { return m && m->use_rccl ? m->xfer_chunk : 0; }

int atls_multi_set_keys(atls_multi* m, const atls_key* keys, uint32_t n) {
  if (!m) return ATLS_INTERNAL_ERROR;
  std::lock_guard<std::mutex> lk(m->mu);
  int status = ATLS_OK;
  for (Part& q : m->parts) {  // each device builds its own key schedules (no exchange needed)
    const int rc = atls_set_keys(q.eng, keys, n);
    if (rc && !status) status = rc;
  }
  return status;
}

int atls_multi_seal_batch(atls_multi* m, const atls_rec* recs, uint32_t n, const void* in, const void* aux, void* out,
                          uint8_t* tags, uint32_t flags) {
  atls::ResidentHold hold;  // RCCL's kernels and the engines' batches must not queue behind a resident server
  return run(m, false, recs, n, in, aux, out, tags, nullptr, nullptr, flags);
}

int atls_multi_open_batch(atls_multi* m, const atls_rec* recs, uint32_t n, const void* in, const void* aux,
                          const uint8_t* tags, void* out, atls_open_result* results, uint32_t flags) {
  atls::ResidentHold hold;
  return run(m, true, recs, n, in, aux, out, nullptr, tags, results, flags);
}

}  // extern "C"
