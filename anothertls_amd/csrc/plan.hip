// Batch plan: three small launches before the record kernels.
//
//  1. plan_count: classifies every record (validation of net/record.rs-style descriptors against
//     the key table, crypto/ciphersuite.rs:78-87 get_cipher: AES-GCM for 0x1301/0x1302 with the
//     AES size from the key, ChaCha20-Poly1305 for 0x1303, anything else InsufficientSecurity)
//     into a work list -- AES-GCM with 10 / 12 / 14 rounds, ChaCha20-Poly1305 -- and a length
//     class; rejected records get their status here (err flag; open results for open batches).
//     Each workgroup counts its chunk of the batch in an LDS histogram.
//  2. plan_scan: one workgroup turns the per-workgroup histograms into offsets, lists in order,
//     classes longest record first.
//  3. plan_scatter: each workgroup writes its records' indices at its offsets (LDS cursors).
//
// The record kernels (gcm.hip, chacha.hip) take their list's positions round-robin (WorkList,
// plan.h), so every worker gets a similar mix of lengths (LPT-like balance for the
// variable-length batches of BASELINE config C5).
#include "plan.h"

namespace atls {

// Work-list key of record i, or kPlanReject (status in *st).
__device__ __forceinline__ uint32_t plan_key(const atls_rec* recs, uint32_t i, const KeySched* ks, uint32_t n_slots,
                                             uint8_t* st, bool open) {
  const atls_rec d = recs[i];
  *st = ATLS_ILLEGAL_PARAMETER;
  if (d.key_slot >= n_slots || d.mode > ATLS_MODE_WIRE) return kPlanReject;
  const KeySched* k = ks + d.key_slot;
  const uint32_t suite = k->suite, valid = k->valid, nr = k->nr;
  uint32_t list;
  if (suite == (uint32_t)kSuiteChacha) {
    if (!valid || (d.mode == ATLS_MODE_RAW && d.iv_len != 12)) return kPlanReject;  // cipher.rs:19
    if (!chacha_len_ok(d, open)) return kPlanReject;                                 // cipher.rs:94
    list = kListChacha;
  } else if (suite == (uint32_t)kSuiteAes128 || suite == (uint32_t)kSuiteAes256) {
    if (!valid) return kPlanReject;
    list = nr == 10 ? kListGcm10 : nr == 12 ? kListGcm12 : kListGcm14;
  } else {
    *st = ATLS_INSUFFICIENT_SECURITY;  // ciphersuite.rs:84-86
    return kPlanReject;
  }
  const uint32_t cls = min(d.len >> 10, (uint32_t)kPlanClasses - 1u);
  return list * kPlanClasses + (kPlanClasses - 1u - cls);  // longest class first within a list
}

// The batch is cut into G contiguous chunks, one per workgroup. Counting and scattering use LDS
// atomics only: per-workgroup class histograms go to global memory (key-major, [k][G]) and one
// scan turns them into each workgroup's start offset per class. (Wave-aggregated global atomics
// on the 64 class counters serialised at L2: 55 us per pass for 32 Ki records.)
__device__ __forceinline__ void plan_chunk(uint32_t n, uint32_t& lo, uint32_t& hi) {
  const uint32_t chunk = (n + gridDim.x - 1u) / gridDim.x;
  lo = min(n, blockIdx.x * chunk);
  hi = min(n, lo + chunk);
}

__global__ __launch_bounds__(256) void plan_count(const atls_rec* recs, uint32_t n, const KeySched* ks,
                                                  uint32_t n_slots, uint32_t open, atls_open_result* res,
                                                  uint32_t* err, uint8_t* keys, uint32_t* wgcount) {
  __shared__ uint32_t hist[kPlanKeys];
  for (uint32_t t = threadIdx.x; t < kPlanKeys; t += blockDim.x) hist[t] = 0;
  __syncthreads();
  uint32_t lo, hi;
  plan_chunk(n, lo, hi);
  for (uint32_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
    uint8_t st = 0;
    const uint32_t key = plan_key(recs, i, ks, n_slots, &st, open != 0);
    keys[i] = (uint8_t)key;
    if (key == kPlanReject) {
      atomicOr(err, 1u);
      if (open) {
        atls_open_result rr = {0, st, 0, {0, 0}};
        res[i] = rr;
      }
    } else {
      atomicAdd(&hist[key], 1u);
    }
  }
  __syncthreads();
  for (uint32_t t = threadIdx.x; t < kPlanKeys; t += blockDim.x) wgcount[t * gridDim.x + blockIdx.x] = hist[t];
}

// One workgroup: exclusive prefix over the G x 64 histogram entries in key-major order, i.e. list
// by list, longest class first, workgroup by workgroup. wgoff[k][b] = start of workgroup b's
// records of key k in idx; P->off[l] = start of list l.
__global__ __launch_bounds__(1024) void plan_scan(const uint32_t* wgcount, uint32_t G, uint32_t* wgoff, PlanHdr* P) {
  __shared__ uint32_t part[1024];
  const uint32_t E = kPlanKeys * G, t = threadIdx.x;
  const uint32_t per = (E + blockDim.x - 1u) / blockDim.x, lo = min(E, t * per), hi = min(E, lo + per);
  // 8 independent loads per pass: one L2 round trip per 8 entries (a plain loop waited for each load,
  // 8 round trips for the 8,192 entries of a 32 Ki-record batch)
  uint32_t sum = 0;
  for (uint32_t e = lo; e < hi; e += 8) {
    uint32_t v[8];
#pragma unroll
    for (int k = 0; k < 8; k++) v[k] = (e + k < hi) ? wgcount[e + k] : 0u;
#pragma unroll
    for (int k = 0; k < 8; k++) sum += v[k];
  }
  part[t] = sum;
  __syncthreads();
  for (uint32_t d = 1; d < blockDim.x; d <<= 1) {  // Hillis-Steele inclusive scan of the partial sums
    const uint32_t v = t >= d ? part[t - d] : 0u;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  uint32_t run = part[t] - sum;
  for (uint32_t e = lo; e < hi; e += 8) {
    uint32_t v[8];
#pragma unroll
    for (int k = 0; k < 8; k++) v[k] = (e + k < hi) ? wgcount[e + k] : 0u;
#pragma unroll
    for (int k = 0; k < 8; k++) {
      if (e + k < hi) {
        if ((e + k) % (G * kPlanClasses) == 0) P->off[(e + k) / (G * kPlanClasses)] = run;
        wgoff[e + k] = run;
        run += v[k];
      }
    }
  }
  if (t == blockDim.x - 1u) P->off[kPlanLists] = part[t];
}

__global__ __launch_bounds__(256) void plan_scatter(uint32_t n, const uint8_t* keys, const uint32_t* wgoff, uint32_t* idx) {
  __shared__ uint32_t cur[kPlanKeys];
  for (uint32_t t = threadIdx.x; t < kPlanKeys; t += blockDim.x) cur[t] = wgoff[t * gridDim.x + blockIdx.x];
  __syncthreads();
  uint32_t lo, hi;
  plan_chunk(n, lo, hi);
  for (uint32_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
    const uint32_t key = keys[i];
    if (key != kPlanReject) idx[atomicAdd(&cur[key], 1u)] = i;
  }
}

// ---- key groups (direct AES-GCM batches) ----------------------------------------------------
// group_count -> group_scan -> group_scatter: a counting sort of the records by key slot (bucket
// n_slots collects refused slots). cnt is all zero between batches: group_scan clears it.
__global__ __launch_bounds__(256) void group_count(const atls_rec* recs, uint32_t n, uint32_t n_slots, uint32_t* cnt) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint32_t k = recs[i].key_slot;
    atomicAdd(&cnt[k < n_slots ? k : n_slots], 1u);
  }
}

__device__ __forceinline__ uint32_t pad_group(uint32_t c) { return (c + kGroupPad - 1u) / kGroupPad * kGroupPad; }

// One workgroup: exclusive prefix of the padded bucket sizes -> cursors; the padding positions
// get kNoRecord; total[0] = padded length of the list, total[1] = 0 (the record kernel's work
// counter).
__global__ __launch_bounds__(1024) void group_scan(uint32_t* cnt, uint32_t nb, uint32_t* cur, uint32_t* gidx,
                                                   uint32_t* total) {
  __shared__ uint32_t part[1024];
  const uint32_t t = threadIdx.x;
  const uint32_t per = (nb + blockDim.x - 1u) / blockDim.x, lo = min(nb, t * per), hi = min(nb, lo + per);
  uint32_t sum = 0;
  for (uint32_t b = lo; b < hi; b++) sum += pad_group(cnt[b]);
  part[t] = sum;
  __syncthreads();
  for (uint32_t d = 1; d < blockDim.x; d <<= 1) {
    const uint32_t v = t >= d ? part[t - d] : 0u;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  uint32_t run = part[t] - sum;
  for (uint32_t b = lo; b < hi; b++) {
    const uint32_t c = cnt[b], pc = pad_group(c);
    cur[b] = run;
    for (uint32_t j = c; j < pc; j++) gidx[run + j] = kNoRecord;
    cnt[b] = 0u;
    run += pc;
  }
  if (t == blockDim.x - 1u) {
    total[0] = part[t];
    total[1] = 0u;
  }
}

__global__ __launch_bounds__(256) void group_scatter(const atls_rec* recs, uint32_t n, uint32_t n_slots, uint32_t* cur,
                                                     uint32_t* gidx) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint32_t k = recs[i].key_slot;
    gidx[atomicAdd(&cur[k < n_slots ? k : n_slots], 1u)] = i;
  }
}

}  // namespace atls

// Key groups of a direct batch: cnt / cur hold n_slots + 1 words (cnt zero on entry and on
// return), gidx n + (kGroupPad - 1) * (n_slots + 1) words, total two words.
extern "C" int atls_launch_group(const atls_rec* recs, uint32_t n, uint32_t n_slots, uint32_t* cnt, uint32_t* cur,
                                 uint32_t* gidx, uint32_t* total, int cus, hipStream_t s) {
  if (n_slots > atls::kGroupMaxSlots) return ATLS_INTERNAL_ERROR;
  const uint32_t want = (n + 255u) / 256u, cap = (uint32_t)(cus > 0 ? 2 * cus : 512);
  const uint32_t G = want ? (want < cap ? want : cap) : 1u;
  hipLaunchKernelGGL(atls::group_count, dim3(G), dim3(256), 0, s, recs, n, n_slots, cnt);
  hipLaunchKernelGGL(atls::group_scan, dim3(1), dim3(1024), 0, s, cnt, n_slots + 1u, cur, gidx, total);
  hipLaunchKernelGGL(atls::group_scatter, dim3(G), dim3(256), 0, s, recs, n, n_slots, cur, gidx);
  return hipGetLastError() == hipSuccess ? 0 : ATLS_INTERNAL_ERROR;
}

// P (device, PlanHdr), keys (n bytes), idx (n words) and wg (2 x 64 x kPlanMaxWG words) are
// engine scratch.
extern "C" int atls_launch_plan(int open, const void* ks, const atls_rec* recs, uint32_t n, uint32_t n_slots,
                                atls_open_result* res, uint32_t* err, void* P, uint8_t* keys, uint32_t* idx,
                                uint32_t* wg, int cus, hipStream_t s) {
  const uint32_t want = (n + 255u) / 256u, cap = (uint32_t)(cus > 0 ? 2 * cus : 512);
  const uint32_t G = want ? (want < cap ? want : cap) : 1u;
  if (G > atls::kPlanMaxWG) return ATLS_INTERNAL_ERROR;
  auto* hdr = (atls::PlanHdr*)P;
  uint32_t* wgcount = wg;
  uint32_t* wgoff = wg + atls::kPlanKeys * atls::kPlanMaxWG;
  hipLaunchKernelGGL(atls::plan_count, dim3(G), dim3(256), 0, s, recs, n, (const atls::KeySched*)ks, n_slots,
                     (uint32_t)(open != 0), res, err, keys, wgcount);
  hipLaunchKernelGGL(atls::plan_scan, dim3(1), dim3(1024), 0, s, (const uint32_t*)wgcount, G, wgoff, hdr);
  hipLaunchKernelGGL(atls::plan_scatter, dim3(G), dim3(256), 0, s, n, (const uint8_t*)keys, (const uint32_t*)wgoff, idx);
  return hipGetLastError() == hipSuccess ? 0 : ATLS_INTERNAL_ERROR;
}
