// Batch plan: two small launches before the record kernels.
//
//  1. plan_count: classifies every record (validation of net/record.rs-style descriptors against
//     the key table, crypto/ciphersuite.rs:78-87 get_cipher: AES-GCM for 0x1301/0x1302 with the
//     AES size from the key, ChaCha20-Poly1305 for 0x1303, anything else InsufficientSecurity)
//     into a work list -- AES-GCM with 10 / 12 / 14 rounds, ChaCha20-Poly1305 -- and a length
//     class; rejected records get their status here (err flag; open results for open batches).
//     Each workgroup counts its chunk of the batch in an LDS histogram.
//  2. plan_scatter: each workgroup turns the per-workgroup histograms into its own offsets (lists
//     in order, classes longest record first) and writes its records' indices there (LDS
//     cursors). (A separate one-workgroup plan_scan launch did the offsets before: 14.5 us of a
//     C5 batch; ATLS_PLAN_FUSED_SCAN=0 restores it.)
//
// The record kernels (gcm.hip, chacha.hip) take their list's positions round-robin (WorkList,
// plan.h) -- AES-GCM with each row spread over the workgroups and odd rows reversed, ChaCha in
// 16-record workgroups dispatched longest first -- so every CU gets a similar mix of lengths
// (LPT-like balance for the variable-length batches of BASELINE config C5).
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

#ifndef ATLS_PLAN_FUSED_SCAN
#define ATLS_PLAN_FUSED_SCAN 1
#endif
// wgoff == nullptr (ATLS_PLAN_FUSED_SCAN): no plan_scan launch; every workgroup derives its own
// start offsets from the G x 64 histograms -- per key the total over all workgroups and the part
// of the workgroups before it (4 threads per key), then an exclusive scan of the 64 totals in one
// wave -- and workgroup 0 writes the list offsets. G x 64 words are read by every workgroup (32 KiB
// at G = 128, from L2) instead of one 1,024-thread workgroup scanning them between two launches.
__global__ __launch_bounds__(256) void plan_scatter(uint32_t n, const uint8_t* keys, const uint32_t* wgoff,
                                                    const uint32_t* wgcount, PlanHdr* P, uint32_t* idx) {
  static_assert(kPlanKeys == 64, "one wave scans the key totals");
  __shared__ uint32_t cur[kPlanKeys];
  if (wgoff) {
    for (uint32_t t = threadIdx.x; t < kPlanKeys; t += blockDim.x) cur[t] = wgoff[t * gridDim.x + blockIdx.x];
  } else {
    __shared__ uint32_t tot[kPlanKeys], pre[kPlanKeys];
    const uint32_t G = gridDim.x, b = blockIdx.x, k = threadIdx.x >> 2, q = threadIdx.x & 3u;
    uint32_t all = 0, before = 0;
    if (k < kPlanKeys) {
      const uint32_t* row = wgcount + k * G;
#pragma unroll 8
      for (uint32_t c = q; c < G; c += 4u) {
        const uint32_t v = row[c];
        all += v;
        before += c < b ? v : 0u;
      }
    }
    all += __shfl_xor(all, 1, 4); all += __shfl_xor(all, 2, 4);
    before += __shfl_xor(before, 1, 4); before += __shfl_xor(before, 2, 4);
    if (q == 0 && k < kPlanKeys) { tot[k] = all; pre[k] = before; }
    __syncthreads();
    if (threadIdx.x < 64) {
      const uint32_t v = tot[threadIdx.x];
      uint32_t inc = v;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = __shfl_up(inc, (unsigned)d, 64);
        if (threadIdx.x >= (uint32_t)d) inc += o;
      }
      cur[threadIdx.x] = inc - v + pre[threadIdx.x];
      if (b == 0) {  // list l starts at its longest class, key l * kPlanClasses
        if (threadIdx.x % kPlanClasses == 0) P->off[threadIdx.x / kPlanClasses] = inc - v;
        if (threadIdx.x == 63) P->off[kPlanLists] = inc;
      }
    }
  }
  __syncthreads();
  uint32_t lo, hi;
  plan_chunk(n, lo, hi);
  for (uint32_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
    const uint32_t key = keys[i];
    if (key != kPlanReject) idx[atomicAdd(&cur[key], 1u)] = i;
  }
}

// ---- key groups (direct AES-GCM batches) ----------------------------------------------------
// group_count -> group_alloc -> group_place: a counting sort of the records by key slot (bucket
// n_slots collects refused slots) into the two regions of plan.h, without a pass over the key
// table: the first record of each slot (its rank 0) reserves the slot's ranges in both regions,
// one atomic per workgroup on the region sizes. cnt / cur are all zero between batches
// (group_place clears them).
struct GroupSlots {  // per-slot scratch, nb = n_slots + 1 entries each
  uint32_t *cnt, *cur, *base_a, *base_b, *full;
};

__global__ __launch_bounds__(256) void group_count(const atls_rec* recs, uint32_t n, uint32_t n_slots, uint32_t* cnt,
                                                   GroupHdr* hdr) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    hdr->n_a = hdr->n_b = 0u;
    for (int x = 0; x < 8; x++) hdr->work[x] = 0u;
  }
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint32_t k = recs[i].key_slot;
    atomicAdd(&cnt[k < n_slots ? k : n_slots], 1u);
  }
}

// rank[i] = record i's rank among its slot's records; rank 0 reserves the slot's ranges.
__global__ __launch_bounds__(256) void group_alloc(const atls_rec* recs, uint32_t n, uint32_t n_slots, GroupSlots S,
                                                   GroupHdr* hdr, uint32_t* rank) {
  __shared__ uint32_t sa[256], sb[256], base[2];
  const uint32_t t = threadIdx.x;
  for (uint32_t i0 = blockIdx.x * blockDim.x; i0 < n; i0 += gridDim.x * blockDim.x) {  // block-uniform trip count
    const uint32_t i = i0 + t;
    uint32_t b = 0, j = 1, fa = 0, fb = 0;
    if (i < n) {
      const uint32_t k = recs[i].key_slot;
      b = k < n_slots ? k : n_slots;
      j = atomicAdd(&S.cur[b], 1u);
      rank[i] = j;
      if (j == 0) {
        const uint32_t c = S.cnt[b];
        fa = b < n_slots ? c / kGroupRun * kGroupRun : 0u;  // refused slots: all to region B
        fb = c - fa;
      }
    }
    sa[t] = fa;
    sb[t] = fb;
    __syncthreads();
    for (uint32_t d = 1; d < blockDim.x; d <<= 1) {  // inclusive scan of the reservations
      const uint32_t va = t >= d ? sa[t - d] : 0u, vb = t >= d ? sb[t - d] : 0u;
      __syncthreads();
      sa[t] += va;
      sb[t] += vb;
      __syncthreads();
    }
    if (t == blockDim.x - 1u) {
      base[0] = sa[t] ? atomicAdd(&hdr->n_a, sa[t]) : 0u;
      base[1] = sb[t] ? atomicAdd(&hdr->n_b, sb[t]) : 0u;
    }
    __syncthreads();
    if (j == 0) {
      S.base_a[b] = base[0] + sa[t] - fa;
      S.base_b[b] = base[1] + sb[t] - fb;
      S.full[b] = fa;
    }
    __syncthreads();  // sa / sb / base reused
  }
}

__global__ __launch_bounds__(256) void group_place(const atls_rec* recs, uint32_t n, uint32_t n_slots, GroupSlots S,
                                                   const GroupHdr* hdr, const uint32_t* rank, uint32_t* gidx) {
  const uint32_t n_a = hdr->n_a;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint32_t k = recs[i].key_slot, b = k < n_slots ? k : n_slots;
    const uint32_t j = rank[i], f = S.full[b];
    const uint32_t pos = j < f ? S.base_a[b] + j : n_a + S.base_b[b] + (j - f);
    if (pos < n) gidx[pos] = i;  // always true while cnt / cur start the batch at zero
    S.cnt[b] = 0u;  // every record of the slot writes the same zeros; nothing here reads them
    S.cur[b] = 0u;
  }
}


// The engine's synchronous return (engine.cpp finish): after everything before it on the engine stream,
// one lane copies the sticky error word and then a completion value into mapped host memory, with a
// system-scope release between them, so the host spins on a flag (~6 us on this box) instead of
// hipStreamSynchronize plus a device-to-host copy of the error word (~11 us + a copy).
__global__ void sync_flag_kernel(const uint32_t* err, uint32_t* out, uint32_t val) {
  if (threadIdx.x == 0) {
    out[1] = *reinterpret_cast<const volatile uint32_t*>(err);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    __hip_atomic_store(out, val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

}  // namespace atls

extern "C" int atls_launch_sync_flag(const uint32_t* err, uint32_t* out, uint32_t val, hipStream_t s) {
  hipLaunchKernelGGL(atls::sync_flag_kernel, dim3(1), dim3(64), 0, s, err, out, val);
  return hipGetLastError() == hipSuccess ? 0 : ATLS_INTERNAL_ERROR;
}

// Key groups of a direct batch. cnt: 2 * (n_slots + 1) words (counts, cursors), zero on entry and
// on return. aux: 3 arrays of n_slots + 1 words followed by the GroupHdr (atls_group_hdr_offset
// bytes in), then n words of record ranks. gidx: n words.
extern "C" size_t atls_group_hdr_offset(uint32_t n_slots) {
  return (3u * ((size_t)n_slots + 1u) * 4u + 15u) / 16u * 16u;
}

extern "C" int atls_launch_group(const atls_rec* recs, uint32_t n, uint32_t n_slots, uint32_t* cnt, void* aux,
                                 uint32_t* gidx, int cus, hipStream_t s) {
  if (n_slots > atls::kGroupMaxSlots) return ATLS_INTERNAL_ERROR;
  const uint32_t nb = n_slots + 1u;
  uint32_t* w = (uint32_t*)aux;
  atls::GroupSlots S{cnt, cnt + nb, w, w + nb, w + 2 * nb};
  auto* hdr = (atls::GroupHdr*)((uint8_t*)aux + atls_group_hdr_offset(n_slots));
  uint32_t* rank = (uint32_t*)(hdr + 1);
  const uint32_t want = (n + 255u) / 256u, cap = (uint32_t)(cus > 0 ? 2 * cus : 512);
  const uint32_t G = want ? (want < cap ? want : cap) : 1u;
  hipLaunchKernelGGL(atls::group_count, dim3(G), dim3(256), 0, s, recs, n, n_slots, cnt, hdr);
  hipLaunchKernelGGL(atls::group_alloc, dim3(G), dim3(256), 0, s, recs, n, n_slots, S, hdr, rank);
  hipLaunchKernelGGL(atls::group_place, dim3(G), dim3(256), 0, s, recs, n, n_slots, S, (const atls::GroupHdr*)hdr,
                     (const uint32_t*)rank, gidx);
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
  if (!ATLS_PLAN_FUSED_SCAN)
    hipLaunchKernelGGL(atls::plan_scan, dim3(1), dim3(1024), 0, s, (const uint32_t*)wgcount, G, wgoff, hdr);
  hipLaunchKernelGGL(atls::plan_scatter, dim3(G), dim3(256), 0, s, n, (const uint8_t*)keys,
                     ATLS_PLAN_FUSED_SCAN ? nullptr : (const uint32_t*)wgoff, (const uint32_t*)wgcount, hdr, idx);
  return hipGetLastError() == hipSuccess ? 0 : ATLS_INTERNAL_ERROR;
}
