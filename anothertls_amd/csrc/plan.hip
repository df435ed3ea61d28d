// Batch plan: three small launches before the record kernels.
//
//  1. plan_count: classifies every record (validation of net/record.rs-style descriptors against
//     the key table, crypto/ciphersuite.rs:78-87 get_cipher: AES-GCM for 0x1301/0x1302 with the
//     AES size from the key, ChaCha20-Poly1305 for 0x1303, anything else InsufficientSecurity)
//     into a work list -- AES-GCM with 10 / 12 / 14 rounds, ChaCha20-Poly1305 -- and a length
//     class; rejected records get their status here (err flag; open results for open batches).
//  2. plan_scan: one wave turns the (list, class) counts into offsets, classes ordered longest
//     record first.
//  3. plan_scatter: writes the record indices of every list in that order.
//
// The record kernels (gcm.hip, chacha.hip) then take records from their list with one atomic
// fetch per record (or 16-lane group), longest first: dynamic scheduling that ends a launch on
// short records (LPT), which the variable-length batches (BASELINE config C5) need.
// Counts and cursors use wave-aggregated atomics: one atomic per (wave, distinct class).
#include "plan.h"

namespace atls {

// Work-list key of record i, or kPlanReject (status in *st).
__device__ __forceinline__ uint32_t plan_key(const atls_rec* recs, uint32_t i, const KeySched* ks, uint32_t n_slots,
                                             uint8_t* st) {
  const atls_rec d = recs[i];
  *st = ATLS_ILLEGAL_PARAMETER;
  if (d.key_slot >= n_slots || d.mode > ATLS_MODE_WIRE) return kPlanReject;
  const KeySched* k = ks + d.key_slot;
  const uint32_t suite = k->suite, valid = k->valid, nr = k->nr;
  uint32_t list;
  if (suite == (uint32_t)kSuiteChacha) {
    if (!valid || (d.mode == ATLS_MODE_RAW && d.iv_len != 12)) return kPlanReject;  // cipher.rs:19
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

// For the lanes holding `key`: the number of lanes with the same key, and this lane's rank
// among them. Loops once per distinct key in the wave.
template <typename F>
__device__ __forceinline__ void wave_groups(uint32_t key, bool live, F&& f) {
  uint64_t todo = __ballot(live);
  const int lane = threadIdx.x & 63;
  while (todo) {
    const int leader = __ffsll((unsigned long long)todo) - 1;
    const uint32_t k = __shfl(key, leader);
    const uint64_t mask = __ballot(live && key == k);
    todo &= ~mask;
    const bool mine = live && key == k;
    const uint32_t rank = (uint32_t)__popcll(mask & ((1ull << lane) - 1ull));
    f(k, mask, leader, mine, rank);
  }
}

__global__ __launch_bounds__(256) void plan_count(const atls_rec* recs, uint32_t n, const KeySched* ks,
                                                  uint32_t n_slots, uint32_t open, atls_open_result* res,
                                                  uint32_t* err, uint8_t* keys, PlanHdr* P) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  uint8_t st = 0;
  const uint32_t key = i < n ? plan_key(recs, i, ks, n_slots, &st) : kPlanReject;
  if (i < n) {
    keys[i] = (uint8_t)key;
    if (key == kPlanReject) {
      atomicOr(err, 1u);
      if (open) {
        atls_open_result rr = {0, st, 0, {0, 0}};
        res[i] = rr;
      }
    }
  }
  const int lane = threadIdx.x & 63;
  wave_groups(key, i < n && key != kPlanReject, [&](uint32_t k, uint64_t mask, int leader, bool, uint32_t) {
    if (lane == leader) atomicAdd(&P->count[k], (uint32_t)__popcll(mask));
  });
}

__global__ __launch_bounds__(64) void plan_scan(PlanHdr* P) {
  // one wave: lane j owns the counts of list j's classes (kPlanClasses <= 64 keys per lane group)
  if (threadIdx.x == 0) {
    uint32_t run = 0;
    for (uint32_t l = 0; l < (uint32_t)kPlanLists; l++) {
      P->off[l] = run;
      for (uint32_t c = 0; c < (uint32_t)kPlanClasses; c++) {
        const uint32_t k = l * kPlanClasses + c;
        P->cursor[k] = run;
        run += P->count[k];
      }
      P->next[l] = 0;
    }
    P->off[kPlanLists] = run;
  }
}

__global__ __launch_bounds__(256) void plan_scatter(uint32_t n, const uint8_t* keys, PlanHdr* P, uint32_t* idx) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t key = i < n ? keys[i] : kPlanReject;
  const int lane = threadIdx.x & 63;
  wave_groups(key, i < n && key != kPlanReject, [&](uint32_t k, uint64_t mask, int leader, bool mine, uint32_t rank) {
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(&P->cursor[k], (uint32_t)__popcll(mask));
    base = __shfl(base, leader);
    if (mine) idx[base + rank] = i;
  });
}

}  // namespace atls

// P (device, PlanHdr), keys (n bytes) and idx (n words) are engine scratch.
extern "C" int atls_launch_plan(int open, const void* ks, const atls_rec* recs, uint32_t n, uint32_t n_slots,
                                atls_open_result* res, uint32_t* err, void* P, uint8_t* keys, uint32_t* idx,
                                hipStream_t s) {
  if (hipMemsetAsync(P, 0, sizeof(atls::PlanHdr), s) != hipSuccess) return ATLS_INTERNAL_ERROR;
  const uint32_t g = (n + 255u) / 256u;
  auto* hdr = (atls::PlanHdr*)P;
  if (n) {
    hipLaunchKernelGGL(atls::plan_count, dim3(g), dim3(256), 0, s, recs, n, (const atls::KeySched*)ks, n_slots,
                       (uint32_t)(open != 0), res, err, keys, hdr);
  }
  hipLaunchKernelGGL(atls::plan_scan, dim3(1), dim3(64), 0, s, hdr);
  if (n) hipLaunchKernelGGL(atls::plan_scatter, dim3(g), dim3(256), 0, s, n, (const uint8_t*)keys, hdr, idx);
  return hipGetLastError() == hipSuccess ? 0 : ATLS_INTERNAL_ERROR;
}
