// Work lists of a batch (plan.hip) as the record kernels read them.
#pragma once
#include "atls_dev.h"

namespace atls {

constexpr uint32_t kListGcm10 = 0, kListGcm12 = 1, kListGcm14 = 2, kListChacha = 3;
constexpr int kPlanLists = 4;
constexpr int kPlanClasses = 16;  // length classes min(len >> 10, 15), longest first
constexpr uint32_t kPlanReject = 0xffu;
constexpr uint32_t kPlanKeys = kPlanLists * kPlanClasses;  // work-list keys (list, length class)
constexpr uint32_t kPlanMaxWG = 1024;                      // plan workgroups (2 per CU)
// Single Cipher-trait calls (engine.cpp single): IV || AAD || input || received tag of up to this many
// bytes travel in the launch's argument block (gcm_single / chacha_single), with the descriptor.
constexpr uint32_t kSingleInline = 3584;

struct PlanHdr {
  uint32_t off[kPlanLists + 1];                  // list l = idx[off[l] .. off[l+1])
  uint32_t next[kPlanLists];                     // unused
  uint32_t count[kPlanLists * kPlanClasses];     // unused
  uint32_t cursor[kPlanLists * kPlanClasses];    // unused
};

// The record kernels' view: list `l` of the plan. Workers (waves or lane groups) take positions
// round-robin: worker w of W takes w, w + W, w + 2W, ... of a list ordered longest first, so every
// worker gets a similar mix of lengths. (A shared atomic fetch counter was measured 2-6x slower:
// device-scope atomics on one address serialise at the memory side.)
// idx == nullptr: no plan ("direct" batches whose key table holds one record kernel's suite and
// round count only): position q is record q and the kernel validates descriptors itself.
struct WorkList {
  const uint32_t* idx;  // record indices, longest first
  PlanHdr* P;
  uint32_t list;
  uint32_t n;           // batch size (direct mode)

  __device__ __forceinline__ uint32_t size() const { return idx ? P->off[list + 1] - P->off[list] : n; }
  __device__ __forceinline__ uint32_t record(uint32_t pos) const { return idx ? idx[P->off[list] + pos] : pos; }
};

// Key groups of a direct AES-GCM batch (group_* kernels, plan.hip): the record indices in two
// regions. Region A: for every key slot, floor(count / kGroupRun) * kGroupRun of its records, so
// every aligned run of kGroupRun positions holds one key (a lane group for gcm.hip gcm_group).
// Region B: the rest (a slot's remainder, refused slots), compact. Nothing is padded.
constexpr uint32_t kGroupRun = 8;  // the records of one wave at 8 lanes each
constexpr uint32_t kGroupMaxSlots = 1u << 24;  // larger key tables are not grouped (per-slot scratch)
// Group plan header after the per-slot arrays (atls_launch_group).
struct GroupHdr {
  uint32_t n_a, n_b;  // region sizes
  uint32_t work[8];   // work counters of the record kernel, one per XCD share of region A
  uint32_t pad[2];
};

// ChaCha20::encrypt counts its 64-byte blocks as (len as f32 / 64.0).ceil() (chacha20/cipher.rs:94),
// exact only while the AEAD input is below 2^24 bytes. Longer ChaCha20-Poly1305 records are
// refused (ILLEGAL_PARAMETER) instead of being sealed differently from the reference.
__device__ __forceinline__ bool chacha_len_ok(const atls_rec& d, bool open) {
  const uint64_t aead = (uint64_t)d.len + ((!open && d.mode != ATLS_MODE_RAW) ? 1u : 0u);  // + type byte
  return aead < (1ull << 24);
}

// Direct mode: the status a record gets in place of sealing / opening (0 = process it), as
// plan_key would give it (plan.hip).
__device__ __forceinline__ uint32_t direct_reject(const atls_rec& d, const KeySched* ks, uint32_t n_slots, bool open) {
  if (d.key_slot >= n_slots || d.mode > ATLS_MODE_WIRE) return ATLS_ILLEGAL_PARAMETER;
  const KeySched* k = ks + d.key_slot;
  const uint32_t suite = k->suite;
  if (suite == (uint32_t)kSuiteChacha)
    return (!k->valid || (d.mode == ATLS_MODE_RAW && d.iv_len != 12) || !chacha_len_ok(d, open)) ? ATLS_ILLEGAL_PARAMETER : 0;
  if (suite == (uint32_t)kSuiteAes128 || suite == (uint32_t)kSuiteAes256) return k->valid ? 0 : ATLS_ILLEGAL_PARAMETER;
  return ATLS_INSUFFICIENT_SECURITY;
}

}  // namespace atls
