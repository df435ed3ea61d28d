// AES-CTR keystream on the VALU (bitsliced AES, aes_bs.h) for part of a direct AES-GCM batch.
//
// The T-table record kernel (gcm.hip) is LDS-bound and leaves the VALU half idle; this kernel
// has no LDS traffic at all. The engine runs it on its second stream for the first records of
// a batch while the T-table kernel seals the rest, then a KS instance of the record kernel
// (gcm_kernel<..., KS = true>) seals the first records with the precomputed keystream: XOR,
// GHASH and tag only.
//
// Work unit = one lane: 8 consecutive counters c = 8u .. 8u+7 of one record (c = 0 is J0, whose
// keystream block E_K(J0) masks the tag; c >= 1 encrypts data block c - 1: gcm.rs:71-74,
// :89-96). Lane q handles record q / kKsUnits, unit q % kKsUnits; its 8 counter blocks share
// the nonce and differ in byte 15 upwards, so the bitsliced state is built with one 32x32 bit
// transpose. Round keys differ per lane (records of one wave have different connections): the
// round-key masks are rebuilt from the key schedule's raw words every round.
// A record gets keystream only when it is a valid AES record with a 96-bit IV and at most
// kKsStride - 2 counters; ok[r] says so, and the record kernel falls back to T-tables otherwise.
#include "plan.h"  // hip runtime first: aes_bs.h is also compiled for the host by the CPU tests
#include "aes_bs.h"

namespace atls {

struct KsArgs {
  const KeySched* ks;
  const atls_rec* recs;
  uint32_t n;
  const uint8_t* aux;
  uint8_t* out;  // keystream: record r's block c at out + 16 (r kKsStride + c)
  uint8_t* ok;   // per record: 1 = keystream written
  uint32_t n_slots;
  int open;
};

// One lane-unit: the keystream of counters 8u .. 8u + 7 of record r.
template <int NR>
__device__ __forceinline__ void ks_unit(const KsArgs& A, uint32_t r, uint32_t u) {
  const atls_rec d = A.recs[r];
  const bool tls = d.mode != ATLS_MODE_RAW;
  bool ok = d.key_slot < A.n_slots && d.mode <= ATLS_MODE_WIRE && (tls || d.iv_len == 12);
  const KeySched* k = A.ks + (ok ? d.key_slot : 0u);
  ok = ok && k->valid && k->nr == (uint32_t)NR && (k->suite == (uint32_t)kSuiteAes128 || k->suite == (uint32_t)kSuiteAes256);
  const uint32_t n_aead = (tls && !A.open) ? d.len + 1u : d.len;
  const uint32_t nb = (uint32_t)(((uint64_t)n_aead + 15u) / 16u);
  ok = ok && nb + 2u <= kKsStride;
  if (u == 0) A.ok[r] = ok ? 1 : 0;
  if (!ok || 8u * u > nb) return;  // (lane-divergent: no cross-lane operations below)

  // nonce words as raw little-endian words (gcm.rs:71-74; key_schedule.rs:51-64 for TLS)
  uint32_t nw[3];
  if (tls) {
    nw[0] = k->siv[0];
    nw[1] = k->siv[1] ^ bswap32((uint32_t)(d.seq >> 32));
    nw[2] = k->siv[2] ^ bswap32((uint32_t)d.seq);
  } else {
    const uint8_t* iv = A.aux + d.aux_off;
#pragma unroll
    for (int w = 0; w < 3; w++)
      nw[w] = (uint32_t)iv[4 * w] | ((uint32_t)iv[4 * w + 1] << 8) | ((uint32_t)iv[4 * w + 2] << 16) |
              ((uint32_t)iv[4 * w + 3] << 24);
  }
  // x[8c + b] = raw word c of counter block b: the nonce, then be32(1 + counter) (J0 = nonce || 1)
  uint32_t x[32];
#pragma unroll
  for (int b = 0; b < 8; b++) {
    x[b] = nw[0];
    x[8 + b] = nw[1];
    x[16 + b] = nw[2];
    x[24 + b] = bswap32(1u + 8u * u + (uint32_t)b);
  }
  atls_bs::StateG<1> st;
  atls_bs::blocks_to_group(x, st[0]);
  atls_bs::Masks m;
  const uint32_t* rk = k->rk;
  {
    const uint4 w4 = *reinterpret_cast<const uint4*>(rk);
    const uint32_t w[4] = {w4.x, w4.y, w4.z, w4.w};
    atls_bs::make_masks(w, m);
  }
  atls_bs::add_round_key<1>(st, m);
#pragma unroll 1
  for (int rd = 1; rd <= NR; rd++) {
    atls_bs::sub_bytes<1>(st);
    const uint4 w4 = *reinterpret_cast<const uint4*>(rk + 4 * rd);
    const uint32_t w[4] = {w4.x, w4.y, w4.z, w4.w};
    atls_bs::make_masks(w, m);
    if (rd < NR) atls_bs::shift_mix_ark<1>(st, m);
    else atls_bs::shift_ark<1>(st, m);
  }
  atls_bs::group_to_blocks(st[0], x);
  uint8_t* o = A.out + 16ull * ((uint64_t)r * kKsStride + 8u * u);
#pragma unroll
  for (int b = 0; b < 8; b++)
    if (8u * u + (uint32_t)b <= nb) st16(o + 16 * b, make_uint4(x[b], x[8 + b], x[16 + b], x[24 + b]));
}

// Persistent grid (a few workgroups per CU, striding over the lane-units): short-lived
// workgroups were placed badly beside the resident T-table workgroups and barely overlapped.
template <int NR>
__global__ __launch_bounds__(256) void ks_kernel(KsArgs A) {
  const uint64_t total = (uint64_t)A.n * kKsUnits;
  for (uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; q < total; q += (uint64_t)gridDim.x * blockDim.x)
    ks_unit<NR>(A, (uint32_t)(q / kKsUnits), (uint32_t)(q % kKsUnits));
}

}  // namespace atls

// Keystream for records [0, n) of recs (one AES round count, nr_mask as in atls_launch_gcm).
extern "C" int atls_launch_ks(int open, const void* ks, const atls_rec* recs, uint32_t n, const uint8_t* aux,
                              uint8_t* out, uint8_t* ok, uint32_t n_slots, int nr_mask, int grid_wgs, hipStream_t s) {
  if (n == 0) return 0;
  const atls::KsArgs A{(const atls::KeySched*)ks, recs, n, aux, out, ok, n_slots, open};
  const uint64_t lanes = (uint64_t)n * atls::kKsUnits;
  const uint64_t want = (lanes + 255) / 256;
  const dim3 grid((unsigned)(want < (uint64_t)grid_wgs ? want : (uint64_t)grid_wgs)), block(256);
  if (nr_mask == 1) hipLaunchKernelGGL(atls::ks_kernel<10>, grid, block, 0, s, A);
  else if (nr_mask == 2) hipLaunchKernelGGL(atls::ks_kernel<12>, grid, block, 0, s, A);
  else if (nr_mask == 4) hipLaunchKernelGGL(atls::ks_kernel<14>, grid, block, 0, s, A);
  else return ATLS_INTERNAL_ERROR;
  return hipGetLastError() == hipSuccess ? 0 : ATLS_INTERNAL_ERROR;
}
