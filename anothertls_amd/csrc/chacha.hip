// ChaCha20-Poly1305 seal/open for TLS records on gfx950.
//
// Restates crypto/chacha20/cipher.rs:12-108 and crypto/chacha20/poly1305.rs:19-99 (RFC 8439
// AEAD) for a batch of records, including the reference's F4 quirk: ChaCha20::encrypt leaves
// the last 64-byte block unencrypted when len % 64 == 0 (cipher.rs:99-102), and the tag is
// computed over that output. Record framing as in net/record.rs:162-240.
//
// Mapping: a group of G lanes per record (G = 16; 4 or 2 for short records, chacha_kernel). Slot j of a record
// is ChaCha20 block counter j: slot 0 = Poly1305 key generation (poly1305.rs:19-22) plus the
// AAD blocks, slot j >= 1 = bytes [64(j-1), 64j) of the record (counter starts at 1,
// poly1305.rs:77). Lane l of the group owns slots j = l (mod 16): each step the group reads and
// writes one contiguous 1 KiB run of the record.
// Poly1305 (p = 2^130-5, 26-bit limbs, v_mad_u64_u32 products): a slot's four 16-byte pieces
// (ciphertext, then the length block) are Horner-folded with r; slots of one lane are folded
// with r^(4G) = r^64; each lane's partial is finally multiplied by r^e (e in 1..65, square-
// and-multiply over r^(2^b)) and the group sums the partials mod p.
// Kernels: chacha_kernel_w2 (direct batches, the default: 2 waves per SIMD, each slot's block loaded a
// step ahead, full slots' MACs folded in one reduction), chacha_kernel<OPEN, false> (direct batches under
// ATLS_CHACHA_W2=0/1, 3 waves per SIMD), chacha_kernel<OPEN, true> (planned mixed batches beside the
// AES-GCM kernel, 128 VGPRs), chacha_kernel_lat (the single call, one record per wave at 64 lanes).
// Bytes per record (roofline): read L, write L + 16.
#include "chacha_q4.h"
#include "plan.h"

namespace atls {

#ifndef ATLS_CHACHA_SHORT
#define ATLS_CHACHA_SHORT 4096  // records up to this length take 4 lanes each, longer ones 16
#endif
// ---- ChaCha20 block (chacha20/cipher.rs:56-87) ----
#define QR(a, b, c, d)                      \
  a += b; d = rotl32(d ^ a, 16);            \
  c += d; b = rotl32(b ^ c, 12);            \
  a += b; d = rotl32(d ^ a, 8);             \
  c += d; b = rotl32(b ^ c, 7);

__device__ __forceinline__ void chacha_block(const uint32_t kw[8], uint32_t ctr, const uint32_t nw[3], uint32_t o[16]) {
  uint32_t x0 = 0x61707865, x1 = 0x3320646e, x2 = 0x79622d32, x3 = 0x6b206574;
  uint32_t x4 = kw[0], x5 = kw[1], x6 = kw[2], x7 = kw[3], x8 = kw[4], x9 = kw[5], x10 = kw[6], x11 = kw[7];
  uint32_t x12 = ctr, x13 = nw[0], x14 = nw[1], x15 = nw[2];
#ifndef ATLS_CHACHA_UNROLL
#define ATLS_CHACHA_UNROLL 2  // double rounds per loop trip: 1 / 5 / 10 measured no better (C5 +1 / +2 / +5 %,
                              // profiles/r02/ab_chacha_unroll.log)
#endif
#pragma unroll ATLS_CHACHA_UNROLL
  for (int i = 0; i < 10; i++) {
    QR(x0, x4, x8, x12) QR(x1, x5, x9, x13) QR(x2, x6, x10, x14) QR(x3, x7, x11, x15)
    QR(x0, x5, x10, x15) QR(x1, x6, x11, x12) QR(x2, x7, x8, x13) QR(x3, x4, x9, x14)
  }
  o[0] = x0 + 0x61707865; o[1] = x1 + 0x3320646e; o[2] = x2 + 0x79622d32; o[3] = x3 + 0x6b206574;
  o[4] = x4 + kw[0]; o[5] = x5 + kw[1]; o[6] = x6 + kw[2]; o[7] = x7 + kw[3];
  o[8] = x8 + kw[4]; o[9] = x9 + kw[5]; o[10] = x10 + kw[6]; o[11] = x11 + kw[7];
  o[12] = x12 + ctr; o[13] = x13 + nw[0]; o[14] = x14 + nw[1]; o[15] = x15 + nw[2];
}
#undef QR

struct ChArgs {
  const KeySched* ks;
  const atls_rec* recs;
  uint32_t n;
  const uint8_t* in;
  const uint8_t* aux;
  uint8_t* out;
  uint8_t* tags_out;
  const uint8_t* tags_in;
  atls_open_result* res;
  const uint32_t* idx;  // batch plan (plan.hip); nullptr: direct
  PlanHdr* plan;
  uint32_t* err;        // direct mode: sticky error word
  uint32_t n_slots;     // direct mode: key-table size
  uint32_t* done;       // one-record latency launch: completion flag (gcm_common.h signal_done)
  uint32_t done_val;
};

// Phase clocks of the single call (timing build -DATLS_LAT_STAMPS, tools/single_call_stamps.py): lane 0
// of a one-record 64-lane wave adds the shader clock at each point to g_lat_stamps[i] after waiting for
// its outstanding memory operations (so a phase ends when its loads have landed); [8] / [9] hold the
// 100 MHz real-time clock at entry / exit, [15] the call count.
#ifdef ATLS_LAT_STAMPS
__device__ unsigned long long g_lat_stamps[16];
#define LAT_STAMP(i, lane0)                                                   \
  do {                                                                        \
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");               \
    const uint64_t t_ = __builtin_amdgcn_s_memtime();                         \
    if (lane0) atomicAdd(&g_lat_stamps[i], (unsigned long long)t_);           \
  } while (0)
#else
#define LAT_STAMP(i, lane0) do { } while (0)
#endif

// LATE: r^2 and r^3 for the lane combine are recomputed after the slot loop instead of living
// through it (10 fewer VGPRs there, 2 more multiplies per record and lane). Same-box A/B over 3
// rounds (profiles/r03/ab_chacha_late_pow.log): the open kernels and the planned seal kernel spill
// less (direct open 33 -> 17 VGPRs, planned open 57 -> 39, planned seal 5 -> 0): C5 open 0.350 ->
// 0.323 ms, C5 seal 0.318 -> 0.316 ms, C3 open within noise; the direct seal kernel (no spills either
// way) keeps them live (C3 seal 0.085-0.087 ms both ways; loading each slot's data before its keystream
// measured 3-8 % slower on C3 in every variant, profiles/r03/ab_chacha_preload.log).
// CARRY (direct batches; lds = this lane's 4 LDS slots of 16 B): a step of G lanes covers the record's
// bytes [64 (base - 1), 64 (base + G - 1)), which starts 64 B before the slot grid, so unless the
// output sits at (dst - 64) % 128 == 0 the window's last `mis` bytes share a 128-B line with the next
// step's first bytes. Written at once, that line is written in two steps far apart and the L2 writes
// it back twice (31 64-B writes per 24-segment record instead of 24.4, tools/recipes/sessions/_r3_traffic3.sh). With
// CARRY those trailing 16-B pieces wait in LDS and are stored in the next step, beside the rest of
// their line.
// MAC_FIRST (opens; 1 = planned kernels, 2 = planned and direct): a data slot's ciphertext is folded
// into the MAC before its keystream is computed, so the 16 keystream words are not live through the
// Poly1305 products. Planned open kernel (128-VGPR cap) spills 128 -> 12 B per lane, direct open 68 ->
// 28. The spills were HBM traffic: C5's ChaCha open read 2.23 M 128-B lines per launch (the seal 1.12
// M) and wrote 3.07 M requests (2.22 M), now 1.13 M / 2.23 M. Same-box A/B over 3 rounds
// (profiles/r03/ab_chacha_mac_first.log): C5 open kernel 0.320 -> 0.306 ms, C3 open 0.1010 -> 0.0994 ms;
// a 3-wave bound for the planned open instead (152 VGPRs, no spills) fixed the traffic but not the
// time (0.325 ms: no wave of it fits beside an AES-GCM workgroup).
#ifndef ATLS_CHACHA_DBG
#define ATLS_CHACHA_DBG 0  // timing builds only (wrong results): 1 = no keystream for data slots, 2 = no MAC of
                           // full seal slots, 4 = no loads or stores of full blocks (PRE >= 2 kernels); round 6
                           // (the per-record share priced part by part): 8 = no r-power lane scan
                           // (R = r^4 on every lane), 16 = no lane-combine products (contrib = acc), 32 = no tag
                           // finish (p_finish), 64 = no r^2 / r^3 / r^4 products (powers = r), 128 = direct
                           // batches: a wave reads its step's record lengths and does nothing else (the launch floor),
                           // 256 (with 1) = no key-block keystream either
#endif
#ifndef ATLS_CHACHA_SOP
#define ATLS_CHACHA_SOP 1
#endif
#ifndef ATLS_CHACHA_KW_RELOAD
#define ATLS_CHACHA_KW_RELOAD 1  // the planned open kernel reloads the key words per keystream block (chacha_record)
#endif
#ifndef ATLS_CHACHA_W2_MAC_FIRST
#define ATLS_CHACHA_W2_MAC_FIRST 0  // 0: the 2-wave kernel's opens compute the keystream first (it has the registers):
                                    // C3 open 0.0942 -> 0.0896 ms (profiles/r03/ab_c3_open2.log, ab_c3_open.log)
#endif
#ifndef ATLS_CHACHA_OPEN_MAC_FIRST
#define ATLS_CHACHA_OPEN_MAC_FIRST 2
#endif
typedef uint32_t v4u32_ch __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4u32_ch lds_uint4;
// PRE: 0 = a slot's data is loaded where it is used (after its keystream); 1 = at the top of its step,
// before the keystream; 2 = one step ahead, before the previous step's stores (chacha_kernel_w2).
// The single call's records beyond the argument block (> 3.5 KiB: more than one 64-lane step from ~4 KiB)
// take 4 waves (G = 256: 16,385 B seal 32.5 -> 23.2 us); those in the argument block stay on one wave,
// where the 4-wave record measured slower (1,537 B seal 15.4 -> 17.1 us: barriers, exchange, a fuller scan).
#ifndef ATLS_CHACHA_SINGLE_4W
#define ATLS_CHACHA_SINGLE_4W 1
#endif
constexpr int kChSingleThreads = 64;
// G = 256: one record on a 4-wave workgroup (the single call; slot j on thread j mod 256): lane scans and
// reductions run per wave, the waves meet in LDS (Poly1305 key broadcast, partial tags, content-type scan),
// and wave w's powers carry the factor r^(256 w) (r^256 = its lane 63's (r^4)^64).
template <bool OPEN, int G, bool LATE, bool CARRY = false, int PRE = G >= 64 ? 1 : 0, bool STAGE = false>
__device__ void chacha_record(const ChArgs& A, const atls_rec& d, const KeySched* k, uint32_t rec_idx, int gl,
                              lds_uint4* lds = nullptr) {
  // TLS and WIRE: nonce from (static IV, seq), 5-byte AAD; WIRE also frames the record
  const bool wire = d.mode == ATLS_MODE_WIRE;
  const bool tls = d.mode != ATLS_MODE_RAW;
  const uint32_t len = d.len;
  const uint32_t n = (tls && !OPEN) ? len + 1 : len;
  const uint8_t* rec_in = A.in + d.in_off;
  const uint8_t* src = rec_in + ((OPEN && wire) ? 5u : 0u);
  uint8_t* dst = A.out + d.out_off + ((!OPEN && wire) ? 5u : 0u);

  // KW_RELOAD (the planned open: 128-VGPR cap beside AES-GCM, MAC folded before the keystream): the 8 key
  // words are loaded again (L1 / L2-resident, 32 B) for each keystream block instead of staying live
  // through the slot's Poly1305 products
  constexpr bool KW_RELOAD = ATLS_CHACHA_KW_RELOAD && OPEN && G == 16 && LATE && PRE == 0 && !CARRY;
  uint32_t kw[8];
  if (!KW_RELOAD)
    for (int i = 0; i < 8; i++) kw[i] = k->kw[i];
  uint32_t nw[3];
  uint32_t aad_len = 5, hdr0 = 0, hdr1 = 0;
  const uint8_t* aadp = nullptr;
  bool hdr_ok = true;
  if (tls) {
    nw[0] = k->siv[0];
    nw[1] = k->siv[1] ^ bswap32((uint32_t)(d.seq >> 32));
    nw[2] = k->siv[2] ^ bswap32((uint32_t)d.seq);
    if (OPEN && wire) {  // the received header is the AAD (record.rs:219)
      hdr_ok = wire_header(rec_in, len, hdr0, hdr1);
    } else {
      const uint32_t L = n + 16;
      hdr0 = 0x17u | (0x03u << 8) | (0x03u << 16) | (((L >> 8) & 0xffu) << 24);
      hdr1 = L & 0xffu;
    }
  } else {
    const uint8_t* iv = A.aux + d.aux_off;
    for (int w = 0; w < 3; w++)
      nw[w] = (uint32_t)iv[4 * w] | ((uint32_t)iv[4 * w + 1] << 8) | ((uint32_t)iv[4 * w + 2] << 16) |
              ((uint32_t)iv[4 * w + 3] << 24);
    aad_len = d.aad_len;
    aadp = iv + 12;
  }
  auto keystream = [&](uint32_t jj, uint32_t (&o)[16]) {
    if constexpr (KW_RELOAD) {
      uint64_t kp = reinterpret_cast<uint64_t>(k->kw);
      asm volatile("" : "+v"(kp));  // opaque: the loads stay at this point instead of being hoisted out of the loop
      const uint4 a = ld16(reinterpret_cast<const uint8_t*>(kp)), b = ld16(reinterpret_cast<const uint8_t*>(kp) + 16);
      const uint32_t kx[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
      chacha_block(kx, jj, nw, o);
    } else {
      chacha_block(kw, jj, nw, o);
    }
  };
  if (G == 64) LAT_STAMP(1, gl == 0);  // descriptor, key words, nonce / AAD in registers
  const uint32_t na = tls ? 1u : (aad_len + 15u) / 16u;
  const uint32_t nct = (n + 15u) / 16u;         // ciphertext pieces (pad16, poly1305.rs:52-56)
  const uint32_t jmax = (n + 63u) / 64u;        // data blocks (f32 ceil is exact below 2^24)
  const uint32_t jL = nct / 4u + 1u;            // slot holding the length piece (c = nct)
  const uint32_t Q = na + nct + 1u;             // Poly1305 blocks
  const bool f4 = (n % 64u) == 0u;              // cipher.rs:100-102: last block not XORed

  // r powers: r, rsq = r^2, rcu = r^3 in every lane; R = (r^4)^(gl+1) by a prefix-product scan over the 16
  // lanes of the group (4 levels); r64 = r^64 (lane 15's R).
  P130 r = p_zero(), rsq = p_zero(), rcu = p_zero(), R = p_zero(), r64 = p_zero();
  constexpr int GW = G > 64 ? 64 : G;  // lanes of one wave in the group
  P130 r256 = p_zero(), r512 = p_zero(), r768 = p_zero();  // G = 256: wave factors
  uint32_t sk[4] = {0, 0, 0, 0};
  P130 acc = p_zero(), innerL = p_zero();
  // open: ((offset + 1) << 8) | byte of the last non-zero plaintext byte, 0 = none (32 bits: ChaCha20-Poly1305
  // records are < 2^24 bytes, plan.h chacha_len_ok; one VGPR instead of a 64-bit pair)
  uint32_t lastnz = 0;
  constexpr bool MAC_FIRST = OPEN && G != 64 && (PRE < 2 || ATLS_CHACHA_W2_MAC_FIRST) &&
                             (CARRY ? ATLS_CHACHA_OPEN_MAC_FIRST >= 2 : ATLS_CHACHA_OPEN_MAC_FIRST >= 1);
  constexpr bool SOP = ATLS_CHACHA_SOP && !LATE;  // full slots: one reduction (p_sop4)
  const uint32_t mis = CARRY ? (uint32_t)((reinterpret_cast<uintptr_t>(dst) - 64u) & 127u) : 0u;
  uint32_t cmask = 0, coff = 0;  // CARRY: pieces of the block at record offset coff waiting in LDS
  auto flush = [&]() {
    if (CARRY && cmask) {
#pragma unroll
      for (int q = 0; q < 4; q++)
        if (cmask & (1u << q)) {
          const v4u32_ch c = lds[q];
          st16(dst + coff + 16 * q, make_uint4(c.x, c.y, c.z, c.w));
        }
      cmask = 0;
    }
  };

  // STAGE (round 4 A/B of VERDICT r3 #6; seals in waves whose records all take the same steps): a step's
  // whole output blocks wait in the lane's LDS slots and go out at the top of the next step, transposed so
  // that lanes 8k..8k+7 of one store instruction write one record's 128 contiguous bytes (the two lanes'
  // blocks), not two 16-B pieces of each of 32 records. Collective: every lane of the wave runs it.
  uint4 sb[4] = {};
  uint8_t* sdst = nullptr;
  bool sv = false;
  auto stage_flush = [&]() {
    if constexpr (STAGE) {
#pragma unroll
      for (int q = 0; q < 4; q++) lds[q] = v4u32_ch{sb[q].x, sb[q].y, sb[q].z, sb[q].w};
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
      const int lane = (int)(threadIdx.x & 63);
      lds_uint4* wbase = lds - 4 * lane;
      const uint64_t pd = reinterpret_cast<uint64_t>(sdst);
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const int sl = 16 * q + lane / 4;  // source lane; piece lane % 4 of its block
        const v4u32_ch v = wbase[64 * q + lane];
        const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)pd, sl, 64), hi = (uint32_t)__shfl((int)(uint32_t)(pd >> 32), sl, 64);
        const int f = __shfl((int)sv, sl, 64);
        if (f) st16(reinterpret_cast<uint8_t*>(((uint64_t)hi << 32) | lo) + 16 * (lane & 3), make_uint4(v.x, v.y, v.z, v.w));
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
      sv = false;
    }
  };

  // PRE >= 2: every lane loads 64 B per step whatever its slot (a whole block of the slot PRE - 1 steps
  // ahead, or the always-readable key schedule): an unconditional load keeps the compiler's s_waitcnt
  // for the current block from waiting on the prefetches too. ring[0] is the current step's block.
  auto blk_addr = [&](uint32_t jj) -> const uint8_t* {
    return (!(ATLS_CHACHA_DBG & 4) && jj >= 1 && jj <= jmax && 64u * (jj - 1) + 64u <= len) ? src + 64u * (jj - 1)
                                                                                             : (const uint8_t*)k;
  };
  constexpr int NR = PRE >= 2 ? PRE - 1 : 1;
  uint4 ring[NR][4] = {};
  uint4 (&pre)[4] = ring[0];
  if (PRE >= 2) {
#pragma unroll
    for (int i = 0; i < NR; i++) {
      const uint8_t* a0 = blk_addr((uint32_t)gl + (uint32_t)(i * G));
#pragma unroll
      for (int q = 0; q < 4; q++) ring[i][q] = ld16(a0 + 16 * q);
    }
  }
  for (uint32_t base = 0; base <= jL; base += G) {
    stage_flush();  // STAGE: the previous step's blocks (every lane, before any lane-dependent branch)
    const uint32_t j = base + (uint32_t)gl;
    const bool active = j <= jL;
    // Latency path (G = 64, one record per wave, the single call): the block's data is loaded before
    // its keystream is computed, so the load's latency (PCIe when the kernel reads pinned host
    // memory) hides under the ChaCha rounds. The throughput paths keep the registers free instead.
    uint4 nxt[4] = {};
    if (PRE >= 2) {
      const uint8_t* an = blk_addr(j + (uint32_t)(NR * G));
#pragma unroll
      for (int q = 0; q < 4; q++) nxt[q] = ld16(an + 16 * q);
    }
    if (PRE == 1 && active && j >= 1 && j <= jmax && 64u * (j - 1) + 64u <= len) {
#pragma unroll
      for (int q = 0; q < 4; q++) pre[q] = ld16(src + 64u * (j - 1) + 16 * q);
    }
    if (G == 64 && base == 0) LAT_STAMP(2, gl == 0);  // the step's data blocks loaded
    uint32_t ks[16];
    if (active && j <= jmax && (!MAC_FIRST || j == 0)) {
      if ((ATLS_CHACHA_DBG & 1) != 0 && (j != 0u || (ATLS_CHACHA_DBG & 256) != 0)) {  // timing build: no keystream for data slots
        // (wrong output); with 256 none for the Poly1305 key block either
#pragma unroll
        for (int q = 0; q < 16; q++) ks[q] = kw[q & 7] ^ j;
      } else {
        keystream(j, ks);
      }
    }
    if (G == 64 && base == 0) LAT_STAMP(3, gl == 0);  // keystream blocks
    if (base == 0) {
      // Poly1305 one-time key from block 0 (poly1305.rs:19-22), broadcast within the group.
      uint32_t r0, r1, r2, r3;
      if constexpr (G > 64) {
        __shared__ uint32_t bc[8];
        if (gl == 0) {
#pragma unroll
          for (int i = 0; i < 8; i++) bc[i] = ks[i];
        }
        __syncthreads();
        r0 = bc[0]; r1 = bc[1]; r2 = bc[2]; r3 = bc[3];
        sk[0] = bc[4]; sk[1] = bc[5]; sk[2] = bc[6]; sk[3] = bc[7];
      } else {
        r0 = __shfl(ks[0], 0, G); r1 = __shfl(ks[1], 0, G); r2 = __shfl(ks[2], 0, G); r3 = __shfl(ks[3], 0, G);
        sk[0] = __shfl(ks[4], 0, G); sk[1] = __shfl(ks[5], 0, G); sk[2] = __shfl(ks[6], 0, G); sk[3] = __shfl(ks[7], 0, G);
      }
      r0 &= 0x0fffffffu; r1 &= 0x0ffffffcu; r2 &= 0x0ffffffcu; r3 &= 0x0ffffffcu;  // clamp (:26)
      r.l[0] = r0 & M26;
      r.l[1] = ((r0 >> 26) | (r1 << 6)) & M26;
      r.l[2] = ((r1 >> 20) | (r2 << 12)) & M26;
      r.l[3] = ((r2 >> 14) | (r3 << 18)) & M26;
      r.l[4] = r3 >> 8;
      if (ATLS_CHACHA_DBG & 64) {  // timing build: no power products
        rsq = r;
        R = r;
        if (!LATE) rcu = r;
      } else {
        rsq = p_mul(r, r);
        R = p_mul(rsq, rsq);  // r^4
        if (!LATE) rcu = p_mul(rsq, r);
      }
#pragma unroll
      for (int d = 1; d < ((ATLS_CHACHA_DBG & 8) ? 1 : GW); d <<= 1) {  // Hillis-Steele prefix product (G = 256: within each wave)
        // one record per wave (the single call): lanes past jL hold no slot, so a record of one step
        // (jL < 32: up to ~1.9 KiB) stops after the levels lanes 0..jL need (5 for an MTU-sized record)
        if (G == 64 && (uint32_t)d > jL) continue;
        P130 t;
#pragma unroll
        for (int i = 0; i < 5; i++) t.l[i] = __shfl_up(R.l[i], (unsigned)d, GW);
        const P130 m = p_mul(R, t);
        if ((gl & (GW - 1)) >= d) R = m;
      }
      if constexpr (G > 64) {  // (r^4)^(l+1) per wave lane l; r^(4G) = r^1024 for the slot Horner
        r256 = shfl_p<64>(R, 63);
        r512 = p_mul(r256, r256);
        r768 = p_mul(r512, r256);
        r64 = p_mul(r512, r512);
      } else {
        r64 = shfl_p<G>(R, G - 1);
      }
      if (G == 64) LAT_STAMP(4, gl == 0);  // r powers (lane scan)
    }
    if (!active) continue;
    const uint4 cur0 = pre[0], cur1 = pre[1], cur2 = pre[2], cur3 = pre[3];
    if (PRE >= 2) {
#pragma unroll
      for (int i = 0; i + 1 < NR; i++)
#pragma unroll
        for (int q = 0; q < 4; q++) ring[i][q] = ring[i + 1][q];
#pragma unroll
      for (int q = 0; q < 4; q++) ring[NR - 1][q] = nxt[q];  // the block PRE - 1 steps ahead
    }

    P130 inner = p_zero();
    uint32_t cnt = 0;
    bool sop = false;
    if (j == 0) {  // AAD blocks (get_mac_data: aad || pad16, poly1305.rs:57-59)
      uint32_t al = aad_len;  // na blocks; the bound is derived here, behind an opaque copy, so that no trip count is
      asm volatile("" : "+v"(al));  // hoisted and kept live through the slot loop (the planned open spilled it)
      for (uint32_t i = 0; 16u * i < al; i++) {
        uint32_t B[4] = {0, 0, 0, 0};
        if (tls) {
          B[0] = hdr0; B[1] = hdr1;
        } else {
#pragma unroll
          for (int q = 0; q < 16; q++)
            if (16 * i + q < aad_len) B[q >> 2] |= (uint32_t)aadp[16 * i + q] << (8 * (q & 3));
        }
        if (cnt) inner = p_mul(inner, r);
        p_add_block(inner, B[0], B[1], B[2], B[3]);
        cnt++;
      }
    } else {
      // Horner of this slot's four 16-byte Poly1305 pieces (ciphertext, then the length block)
      auto fold = [&](const uint32_t (&X)[16]) {
#pragma unroll
        for (int u = 0; u < 4; u++) {
          const uint32_t c = 4u * (j - 1) + u;
          if (c < nct) {
            if (u) inner = p_mul(inner, r);  // piece u = 0 starts the slot's Horner
            p_add_block(inner, X[4 * u], X[4 * u + 1], X[4 * u + 2], X[4 * u + 3]);
            cnt++;
          } else if (c == nct) {  // le64(aad_len) || le64(ct_len) (poly1305.rs:63-64)
            if (u) inner = p_mul(inner, r);
            p_add_block(inner, tls ? 5u : aad_len, 0u, n, 0u);
            cnt++;
          }
        }
      };
      // bytes past `valid` of a partial block are zero (the MAC's zero padding, the stores' mask)
      auto mask_valid = [](uint32_t (&X)[16], uint32_t valid) {
        if (valid < 64) {
#pragma unroll
          for (int q = 0; q < 16; q++) {
            const int lo = 4 * q;
            if ((int)valid < lo + 4) X[q] &= ((int)valid <= lo) ? 0u : (0xffffffffu >> (8 * (lo + 4 - (int)valid)));
          }
        }
      };
      if (j <= jmax) {
        const uint32_t off = 64u * (j - 1);
        uint32_t P[16];
        const uint32_t valid = min(64u, n - off);
        if (off + 64 <= len) {
#pragma unroll
          for (int q = 0; q < 4; q++) {
            const uint4 v = PRE ? (q == 0 ? cur0 : q == 1 ? cur1 : q == 2 ? cur2 : cur3) : ld16(src + off + 16 * q);
            P[4 * q] = v.x; P[4 * q + 1] = v.y; P[4 * q + 2] = v.z; P[4 * q + 3] = v.w;
          }
        } else {
          // a partial block, word by word (compile-time word index: P stays in registers): a word wholly
          // inside the input is one 4-byte load, the word holding the input's end is assembled from
          // bytes and the content type (record.rs:173); words past `valid` stay zero
#pragma unroll
          for (int w = 0; w < 16; w++) {
            P[w] = 0;
            const uint32_t b0 = 4u * (uint32_t)w;
            if (b0 < valid) {
              if (off + b0 + 4u <= len) {
                P[w] = ld4(src + off + b0);
              } else {
#pragma unroll
                for (int q = 0; q < 4; q++)
                  if (b0 + (uint32_t)q < valid)
                    P[w] |= ((off + b0 + (uint32_t)q < len) ? (uint32_t)src[off + b0 + q] : (uint32_t)d.content_type)
                            << (8 * q);
              }
            }
          }
        }
        const bool skip_xor = f4 && j == jmax;  // cipher.rs:99-102: the last block is not XORed
        if (OPEN) {
          // MAC over the received ciphertext first, then the plaintext in the same registers (no
          // second 16-word block live beside the keystream: the open kernels stay within their caps)
          mask_valid(P, valid);
          if (SOP && valid == 64u) {
            p_sop4(acc, base == 0, r64, P, r, rsq, rcu);
            sop = true;
          } else {
            fold(P);
          }
          if (MAC_FIRST) keystream(j, ks);
#pragma unroll
          for (int q = 0; q < 16; q++) P[q] = skip_xor ? P[q] : (P[q] ^ ks[q]);
          mask_valid(P, valid);
        } else {
#pragma unroll
          for (int q = 0; q < 16; q++) P[q] = skip_xor ? P[q] : (P[q] ^ ks[q]);
          mask_valid(P, valid);
        }
        flush();  // the previous step's trailing pieces go out with the rest of their line
        if (valid == 64) {
          const uint32_t thr = 64u * (base + G - 1u) - mis;  // record offset where the window's partial line starts
#pragma unroll
          for (int q = 0; q < 4; q++) {
            const uint4 v = make_uint4(P[4 * q], P[4 * q + 1], P[4 * q + 2], P[4 * q + 3]);
            if (STAGE) {
              sb[q] = v;
              sdst = dst + off;
              sv = true;
            } else if (CARRY && mis && off + 16u * q >= thr) {
              lds[q] = v4u32_ch{v.x, v.y, v.z, v.w};
              cmask |= 1u << q;
              coff = off;
            } else {
              if (!(ATLS_CHACHA_DBG & 4)) st16(dst + off + 16 * q, v);
            }
          }
        } else {
#pragma unroll
          for (int w = 0; w < 16; w++) {  // word by word, bytes only for the word holding the end
            const uint32_t b0 = 4u * (uint32_t)w;
            if (b0 + 4u <= valid) {
              st4(dst + off + b0, P[w]);
            } else if (b0 < valid) {
#pragma unroll
              for (int q = 0; q < 4; q++)
                if (b0 + (uint32_t)q < valid) dst[off + b0 + q] = (uint8_t)(P[w] >> (8 * q));
            }
          }
        }
        if (OPEN) {
          if (tls) {
            for (int q = 15; q >= 0; q--) {
              if (P[q]) {
                const int bi = 4 * q + (31 - __builtin_clz(P[q])) / 8;
                lastnz = ((off + (uint32_t)bi + 1u) << 8) | ((P[q] >> (8 * (bi & 3))) & 0xffu);
                break;
              }
            }
          }
        } else if (SOP && valid == 64u) {
          if (ATLS_CHACHA_DBG & 2) acc.l[0] ^= P[0] ^ P[5] ^ P[10] ^ P[15];  // timing build: no MAC (wrong tags)
          else p_sop4(acc, base == 0, r64, P, r, rsq, rcu);  // seal: the MAC over the ciphertext just written
          sop = true;
        } else {
          fold(P);  // seal: the MAC runs over the ciphertext just written
        }
      } else {
        uint32_t Z[16];
#pragma unroll
        for (int q = 0; q < 16; q++) Z[q] = 0;
        fold(Z);
      }
    }
    if (sop) {
      // acc already holds this slot (p_sop4)
    } else if (j == jL) {
      innerL = inner;  // ref = Q-1: contributes inner * r^1
    } else {
      if (base) acc = p_mul(acc, r64);  // r^(4G) = r^64; a lane's first slot is in the first step
      p_add(acc, inner);
    }
    (void)cnt;
  }

  flush();
  stage_flush();
  if (G == 64) LAT_STAMP(5, gl == 0);  // slots: XOR, stores issued, slot MACs

  // Lane partial: acc covers refs up to its last folded slot jf; contribution acc * r^(Q - ref).
  P130 contrib = p_zero();
  {
    const uint32_t l = (uint32_t)gl;
    if (jL >= 1 && l <= jL - 1) {
      const uint32_t jf = l + ((jL - 1 - l) / G) * G;
      const uint32_t ref = (jf == 0) ? na - 1u : na + 4u * jf - 1u;
      const uint32_t e = Q - ref;  // 1..4G+1
      // r^e = r^(e mod 4) * (r^4)^(e >> 2); (r^4)^u is lane u-1's R (G = 256: lane (u-1) mod 64's R of
      // any wave times r^(256 ((u-1) >> 6)))
      const uint32_t u = e >> 2, c = e & 3u;
      P130 ru;
      if constexpr (G > 64) {
        const uint32_t ix = u ? u - 1u : 0u, wq = ix >> 6;
        ru = shfl_p<64>(R, (int)(ix & 63u));
        if (wq) ru = p_mul(ru, wq == 1u ? r256 : wq == 2u ? r512 : r768);
      } else {
        ru = shfl_p<G>(R, (int)(u ? u - 1u : 0u));
      }
      if (u == 0) { ru = p_zero(); ru.l[0] = 1; }
      P130 pw;
      if (c == 0) pw = ru;
      else {
        if (LATE) {  // r^2, r^3 again here rather than live through the slot loop
          rsq = p_mul(r, r);
          rcu = p_mul(rsq, r);
        }
        pw = p_mul(ru, c == 1 ? r : c == 2 ? rsq : rcu);
      }
      if (!(jf == 0 && na == 0)) contrib = (ATLS_CHACHA_DBG & 16) ? acc : p_mul(acc, pw);
    }
    if (l == jL % G) p_add(contrib, (ATLS_CHACHA_DBG & 16) ? innerL : p_mul(innerL, r));
  }
  for (int off = GW / 2; off >= 1; off >>= 1) {
    P130 o = p_zero();
    for (int i = 0; i < 5; i++) o.l[i] = __shfl_xor(contrib.l[i], off, GW);
    p_add(contrib, o);
  }
  if constexpr (G > 64) {  // the waves' partial sums (and content-type maxima) meet in LDS
    if (OPEN) {
      for (int off = 32; off >= 1; off >>= 1) {
        lastnz = max(lastnz, (uint32_t)__shfl_xor((int)lastnz, off, 64));
      }
    }
    __shared__ uint32_t xc[G / 64][5];
    __shared__ uint32_t xl[G / 64];
    p_carry(contrib);  // limbs < 2^26 again, so four partials add without overflow
    if ((gl & 63) == 0) {
#pragma unroll
      for (int i = 0; i < 5; i++) xc[gl >> 6][i] = contrib.l[i];
      xl[gl >> 6] = lastnz;
    }
    __syncthreads();
    if (gl == 0) {
#pragma unroll
      for (int w = 1; w < G / 64; w++) {
#pragma unroll
        for (int i = 0; i < 5; i++) contrib.l[i] += xc[w][i];
        lastnz = xl[w] > lastnz ? xl[w] : lastnz;
      }
    }
  }
  uint32_t tag[4];
  if (ATLS_CHACHA_DBG & 32) {  // timing build: no tag finish
    tag[0] = contrib.l[0] ^ sk[0]; tag[1] = contrib.l[1] ^ sk[1]; tag[2] = contrib.l[2] ^ sk[2]; tag[3] = contrib.l[3] ^ sk[3];
  } else {
    p_finish(contrib, sk, tag);
  }
  if (G == 64) LAT_STAMP(6, gl == 0);  // lane combine, reduction, tag

  if (!OPEN) {
    if (gl == 0) {
      const uint4 t = make_uint4(tag[0], tag[1], tag[2], tag[3]);
      if (A.tags_out) st16(A.tags_out + 16ull * rec_idx, t);
      if (wire) {  // header || ciphertext || tag (record.rs:175-197)
        uint8_t* h = dst - 5;
        h[0] = (uint8_t)hdr0; h[1] = (uint8_t)(hdr0 >> 8); h[2] = (uint8_t)(hdr0 >> 16);
        h[3] = (uint8_t)(hdr0 >> 24); h[4] = (uint8_t)hdr1;
        st16(dst + n, t);
      }
    }
  } else {
    if (G <= 64) {
      for (int off = G / 2; off >= 1; off >>= 1) {
        lastnz = max(lastnz, (uint32_t)__shfl_xor((int)lastnz, off, G));
      }
    }
    if (gl == 0) {
      const uint4 tg = ld16(wire ? src + len : A.tags_in + 16ull * rec_idx);  // WIRE: tag follows the ct
      const bool ok = (tg.x == tag[0]) & (tg.y == tag[1]) & (tg.z == tag[2]) & (tg.w == tag[3]);
      atls_open_result rr;
      rr.reserved[0] = rr.reserved[1] = 0;
      if (!hdr_ok) {  // WIRE: the header does not frame this record (record.rs:81-102)
        rr.status = ATLS_DECODE_ERROR;
        rr.content_len = 0;
        rr.content_type = 0;
      } else if (!tls) {
        rr.status = ok ? ATLS_OK : ATLS_BAD_RECORD_MAC;
        rr.content_len = len;
        rr.content_type = 0;
      } else if (!ok) {
        rr.status = ATLS_DECRYPT_ERROR;
        rr.content_len = 0;
        rr.content_type = 0;
      } else {
        const uint32_t ty = lastnz & 0xffu;
        const bool vt = ty == 0 || ty == 20 || ty == 21 || ty == 22 || ty == 23;
        rr.status = vt ? ATLS_OK : ATLS_DECODE_ERROR;
        rr.content_len = (vt && lastnz) ? (lastnz >> 8) - 1u : 0u;
        rr.content_type = vt ? (uint8_t)ty : 0;
      }
      A.res[rec_idx] = rr;
    }
  }
}

// One group of G lanes seals / opens the record at work-list position q (direct batches: the
// kernel validates the descriptor itself).
template <bool OPEN, int G, bool LATE, bool CARRY = false, int PRE = G >= 64 ? 1 : 0, bool STAGE = false>
__device__ __forceinline__ void chacha_group(const ChArgs& A, const WorkList& W, uint32_t q, uint32_t cnt, int gl,
                                             lds_uint4* lds = nullptr) {
  if (q >= cnt) return;
  const uint32_t r = W.record(q);
  const atls_rec d = A.recs[r];
  const uint32_t st = A.idx ? 0u : direct_reject(d, A.ks, A.n_slots, OPEN);  // direct mode
  if (st) {
    if (gl == 0) {
      atomicOr(A.err, 1u);
      if (OPEN) {
        atls_open_result rr = {0, (uint8_t)st, 0, {0, 0}};
        A.res[r] = rr;
      }
    }
  } else {
    chacha_record<OPEN, G, LATE, CARRY, PRE, STAGE>(A, d, A.ks + d.key_slot, r, gl, lds);
  }
}

// G = 16: the waves take the work list (plan.hip, longest first; or the batch itself)
// round-robin, 4 consecutive positions per wave and step, one per 16-lane group.
// G = 4 (batches whose records are all short, ATLS_CHACHA_SHORT): 16 positions per wave and step,
// one per 4-lane group: the per-record Poly1305 set-up (r powers, lane scan, combine) is shared
// by 4 lanes instead of 16, and a 1.5 KiB record's 26 ChaCha blocks fill 28 lane-slots instead
// of 32 (C3: 690 -> 906 GiB/s). Direct batches: a wave takes 32 consecutive positions per step
// and picks the width from their longest record -- 2 lanes each if all are tiny (ATLS_CHACHA_TINY),
// 4 lanes in two rounds of 16 records if all are short, else 16 lanes in eight rounds of 4 records
// -- so no pass over the batch precedes the launch (an earlier version ran a
// batch_prep kernel for the batch's longest record and launched one kernel per width: two extra
// dispatches, ≈10 µs of every C3 batch). Planned batches (mixed lengths, longest first) run
// G = 16, 4 positions per wave and step, keeping the fine round-robin the longest-first order
// needs for balance.
// Minimum waves per SIMD of the seal / open kernels (__launch_bounds__): caps their VGPRs
// (3 -> 168, 4 -> 128), i.e. how many waves of each a SIMD holds.
#ifndef ATLS_CHACHA_MINW_SEAL
#define ATLS_CHACHA_MINW_SEAL 3  // the 2-lane path took the seal kernel to 171 VGPRs (2 waves per SIMD); capped
                                 // at 168 (1 spill): C3 0.0868 -> 0.0864 ms (profiles/r02/ab_chacha_tiny.log)
#endif
#ifndef ATLS_CHACHA_MINW_OPEN
#define ATLS_CHACHA_MINW_OPEN 3  // 169 -> 168 VGPRs: 3 open waves per SIMD instead of 2 (C3 open 0.113 -> 0.106 ms)
#endif
// Planned (mixed-suite) batches run the ChaCha kernel beside the AES-GCM kernel, whose workgroup
// holds 3 waves x 128 VGPRs per SIMD: at <= 128 VGPRs a ChaCha wave still fits next to it, so the
// LDS-bound and the VALU-bound kernel share every CU (C5 658-670 -> 705-712 GiB/s, same-box A/B;
// the direct C3 batch loses 19 % at that register cap and keeps the bounds above).
#ifndef ATLS_CHACHA_MINW_SIDE
#define ATLS_CHACHA_MINW_SIDE 4
#endif
#ifndef ATLS_CHACHA_MINW_SIDE_OPEN
#define ATLS_CHACHA_MINW_SIDE_OPEN ATLS_CHACHA_MINW_SIDE
#endif
#ifndef ATLS_CHACHA_PLANNED_EARLY
#define ATLS_CHACHA_PLANNED_EARLY 0  // 1: planned seals keep r^2, r^3 live and fold full slots by SOP -- 31
                                     // spilled VGPRs at the 128 cap, C5 seal 0.327 -> 0.349 ms (ab_c35_early.log)
#endif
#ifndef ATLS_CHACHA_PLANNED_PRE
#define ATLS_CHACHA_PLANNED_PRE 0  // 2: planned batches prefetch a step ahead with early powers (180 VGPRs, so
                                   // MINW_SIDE 2 or 3): C5 seal 0.325 -> 0.334 ms, open 0.310 -> 0.329 ms
                                   // (profiles/r03/ab_c5_planned_pf.log); off
#endif
#ifndef ATLS_CHACHA_PLANNED_G
#define ATLS_CHACHA_PLANNED_G 16  // lanes per record in planned (mixed) batches; C5 0.341 ms at 16, 0.359 at
                                  // 8, 0.435 at 4 (profiles/r02/ab_chacha_planned_g.log)
#endif
template <bool OPEN, int G>
__device__ __forceinline__ void chacha_batch(const ChArgs& A, int lane) {
  const WorkList W{A.idx, A.plan, kListChacha, A.n};
  const uint32_t cnt = W.size();
  constexpr uint32_t kPer = 64u / G;
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) / 64u;
  const uint32_t stride = gridDim.x * blockDim.x / 64u * kPer;
  for (uint32_t q0 = wave * kPer; q0 < cnt; q0 += stride)
    chacha_group<OPEN, G, (ATLS_CHACHA_PLANNED_EARLY | ATLS_CHACHA_PLANNED_PRE) == 0, false, ATLS_CHACHA_PLANNED_PRE>(
        A, W, q0 + (uint32_t)lane / (uint32_t)G, cnt, lane & (G - 1));
}

// Records up to ATLS_CHACHA_TINY bytes (every record of a wave step) take ATLS_CHACHA_TINY_G
// lanes each: a direct batch's wave step then covers 64 / TINY_G positions (0: off, 16 per step).
// At 2 lanes an MTU-sized record's Poly1305 set-up (r powers, a one-level lane scan, combine) is
// shared by 2 lanes instead of 4 and its 26 ChaCha blocks fill 26 lane-slots instead of 28; a
// 64 Ki-record batch still gives 2 waves per SIMD. Same-box A/B, 3 rounds
// (profiles/r02/ab_chacha_tiny.log): C3 seal kernel 0.0895 ms (4 lanes) -> 0.0864 ms (2 lanes,
// -3.5 %); 1 lane per record (one wave per SIMD) 0.0982 ms; opens and C5 unchanged.
#ifndef ATLS_CHACHA_TINY
#define ATLS_CHACHA_TINY 2048
#endif
#ifndef ATLS_CHACHA_TINY_G
#define ATLS_CHACHA_TINY_G 2
#endif

// CARRY on seals: C3 seal traffic 1.28x -> 1.11x of the algorithmic bytes but the kernel 0.0873 ->
// 0.0905 ms (+3.7 %; 2 more spilled VGPRs); opens 0.1023 -> 0.1004 ms with traffic 1.47x -> 1.29x
// (profiles/r03/ab_chacha_carry.log). The seal kernel is not HBM-bound, so carry stays on opens only.
// Re-measured on the SOP seal kernel (profiles/r03/ab_c3_carry_seal_sop.log): traffic 1.31x -> 1.16x,
// kernel 0.0851 -> 0.0892 ms (+4.8 %); still off.
#ifndef ATLS_CHACHA_CARRY_SEAL
#define ATLS_CHACHA_CARRY_SEAL 0
#endif
#ifndef ATLS_CHACHA_CARRY_OPEN
#define ATLS_CHACHA_CARRY_OPEN 1
#endif
#ifndef ATLS_CHACHA_W2_CARRY_OPEN
#define ATLS_CHACHA_W2_CARRY_OPEN 0  // the 2-wave kernel's opens without the carry: C3 open 0.0896 -> 0.0849 ms
                                     // (traffic 1.17x -> 1.33x; profiles/r03/ab_c3_open2.log)
#endif

#ifndef ATLS_CHACHA_W2
#define ATLS_CHACHA_W2 1
#endif
#ifndef ATLS_CHACHA_STAGE
#define ATLS_CHACHA_STAGE 0  // 1: whole-line transposed stores through LDS in the 2-wave seal kernel (A/B, chacha_record STAGE)
#endif
#ifndef ATLS_CHACHA_W2_PRE
#define ATLS_CHACHA_W2_PRE 2  // 1: load a slot's data at the top of its step; 2: one step ahead (C3 open 0.0962 ->
                              // 0.0926 ms, seal 0.0834 -> 0.0806 ms: profiles/r03/ab_c3_pf.log)
#endif
#ifndef ATLS_CHACHA_W2_SEAL
#define ATLS_CHACHA_W2_SEAL 1  // seals take the 2-wave kernel too (with the prefetch; with PRE = 1 they measured 3 % slower)
#endif
#ifndef ATLS_CHACHA_W2_EARLY
#define ATLS_CHACHA_W2_EARLY 1  // the 2-wave kernel keeps r^2, r^3 live (not LATE), so its opens fold by SOP too:
                                // C3 open 0.1015 -> 0.0977 ms (profiles/r03/ab_c35_early.log)
#endif

// Direct batch: P positions per wave and step, the width chosen per step from their longest record.
template <bool OPEN, int PRE = 0>
__device__ __forceinline__ void chacha_direct(const ChArgs& A, int lane) {
  constexpr bool LATE = OPEN && !(PRE && ATLS_CHACHA_W2_EARLY);
  __shared__ v4u32_ch carry[256 * 4];  // CARRY: 4 pieces of 16 B per lane (16 KiB per workgroup)
  lds_uint4* lds = (lds_uint4*)(carry) + 4u * threadIdx.x;
  const WorkList W{nullptr, nullptr, kListChacha, A.n};
  const uint32_t cnt = A.n;
  constexpr uint32_t P = ATLS_CHACHA_TINY ? 64u / ATLS_CHACHA_TINY_G : 16u;
  static_assert(P >= 16 && P <= 64, "a wave step covers 16 to 64 positions");
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) / 64u;
  const uint32_t stride = gridDim.x * blockDim.x / 64u * P;
  for (uint32_t q0 = wave * P; q0 < cnt; q0 += stride) {
    uint32_t mx = ((uint32_t)lane < P && q0 + (uint32_t)lane < cnt) ? A.recs[q0 + (uint32_t)lane].len : 0u;
#pragma unroll
    for (int off = (int)P / 2; off >= 1; off >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, off, 64));
    mx = (uint32_t)__builtin_amdgcn_readfirstlane((int)mx);
    if (ATLS_CHACHA_DBG & 128) {  // timing build: the launch floor (no record is processed)
      if (mx == 0xffffffffu) A.err[0] = 1u;  // keeps the length reads
      continue;
    }
    if (ATLS_CHACHA_STAGE && !OPEN && PRE >= 2 && ATLS_CHACHA_TINY && mx <= (uint32_t)ATLS_CHACHA_TINY &&
        q0 + P <= cnt) {
      // STAGE needs every lane in the same steps: a full wave step of TLS / RAW records of one length,
      // none refused (else the unstaged path below)
      uint32_t mn = 0xffffffffu, ok = 1u;
      if ((uint32_t)lane < P) {
        const atls_rec d = A.recs[q0 + (uint32_t)lane];
        mn = d.len;
        ok = (d.mode != ATLS_MODE_WIRE && d.mode == A.recs[q0].mode && !direct_reject(d, A.ks, A.n_slots, OPEN)) ? 1u : 0u;
      }
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) {
        mn = min(mn, (uint32_t)__shfl_xor((int)mn, off, 64));
        ok &= (uint32_t)__shfl_xor((int)ok, off, 64);
      }
      if (__builtin_amdgcn_readfirstlane((int)(ok && mn == mx))) {
        constexpr int G = ATLS_CHACHA_TINY_G;
        chacha_group<OPEN, G, LATE, false, PRE, true>(A, W, q0 + (uint32_t)lane / (uint32_t)G, cnt, lane & (G - 1), lds);
        continue;
      }
    }
    if (ATLS_CHACHA_TINY && mx <= (uint32_t)ATLS_CHACHA_TINY) {
      constexpr int G = ATLS_CHACHA_TINY ? ATLS_CHACHA_TINY_G : 4;
      chacha_group<OPEN, G, LATE, (OPEN ? (PRE >= 2 ? ATLS_CHACHA_W2_CARRY_OPEN : ATLS_CHACHA_CARRY_OPEN) : ATLS_CHACHA_CARRY_SEAL), PRE>(A, W, q0 + (uint32_t)lane / (uint32_t)G, cnt, lane & (G - 1), lds);
    } else if (mx <= (uint32_t)ATLS_CHACHA_SHORT) {
#pragma unroll 1
      for (uint32_t rr = 0; rr < P / 16u; rr++) chacha_group<OPEN, 4, LATE, (OPEN ? (PRE >= 2 ? ATLS_CHACHA_W2_CARRY_OPEN : ATLS_CHACHA_CARRY_OPEN) : ATLS_CHACHA_CARRY_SEAL), PRE>(A, W, q0 + 16u * rr + (uint32_t)lane / 4u, cnt, lane & 3, lds);
    } else {
#pragma unroll 1
      for (uint32_t rr = 0; rr < P / 4u; rr++) chacha_group<OPEN, 16, LATE, (OPEN ? (PRE >= 2 ? ATLS_CHACHA_W2_CARRY_OPEN : ATLS_CHACHA_CARRY_OPEN) : ATLS_CHACHA_CARRY_SEAL), PRE>(A, W, q0 + 4u * rr + (uint32_t)lane / 16u, cnt, lane & 15, lds);
    }
  }
}

template <bool OPEN, bool PLANNED>
__global__ __launch_bounds__(256, PLANNED ? (OPEN ? ATLS_CHACHA_MINW_SIDE_OPEN : ATLS_CHACHA_MINW_SIDE) : OPEN ? ATLS_CHACHA_MINW_OPEN : ATLS_CHACHA_MINW_SEAL) void chacha_kernel(ChArgs A) {
  const int lane = threadIdx.x & 63;
  if constexpr (PLANNED) chacha_batch<OPEN, ATLS_CHACHA_PLANNED_G>(A, lane);
  else chacha_direct<OPEN>(A, lane);
}

// Direct batches that give at most two waves per SIMD (C3: 65,536 MTU-sized records = 2,048 waves of 32
// records on 1,024 SIMDs) lose nothing to a 2-wave register bound, and 256 VGPRs let each lane load its
// next slot's data a step ahead (PRE == 2) and keep r^2, r^3 live for SOP without spilling. The C3
// kernels' waves sat at s_waitcnt a quarter of their cycles (profiles/r03/c3_pmc_stall_*.csv). Same-box
// A/Bs over 3 rounds: C3 open 0.1016 -> 0.0977 ms (data at the top of the step, SOP;
// profiles/r03/ab_c3_w2.log, ab_c35_early.log) -> 0.0926 ms (a step ahead, ab_c3_pf.log); C3 seal 0.0834
// (3-wave kernel, SOP) -> 0.0806 ms (2-wave kernel, a step ahead) -- loading at the top of the same step
// had made seals 3 % slower: the wait for that block also waited for the previous step's stores.
template <bool OPEN>
__global__ __launch_bounds__(256, 2) void chacha_kernel_w2(ChArgs A) {
  chacha_direct<OPEN, ATLS_CHACHA_W2_PRE>(A, threadIdx.x & 63);
}

// Latency path for a few records (the Cipher-trait single call, record.rs:191-193): one record per
// wave at 64 lanes, so a 1.5 KiB record's 26 ChaCha blocks run side by side instead of 13 deep at
// 2 lanes (the per-record Poly1305 scan is 6 levels instead of 1; throughput is not the point).
#ifndef ATLS_CHACHA_LAT_MAX
#define ATLS_CHACHA_LAT_MAX 32  // direct batches of at most this many records
#endif
template <bool OPEN>
__global__ __launch_bounds__(64) void chacha_kernel_lat(ChArgs A) {
  const WorkList W{nullptr, nullptr, kListChacha, A.n};
  chacha_group<OPEN, 64, false>(A, W, blockIdx.x, A.n, (int)(threadIdx.x & 63));
  if (A.done && A.n == 1u) {  // the single call's completion flag, after every store of the record
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // MI355X_MICROARCH.md: the compiler may drop it
    if ((threadIdx.x & 63) == 0) __hip_atomic_store(A.done, A.done_val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// The single call with its descriptor, IV || AAD, input and received tag in the launch's argument block
// (kSingleInline bytes at most): the wave starts with everything but the key schedule (device memory)
// at hand, where chacha_kernel_lat reads the descriptor from mapped host memory first and the key slot,
// nonce / AAD and data after it -- dependent PCIe round trips before the first ChaCha round. Outputs,
// tag, open result and the completion flag still go to the caller's mapped pinned block.
struct ChSingle {
  ChArgs A;
  atls_rec d;          // in_off / aux_off relative to bytes
  uint32_t tag_off;    // open: the received tag at bytes + tag_off
  uint32_t pad[3];
  uint8_t bytes[kSingleInline];
};
template <bool OPEN>
__global__ __launch_bounds__(kChSingleThreads) void chacha_single(ChSingle) {
  // the argument block itself (the only explicit argument, at offset 0), read in place: naming the
  // by-value parameter's members by address would copy all of it to scratch first
  const ChSingle* S = (const ChSingle*)__builtin_amdgcn_kernarg_segment_ptr();
  ChArgs A = S->A;
  A.recs = &S->d;
  A.in = S->bytes;
  A.aux = S->bytes;
  if (OPEN) A.tags_in = S->bytes + S->tag_off;
  const WorkList W{nullptr, nullptr, kListChacha, 1u};
#ifdef ATLS_LAT_STAMPS
  if (threadIdx.x == 0) {
    atomicAdd(&g_lat_stamps[8], (unsigned long long)__builtin_amdgcn_s_memrealtime());
    atomicAdd(&g_lat_stamps[15], 1ull);
  }
  LAT_STAMP(0, threadIdx.x == 0);
#endif
  chacha_group<OPEN, kChSingleThreads, false>(A, W, 0u, 1u, (int)threadIdx.x);  // one record on all the waves
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // every wave's stores have left
#ifdef ATLS_LAT_STAMPS
  LAT_STAMP(7, threadIdx.x == 0);  // outputs written to the caller's mapped memory
  if (threadIdx.x == 0) atomicAdd(&g_lat_stamps[9], (unsigned long long)__builtin_amdgcn_s_memrealtime());
#endif
  if (threadIdx.x == 0) __hip_atomic_store(A.done, A.done_val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}


// q4_record with the record's bytes and its output passing through LDS in 16-byte pieces: its 4-byte and byte
// accesses straight to mapped host memory would each be a PCIe transaction (the resident server's request and
// reply live there: 20.8 us per 1,537-B call that way). in: IV || AAD || input (|| tag), read 16 B at a time
// (d.in_off / aux_off / tag_off index it); out + d.out_off (16-byte aligned) receives the output.
template <bool OPEN>
__device__ __forceinline__ void q4_staged(const KeySched* k, const atls_rec& d, const uint8_t* in, uint32_t tag_off,
                                          uint8_t* out, uint8_t* tag_out, atls_open_result* res) {
  __shared__ uint4 stage_in[kSingleInline / 16], stage_out[kSingleInline / 16];
  __shared__ Q4Lds q4l;
  const uint32_t t = threadIdx.x;
  const uint32_t nin = (tag_off + (OPEN ? 16u : 0u) + 15u) / 16u, nout = (d.len + 15u) / 16u;  // <= 224 each
  for (uint32_t i = t; i < nin; i += 256u) stage_in[i] = ld16(in + 16u * i);
  __syncthreads();
  atls_rec dl = d;
  dl.out_off = 0;
  q4_record<OPEN>(k, dl, (const uint8_t*)stage_in, tag_off, (uint8_t*)stage_out, tag_out, res, q4l);
  __syncthreads();  // the output is whole in LDS
  for (uint32_t i = t; i < nout; i += 256u) st16(out + d.out_off + 16u * i, stage_out[i]);
}

template <bool OPEN>
__global__ __launch_bounds__(256) void chacha_single_q4(ChSingle) {
  const ChSingle* S = (const ChSingle*)__builtin_amdgcn_kernarg_segment_ptr();
  const ChArgs& A = S->A;
  q4_staged<OPEN>(A.ks + S->d.key_slot, S->d, S->bytes, S->tag_off, A.out, A.tags_out, A.res);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // every wave's stores have left
  if (threadIdx.x == 0) __hip_atomic_store(A.done, A.done_val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <bool OPEN>
__global__ __launch_bounds__(256) void chacha_single_ptr(ChArgs A) {
  const WorkList W{nullptr, nullptr, kListChacha, 1u};
  chacha_group<OPEN, 256, false>(A, W, 0u, 1u, (int)threadIdx.x);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(A.done, A.done_val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace atls

extern "C" unsigned atls_chacha_dbg(void) {
#ifdef ATLS_LAT_STAMPS
  return ATLS_CHACHA_DBG | 0x100u;  // a timing build (reported by atls_build_flags)
#else
  return ATLS_CHACHA_DBG;
#endif
}

// Debug: copy out (and reset) the single call's phase clocks of a -DATLS_LAT_STAMPS build; -1 otherwise.
extern "C" int atls_debug_lat_stamps(unsigned long long* out) {
#ifdef ATLS_LAT_STAMPS
  unsigned long long h[16], z[16] = {};
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(atls::g_lat_stamps), sizeof(h)) != hipSuccess) return -1;
  if (hipMemcpyToSymbol(HIP_SYMBOL(atls::g_lat_stamps), z, sizeof(z)) != hipSuccess) return -1;
  for (int i = 0; i < 16; i++) out[i] = h[i];
  return 0;
#else
  (void)out;
  return -1;
#endif
}

// One RAW record (the Cipher-trait single call) from the argument block: d's in_off / aux_off index
// `bytes` (nbytes <= kSingleInline, IV || AAD || input || tag), outputs at out + d.out_off, tags_out,
// res; done is set to done_val once they are visible.
extern "C" int atls_launch_chacha_single(int open, const void* ks, uint32_t n_slots, const atls_rec* d,
                                         const uint8_t* bytes, uint32_t nbytes, uint32_t tag_off, uint8_t* out,
                                         uint8_t* tags_out, atls_open_result* res, uint32_t* err, uint32_t* done,
                                         uint32_t done_val, hipStream_t s) {
  if (nbytes > atls::kSingleInline || !done) return ATLS_INTERNAL_ERROR;
  atls::ChSingle S;
  S.A = atls::ChArgs{(const atls::KeySched*)ks, nullptr, 1u, nullptr, nullptr, out, tags_out, nullptr, res, nullptr,
                     nullptr, err, n_slots, done, done_val};
  S.d = *d;
  S.tag_off = tag_off;
  __builtin_memcpy(S.bytes, bytes, nbytes);
  const uint32_t Q = (d->aad_len + 15u) / 16u + (d->len + 15u) / 16u + 1u;
  if (ATLS_CHACHA_SINGLE_Q4 && d->mode == ATLS_MODE_RAW && d->iv_len == 12 && Q <= 256u && (d->len + 63u) / 64u <= 63u) {
    if (open) hipLaunchKernelGGL((atls::chacha_single_q4<true>), dim3(1), dim3(256), 0, s, S);
    else hipLaunchKernelGGL((atls::chacha_single_q4<false>), dim3(1), dim3(256), 0, s, S);
  } else if (open) {
    hipLaunchKernelGGL((atls::chacha_single<true>), dim3(1), dim3(atls::kChSingleThreads), 0, s, S);
  } else {
    hipLaunchKernelGGL((atls::chacha_single<false>), dim3(1), dim3(atls::kChSingleThreads), 0, s, S);
  }
  return hipGetLastError() == hipSuccess ? 0 : ATLS_INTERNAL_ERROR;
}


// idx / plan: the batch plan's work lists (G = 16), or nullptr for a direct batch (per-step widths).
extern "C" int atls_launch_chacha(int open, const void* ks, const atls_rec* recs, uint32_t n, const uint8_t* in,
                                  const uint8_t* aux, uint8_t* out, uint8_t* tags_out, const uint8_t* tags_in,
                                  atls_open_result* res, const uint32_t* idx, void* plan, uint32_t* err,
                                  uint32_t n_slots, int grid, hipStream_t s, uint32_t* done, uint32_t done_val,
                                  int cus) {
  if (n == 0) return 0;
  atls::ChArgs A{(const atls::KeySched*)ks, recs, n, in, aux, out, tags_out, tags_in, res, idx,
                 (atls::PlanHdr*)plan, err, n_slots, n == 1 ? done : nullptr, done_val};
  // the grid of the wider need (4 waves x 4 positions per workgroup at G = 16); the G = 4 path
  // strides over 16 positions per wave and simply finishes its list sooner
  const uint32_t want16 = (n + 15u) / 16u;
  const uint32_t g = (uint32_t)grid < want16 ? (uint32_t)grid : want16;
  if (ATLS_CHACHA_SINGLE_4W && !idx && n == 1 && done) {  // the single call's longer records: 4 waves
    if (open) hipLaunchKernelGGL((atls::chacha_single_ptr<true>), dim3(1), dim3(256), 0, s, A);
    else hipLaunchKernelGGL((atls::chacha_single_ptr<false>), dim3(1), dim3(256), 0, s, A);
  } else if (!idx && n <= (uint32_t)ATLS_CHACHA_LAT_MAX) {
    if (open) hipLaunchKernelGGL((atls::chacha_kernel_lat<true>), dim3(n), dim3(64), 0, s, A);
    else hipLaunchKernelGGL((atls::chacha_kernel_lat<false>), dim3(n), dim3(64), 0, s, A);
  } else if (idx) {
    if (open) hipLaunchKernelGGL((atls::chacha_kernel<true, true>), dim3(g), dim3(256), 0, s, A);
    else hipLaunchKernelGGL((atls::chacha_kernel<false, true>), dim3(g), dim3(256), 0, s, A);
  } else if (ATLS_CHACHA_W2 && (open || ATLS_CHACHA_W2_SEAL) && cus > 0 && (n + 31u) / 32u <= 8u * (uint32_t)cus) {
    // a wave step covers 32 positions: at most 2 waves per SIMD of work (chacha_kernel_w2)
    if (open) hipLaunchKernelGGL((atls::chacha_kernel_w2<true>), dim3(g), dim3(256), 0, s, A);
    else hipLaunchKernelGGL((atls::chacha_kernel_w2<false>), dim3(g), dim3(256), 0, s, A);
  } else {
    if (open) hipLaunchKernelGGL((atls::chacha_kernel<true, false>), dim3(g), dim3(256), 0, s, A);
    else hipLaunchKernelGGL((atls::chacha_kernel<false, false>), dim3(g), dim3(256), 0, s, A);
  }
  return hipGetLastError() == hipSuccess ? 0 : ATLS_INTERNAL_ERROR;
}
