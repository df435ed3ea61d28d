// Device key setup: one wavefront per key slot (a connection's write key). Everything the record
// kernels need per key is computed here once, instead of per record as the reference does
// (gcm.rs:52-56 re-expands the key and recomputes H on every call):
//   * AES round keys (crypto/aes/cipher.rs:216-249) as raw words for the T-table rounds, and their rotl16;
//   * H = E_K(0^128) (gcm.rs:56), H^1..H^64 (lane-combine multipliers), and
//     x^(4p)*H^64 and x^(4p)*H^(8<<t), t = 0..2, for p = 0..31 (seeds of the 4-bit GHASH tables);
//   * ChaCha20 key words (chacha20/cipher.rs:29-31) and the static IV (key_schedule.rs:34).
// Also builds the 256-entry AES T-table T0 used (replicated per LDS bank) by gcm.hip.
//
// Round 4: the first version ran one serial thread per key -- a private byte array AES
// and 64 + 128 bit-serial products -- and took 0.459 ms for C2's 4,096 keys. Now a wave owns a key:
//   * the key expansion and E_K(0) are wave-uniform T-table work on an LDS copy of T0 (unrolled per key
//     size, so the round keys stay in registers);
//   * H^1..H^64 come from a 6-level doubling scan -- at level k lanes [2^k, 2^(k+1)) multiply the
//     power 2^k lanes below by H^(2^k), one factor for the whole wave -- each product by a 4-bit table of
//     that factor built in the wave's LDS (gcm_common.h ghash_table_entries / ghash_mul_tab, the record
//     kernels' own GHASH machinery: 32 lookups per product instead of a 128-step bit-serial loop);
//   * every table seed x^k * Y is one shift and one reduction (gcm_common.h gf_mulxk), so the 32 seeds of a table
//     and the 128 record-table seeds are computed by all lanes at once.
#include "aes_sbox.h"
#include "gcm_common.h"

namespace atls {

// T0[x] = {2S, S, S, 3S} little-endian: MixColumns column of S[x] entering at row 0.
__device__ __forceinline__ uint32_t t0_entry(int x) {
  const uint8_t s = kSbox[x], s2 = xtime(s), s3 = (uint8_t)(s2 ^ s);
  return (uint32_t)s2 | ((uint32_t)s << 8) | ((uint32_t)s << 16) | ((uint32_t)s3 << 24);
}

__global__ void build_t0_kernel(uint32_t* __restrict__ t0) { t0[threadIdx.x] = t0_entry((int)threadIdx.x); }

// The wave's 4-bit table of the wave-uniform factor y (be words) at LDS byte address wb: lane l writes
// entries 8 (l & 1) .. +7 of position l >> 1 from the seed x^(4p) * y (gcm_common.h layout).
__device__ __forceinline__ void table_of(uint32_t wb, const uint32_t (&y)[4], int lane) {
  const int p = lane >> 1;
  uint32_t seed[4] = {y[0], y[1], y[2], y[3]};
  gf_mulxk(seed, 4u * (uint32_t)p);
  ghash_table_entries<8>(wb, seed, p, (lane & 1) * 8);
}

// x <- x * (the table's factor), be words in and out.
__device__ __forceinline__ void table_mul(uint32_t (&x)[4], uint32_t wb) {
  uint32_t r[4] = {bswap32(x[0]), bswap32(x[1]), bswap32(x[2]), bswap32(x[3])};
  ghash_mul_tab(r, wb);
  for (int w = 0; w < 4; w++) x[w] = bswap32(r[w]);
}

__device__ __forceinline__ uint32_t sbox_lds(const uint32_t* t0, uint32_t x) { return (t0[x & 255u] >> 8) & 0xffu; }
__device__ __forceinline__ uint32_t sub_word(const uint32_t* t0, uint32_t w) {
  return sbox_lds(t0, w) | (sbox_lds(t0, w >> 8) << 8) | (sbox_lds(t0, w >> 16) << 16) | (sbox_lds(t0, w >> 24) << 24);
}

// FIPS-197 key expansion (crypto/aes/cipher.rs:216-249) in raw little-endian words (word w = bytes 4w..4w+3
// of the expanded key), unrolled per key size so every round key lives in a register; then H = E_K(0^128)
// (gcm.rs:56) by T-table rounds (wave-uniform indices: LDS broadcasts). h_raw: H as raw words.
template <int NK>
__device__ __forceinline__ void expand_and_h(const uint32_t (&kw)[8], const uint32_t* t0, uint32_t (&rk)[60],
                                             uint32_t (&h_raw)[4]) {
  constexpr int NR = NK + 6, NW = 4 * (NR + 1);
  constexpr uint32_t kRcon[10] = {0x01, 0x02, 0x04, 0x08, 0x10, 0x20, 0x40, 0x80, 0x1B, 0x36};
#pragma unroll
  for (int w = 0; w < 60; w++) rk[w] = w < NK ? kw[w] : 0u;
#pragma unroll
  for (int w = NK; w < NW; w++) {
    uint32_t t = rk[w - 1];
    if (w % NK == 0) t = sub_word(t0, rotl32(t, 24)) ^ kRcon[w / NK - 1];  // RotWord = bytes (1,2,3,0)
    else if (NK > 6 && w % NK == 4) t = sub_word(t0, t);
    rk[w] = rk[w - NK] ^ t;
  }
  uint32_t s0 = rk[0], s1 = rk[1], s2 = rk[2], s3 = rk[3];  // AddRoundKey of the zero block
#pragma unroll
  for (int r = 1; r < NR; r++) {
    const uint32_t a0 = t0[s0 & 255u] ^ rotl32(t0[(s1 >> 8) & 255u], 8) ^ rotl32(t0[(s2 >> 16) & 255u], 16) ^
                        rotl32(t0[s3 >> 24], 24) ^ rk[4 * r];
    const uint32_t a1 = t0[s1 & 255u] ^ rotl32(t0[(s2 >> 8) & 255u], 8) ^ rotl32(t0[(s3 >> 16) & 255u], 16) ^
                        rotl32(t0[s0 >> 24], 24) ^ rk[4 * r + 1];
    const uint32_t a2 = t0[s2 & 255u] ^ rotl32(t0[(s3 >> 8) & 255u], 8) ^ rotl32(t0[(s0 >> 16) & 255u], 16) ^
                        rotl32(t0[s1 >> 24], 24) ^ rk[4 * r + 2];
    const uint32_t a3 = t0[s3 & 255u] ^ rotl32(t0[(s0 >> 8) & 255u], 8) ^ rotl32(t0[(s1 >> 16) & 255u], 16) ^
                        rotl32(t0[s2 >> 24], 24) ^ rk[4 * r + 3];
    s0 = a0; s1 = a1; s2 = a2; s3 = a3;
  }
  const uint32_t st[4] = {s0, s1, s2, s3};
#pragma unroll
  for (int c = 0; c < 4; c++)  // SubBytes + ShiftRows (row r from column c + r) + the last round key
    h_raw[c] = (sbox_lds(t0, st[c]) | (sbox_lds(t0, st[(c + 1) & 3] >> 8) << 8) |
                (sbox_lds(t0, st[(c + 2) & 3] >> 16) << 16) | (sbox_lds(t0, st[(c + 3) & 3] >> 24) << 24)) ^
               rk[4 * NR + c];
}

#ifndef ATLS_KS_ONE
#define ATLS_KS_ONE 1  // a single key takes key_setup_kernel<true> (squared factors, all tables at once)
#endif

// Up to kInlineKeys keys travel in the kernel arguments (a connection's new key: no staging copy).
constexpr int kInlineKeys = 4;
constexpr int kSetupWaves = 4;                 // keys per workgroup
constexpr uint32_t kSetupTab = 8192;           // one 4-bit table per wave
constexpr uint32_t kSetupT0 = kSetupWaves * kSetupTab;
constexpr int kOneTabs = 6;                    // ONE: the tables of H^(2^b), b = 0..5
constexpr uint32_t kOneT0 = kOneTabs * kSetupTab;
struct KeySetupArgs {
  const atls_key* keys;  // device array, or nullptr: the keys are in `inl`
  uint32_t n;
  KeySched* ks;
  const uint32_t* t0;    // the engine's T0 (gcm.hip's table, built at engine creation)
  uint32_t inl[kInlineKeys][16];
};
static_assert(sizeof(atls_key) == 64, "atls_key is 16 words");

// Phase clocks of a key install (timing build -DATLS_KS_STAMPS, tools/key_setup_stamps.py): lane 0 of wave
// 0 of key 0 adds the shader clock at each phase end (after its memory operations) to g_ks_stamps[i];
// [14] / [15] the 100 MHz real-time clock at entry / exit, [13] the launch count.
#ifdef ATLS_KS_STAMPS
__device__ unsigned long long g_ks_stamps[16];
#define KS_STAMP(i)                                                                          \
  do {                                                                                       \
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");                              \
    const uint64_t t_ = __builtin_amdgcn_s_memtime();                                        \
    if (i_key == 0 && threadIdx.x == 0) atomicAdd(&g_ks_stamps[i], (unsigned long long)t_);  \
  } while (0)
#else
#define KS_STAMP(i) do { } while (0)
#endif

// ONE (a single key: the latency of a connection's new key, the single call's cache miss; round 4,
// tools/key_setup_stamps.py, profiles/r04/key_setup_stamps.json): the per-wave scan spends ~1.1 us per level
// on a table build and a product (six levels). Here the factors H^(2^b) come from squarings (linear: a bit
// spread and one fold, no table), the four waves build all six factor tables at once (48 KiB), and lane l
// forms H^(l+1) as the product of the factors of l + 1's set bits -- six table products and no build
// between them. H^64 is the sixth square. The record-table seeds (x^(4p) * H^8 / H^16 / H^32 / H^64) need
// only the factors, so waves 1-3 write them while wave 0 forms the powers. (Base-4 digits -- two products
// per lane from tables of H^(j 4^k) -- measured slower: the H^3 they need took a comb multiply that cost
// more at one wave than the four products it saved.)
template <bool ONE>
__global__ __launch_bounds__(64 * kSetupWaves) void key_setup_kernel(KeySetupArgs A) {
  extern __shared__ __attribute__((aligned(256))) uint32_t smem[];
  const int wave = (int)uni(threadIdx.x >> 6), lane = (int)(threadIdx.x & 63);
  const uint32_t i = ONE ? 0u : blockIdx.x * kSetupWaves + (uint32_t)wave;
#ifdef ATLS_KS_STAMPS
  const uint32_t i_key = blockIdx.x;
  if (i_key == 0 && threadIdx.x == 0) {
    atomicAdd(&g_ks_stamps[14], (unsigned long long)__builtin_amdgcn_s_memrealtime());
    atomicAdd(&g_ks_stamps[13], 1ull);
  }
  KS_STAMP(0);
#endif
  uint32_t* t0 = smem + (ONE ? kOneT0 : kSetupT0) / 4;
  t0[threadIdx.x] = A.t0[threadIdx.x];  // one load per thread of a table the engine already holds
  __syncthreads();
  KS_STAMP(1);
  if (i >= A.n) return;
  const bool writer = !ONE || wave == 0;  // the wave that stores the key's per-slot fields
  // the key's 16 words (atls_key: suite | key_len | iv_len, key[32], static_iv[12], reserved)
  uint32_t k[16];
  if (A.keys) {
#pragma unroll
    for (int q = 0; q < 16; q++) k[q] = cptr(reinterpret_cast<const uint32_t*>(A.keys + i))[q];
  } else {
#pragma unroll
    for (int q = 0; q < 16; q++) k[q] = i == 0 ? A.inl[0][q] : i == 1 ? A.inl[1][q] : i == 2 ? A.inl[2][q] : A.inl[3][q];
  }
  const uint32_t suite = k[0] & 0xffffu, key_len = (k[0] >> 16) & 0xffu;
  KeySched* o = A.ks + i;
  uint32_t kw[8];
#pragma unroll
  for (int q = 0; q < 8; q++) kw[q] = k[1 + q];
  // ChaCha20 key words and the static IV for every slot (the GCM kernels read siv too): word q of each
  // from lane q (selects, no indexed register access)
  if (writer) {
    uint32_t kq = 0, sq = 0;
#pragma unroll
    for (int q = 0; q < 8; q++) kq = lane == q ? kw[q] : kq;
#pragma unroll
    for (int q = 0; q < 3; q++) sq = lane == q ? k[9 + q] : sq;
    if (lane < 8) o->kw[lane] = kq;
    if (lane < 4) o->siv[lane] = sq;
  }
  const bool aes = (suite == kSuiteAes128 || suite == kSuiteAes256) && (key_len == 16 || key_len == 24 || key_len == 32);
  if (!aes) {
    if (writer && lane == 0) {
      o->suite = suite;
      o->nr = 0;
      o->key_len = key_len;
      o->valid = (suite == kSuiteChacha && key_len == 32) ? 1u : 0u;
    }
    return;
  }
  KS_STAMP(2);
  uint32_t rk[60], h[4];
  if (key_len == 16) expand_and_h<4>(kw, t0, rk, h);
  else if (key_len == 24) expand_and_h<6>(kw, t0, rk, h);
  else expand_and_h<8>(kw, t0, rk, h);
  KS_STAMP(3);
  const uint32_t nr = key_len / 4 + 6;
  if (writer) {  // round key w from lane w (one coalesced store each for rk and rkr)
    uint32_t mine = 0;
#pragma unroll
    for (int w = 0; w < 60; w++) mine = lane == w ? rk[w] : mine;
    if (lane < 60) {
      o->rk[lane] = mine;
      o->rkr[lane] = rot16(mine);
    }
  }
  uint32_t hb[4];
#pragma unroll
  for (int w = 0; w < 4; w++) hb[w] = bswap32(h[w]);
  if (writer && lane < 4) o->h_be[lane] = lane == 0 ? hb[0] : lane == 1 ? hb[1] : lane == 2 ? hb[2] : hb[3];
  KS_STAMP(4);
  uint32_t P[4] = {hb[0], hb[1], hb[2], hb[3]};
  if constexpr (ONE) {
    // F[b] = H^(2^b), b = 0..6, by squarings, wave-uniform (every wave squares the same values; in SGPRs)
    uint32_t F[7][4];
#pragma unroll
    for (int w = 0; w < 4; w++) F[0][w] = uni(hb[w]);
#pragma unroll
    for (int b = 1; b < 7; b++) {
#pragma unroll
      for (int w = 0; w < 4; w++) F[b][w] = F[b - 1][w];
      gf_square(F[b]);
    }
    // the six factor tables: 6 x 32 positions x 2 halves = 384 units over the 256 threads
#pragma unroll
    for (int u = (int)threadIdx.x; u < 2 * 32 * kOneTabs; u += 64 * kSetupWaves) {
      const int b = u >> 6, p = (u >> 1) & 31;
      uint32_t seed[4];
#pragma unroll
      for (int w = 0; w < 4; w++) seed[w] = b == 0 ? F[0][w] : b == 1 ? F[1][w] : b == 2 ? F[2][w] : b == 3 ? F[3][w]
                                               : b == 4 ? F[4][w] : F[5][w];
      gf_mulxk(seed, 4u * (uint32_t)p);
      ghash_table_entries<8>((uint32_t)b * kSetupTab, seed, p, (u & 1) * 8);
    }
    __syncthreads();
    KS_STAMP(5);
    if (wave == 0) {
      // H^(l+1) = product of F[b] over the set bits b of l + 1 (lane 63: H^64 = F[6])
      const uint32_t e = (uint32_t)lane + 1u;
      uint32_t acc[4] = {0x80000000u, 0u, 0u, 0u};  // 1 = x^0
#pragma unroll
      for (int b = 0; b < kOneTabs; b++) {
        uint32_t x[4] = {acc[0], acc[1], acc[2], acc[3]};
        table_mul(x, (uint32_t)b * kSetupTab);  // every lane runs the product; the bit decides
        if ((e >> b) & 1u) {
#pragma unroll
          for (int w = 0; w < 4; w++) acc[w] = x[w];
        }
      }
#pragma unroll
      for (int w = 0; w < 4; w++) P[w] = lane == 63 ? F[6][w] : acc[w];
      *reinterpret_cast<uint4*>(o->hpow_be[lane]) = make_uint4(P[0], P[1], P[2], P[3]);
    } else {
      // seeds x^(4p) * H^64 (p4_be) and x^(4p) * H^(8 << t) (p4g_be[t]): 128, on the 192 lanes of waves 1-3
      const int idx = 64 * (wave - 1) + lane;
      if (idx < 128) {
        const int set = idx >> 5, p = idx & 31;
        uint32_t v[4];
#pragma unroll
        for (int w = 0; w < 4; w++) v[w] = set == 0 ? F[6][w] : set == 1 ? F[3][w] : set == 2 ? F[4][w] : F[5][w];
        gf_mulxk(v, 4u * (uint32_t)p);
        uint32_t* dst = set == 0 ? o->p4_be[p] : o->p4g_be[set - 1][p];
        *reinterpret_cast<uint4*>(dst) = make_uint4(v[0], v[1], v[2], v[3]);
      }
    }
    KS_STAMP(6);
  } else {
    // H^(lane+1): doubling scan, each level's products by a table of the level's one factor H^(2^k)
    const uint32_t wb = (uint32_t)wave * kSetupTab;
#pragma unroll 1
    for (int d = 1; d < 64; d <<= 1) {
      uint32_t y[4];
#pragma unroll
      for (int w = 0; w < 4; w++) y[w] = (uint32_t)__builtin_amdgcn_readlane((int)P[w], d - 1);
      wave_lds_sync();  // the previous level's table reads are done before the table is rebuilt
      table_of(wb, y, lane);
      wave_lds_sync();
      uint32_t x[4];
      const int src = lane >= d ? lane - d : lane;
#pragma unroll
      for (int w = 0; w < 4; w++) x[w] = (uint32_t)__shfl((int)P[w], src, 64);
      table_mul(x, wb);
      if (lane >= d && lane < 2 * d) {
#pragma unroll
        for (int w = 0; w < 4; w++) P[w] = x[w];
      }
      if (d == 1) KS_STAMP(5);
    }
    KS_STAMP(6);
    *reinterpret_cast<uint4*>(o->hpow_be[lane]) = make_uint4(P[0], P[1], P[2], P[3]);
    // record-table seeds: x^(4p) * H^64 (p4_be) and x^(4p) * H^(8 << t) (p4g_be[t]), 128 in all, 2 per lane
#pragma unroll
    for (int s = 0; s < 2; s++) {
      const int idx = lane + 64 * s, set = idx >> 5, p = idx & 31;
      const int from = set == 0 ? 63 : (8 << (set - 1)) - 1;  // lane holding H^64, H^8, H^16, H^32
      uint32_t v[4];
#pragma unroll
      for (int w = 0; w < 4; w++) v[w] = (uint32_t)__shfl((int)P[w], from, 64);
      gf_mulxk(v, 4u * (uint32_t)p);
      uint32_t* dst = set == 0 ? o->p4_be[p] : o->p4g_be[set - 1][p];
      *reinterpret_cast<uint4*>(dst) = make_uint4(v[0], v[1], v[2], v[3]);
    }
  }
  if (writer && lane == 0) {
    o->suite = suite;
    o->nr = nr;
    o->key_len = key_len;
    o->valid = 1u;
  }
#ifdef ATLS_KS_STAMPS
  KS_STAMP(7);
  if (i_key == 0 && threadIdx.x == 0) atomicAdd(&g_ks_stamps[15], (unsigned long long)__builtin_amdgcn_s_memrealtime());
#endif
}

}  // namespace atls

extern "C" int atls_launch_build_t0(uint32_t* t0, hipStream_t s) {
  hipLaunchKernelGGL(atls::build_t0_kernel, dim3(1), dim3(256), 0, s, t0);
  return hipGetLastError() == hipSuccess ? 0 : ATLS_INTERNAL_ERROR;
}

// keys: a device array of n keys, or (n <= atls_key_setup_inline_max()) nullptr with host_keys, whose
// contents then travel in the kernel arguments (no copy, nothing to wait for before the call returns).
extern "C" int atls_key_setup_inline_max(void) { return atls::kInlineKeys; }

// Debug: copy out (and reset) the key installs' phase clocks of a -DATLS_KS_STAMPS build; -1 otherwise.
extern "C" int atls_debug_ks_stamps(unsigned long long* out) {
#ifdef ATLS_KS_STAMPS
  unsigned long long h[16], z[16] = {};
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(atls::g_ks_stamps), sizeof(h)) != hipSuccess) return -1;
  if (hipMemcpyToSymbol(HIP_SYMBOL(atls::g_ks_stamps), z, sizeof(z)) != hipSuccess) return -1;
  for (int i = 0; i < 16; i++) out[i] = h[i];
  return 0;
#else
  (void)out;
  return -1;
#endif
}
extern "C" int atls_launch_key_setup(const atls_key* keys, const atls_key* host_keys, uint32_t n, void* ks,
                                     const uint32_t* t0, hipStream_t s) {
  if (n == 0) return 0;
  atls::KeySetupArgs A{};
  A.keys = keys;
  A.n = n;
  A.ks = (atls::KeySched*)ks;
  A.t0 = t0;
  if (!keys) {
    if (!host_keys || n > (uint32_t)atls::kInlineKeys) return ATLS_INTERNAL_ERROR;
    __builtin_memcpy(A.inl, host_keys, sizeof(atls_key) * n);
  }
  const uint32_t blocks = (n + atls::kSetupWaves - 1) / atls::kSetupWaves;
  if (n == 1 && ATLS_KS_ONE)  // one key: the whole workgroup on it (latency)
    hipLaunchKernelGGL(atls::key_setup_kernel<true>, dim3(1), dim3(64 * atls::kSetupWaves), atls::kOneT0 + 1024, s, A);
  else
    hipLaunchKernelGGL(atls::key_setup_kernel<false>, dim3(blocks), dim3(64 * atls::kSetupWaves),
                       atls::kSetupT0 + 1024, s, A);
  return hipGetLastError() == hipSuccess ? 0 : ATLS_INTERNAL_ERROR;
}
