// Microbenchmark of the AES-GCM fast step (gcm.hip): per 64-slot step a wave loads 1 KiB of
// payload from HBM, runs T-table AES-CTR on 64 counter blocks, stores 1 KiB, and folds 64
// ciphertext blocks into its lane-strided GHASH (4-bit table multiply). Variants differ only in
// instruction scheduling / key placement, to find the fastest form before it goes into gcm.hip.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include "../../anothertls_amd/csrc/gcm_common.h"

using namespace atls;
#define TA(w, sh) perm((w), lb, 0x0c0c0000u | ((4u + (sh) / 8u) << 8))
typedef const __attribute__((address_space(4))) v4u32 kv4;

// V_SCHED: 0 = compiler schedule; 1 = batch 16 lookups per round (sched_barrier)
template <int V_SCHED>
__device__ __forceinline__ void round_tt(uint32_t (&s)[4], uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3, uint32_t lb) {
  if (V_SCHED == 0) {
    const uint32_t s0 = s[0], s1 = s[1], s2 = s[2], s3 = s[3];
    const uint32_t kk[4] = {k0, k1, k2, k3};
    uint32_t t[4];
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const uint32_t a = (c == 0 ? s0 : c == 1 ? s1 : c == 2 ? s2 : s3);
      const uint32_t bb = (c == 0 ? s1 : c == 1 ? s2 : c == 2 ? s3 : s0);
      const uint32_t cc = (c == 0 ? s2 : c == 1 ? s3 : c == 2 ? s0 : s1);
      const uint32_t dd = (c == 0 ? s3 : c == 1 ? s0 : c == 2 ? s1 : s2);
      const uint32_t u = xor3(lds_u32(TA(cc, 16)), lds_u32(TA(dd, 24) + 128), kk[c]);
      t[c] = xor3(lds_u32(TA(a, 0)), lds_u32(TA(bb, 8) + 128), rot16(u));
    }
#pragma unroll
    for (int c = 0; c < 4; c++) s[c] = t[c];
  } else {
    uint32_t v[16];
#pragma unroll
    for (int c = 0; c < 4; c++) {
      v[4 * c + 0] = lds_u32(TA(s[c], 0));
      v[4 * c + 1] = lds_u32(TA(s[(c + 1) & 3], 8) + 128);
      v[4 * c + 2] = lds_u32(TA(s[(c + 2) & 3], 16));
      v[4 * c + 3] = lds_u32(TA(s[(c + 3) & 3], 24) + 128);
    }
    __builtin_amdgcn_sched_barrier(0);
    s[0] = xor3(v[0], v[1], rot16(xor3(v[2], v[3], k0)));
    s[1] = xor3(v[4], v[5], rot16(xor3(v[6], v[7], k1)));
    s[2] = xor3(v[8], v[9], rot16(xor3(v[10], v[11], k2)));
    s[3] = xor3(v[12], v[13], rot16(xor3(v[14], v[15], k3)));
  }
}

template <int V_SCHED>
__device__ __forceinline__ void final_tt(uint32_t (&s)[4], uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3, uint32_t lb) {
  uint32_t v[16];
#pragma unroll
  for (int c = 0; c < 4; c++) {
    v[4 * c + 0] = lds_u32(TA(s[c], 0));
    v[4 * c + 1] = lds_u32(TA(s[(c + 1) & 3], 8));
    v[4 * c + 2] = lds_u32(TA(s[(c + 2) & 3], 16) + 128);
    v[4 * c + 3] = lds_u32(TA(s[(c + 3) & 3], 24) + 128);
  }
  if (V_SCHED) __builtin_amdgcn_sched_barrier(0);
  const uint32_t kw[4] = {k0, k1, k2, k3};
#pragma unroll
  for (int c = 0; c < 4; c++) {
    const uint32_t lo = perm(v[4 * c + 1], v[4 * c], 0x0c0c0501u);
    const uint32_t hi = perm(v[4 * c + 3], v[4 * c + 2], 0x07020c0cu);
    s[c] = __builtin_amdgcn_bitop3_b32(lo, hi, kw[c], 0x56);
  }
}

// V_KEYS: 0 = all round keys loaded once into (uniform) registers; 1 = rolled round loop with a
// scalar load per round.  V_GH: 0 = ghash_mul_tab (compiler schedule); W > 0 = ghash_mul_tab_wide<W>.
template <int V_SCHED, int V_KEYS, int V_GH, int WAVES>
__global__ __launch_bounds__(64 * WAVES) void k_step(const uint32_t* rkg, const uint8_t* in, uint8_t* out, uint32_t* yout,
                                                     int steps_per_wave) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  for (int i = threadIdx.x; i < 16384; i += blockDim.x) smem[i] = i * 0x9E3779B9u;
  for (int i = threadIdx.x; i < WAVES * 2048; i += blockDim.x) smem[16384 + i] = i * 0x85EBCA6Bu;
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t lb = 4u * (lane & 31), wb = 65536u + wave * 8192u;
  const uint32_t gw = blockIdx.x * WAVES + wave;
  uint32_t y[4] = {0, 0, 0, 0};
  uint32_t rk[44];
  if constexpr (V_KEYS == 0) {
#pragma unroll
    for (int i = 0; i < 44; i++) rk[i] = ((const __attribute__((address_space(4))) uint32_t*)rkg)[i];
  }
  for (int st = 0; st < steps_per_wave; st++) {
    const size_t off = ((size_t)gw * steps_per_wave + st) * 1024 + lane * 16;
    const v4u32 P = *reinterpret_cast<const v4u32*>(in + off);
    uint32_t s[4] = {0x11u ^ rkg[0], 0x22u, (uint32_t)st, (uint32_t)(st * 64 + lane)};
    if constexpr (V_KEYS == 0) {
#pragma unroll
      for (int r = 1; r < 10; r++) round_tt<V_SCHED>(s, rk[4 * r], rk[4 * r + 1], rk[4 * r + 2], rk[4 * r + 3], lb);
      final_tt<V_SCHED>(s, rk[40], rk[41], rk[42], rk[43], lb);
    } else {
#pragma unroll 1
      for (int r = 1; r < 10; r++) {
        const v4u32 kr = *(kv4*)(rkg + 4 * r);
        round_tt<V_SCHED>(s, kr.x, kr.y, kr.z, kr.w, lb);
      }
      const v4u32 kf = *(kv4*)(rkg + 40);
      final_tt<V_SCHED>(s, kf.x, kf.y, kf.z, kf.w, lb);
    }
    const v4u32 C = {P.x ^ s[0], P.y ^ s[1], P.z ^ s[2], P.w ^ s[3]};
    *reinterpret_cast<v4u32*>(out + off) = C;
    if constexpr (V_GH == 0) ghash_mul_tab(y, wb);
    else ghash_mul_tab_wide<V_GH>(y, wb);
    y[0] ^= C.x; y[1] ^= C.y; y[2] ^= C.z; y[3] ^= C.w;
  }
  yout[(blockIdx.x * blockDim.x + threadIdx.x)] = y[0] ^ y[1] ^ y[2] ^ y[3];
}

template <int V_SCHED, int V_KEYS, int V_GH, int WAVES>
void run(const char* name, const uint32_t* drk, const uint8_t* din, uint8_t* dout, uint32_t* dy) {
  const int grid = 256, steps = 64;  // 256 WG x WAVES x 64 steps x 1 KiB
  const size_t lds = 65536 + WAVES * 8192;
  hipLaunchKernelGGL((k_step<V_SCHED, V_KEYS, V_GH, WAVES>), dim3(grid), dim3(64 * WAVES), lds, 0, drk, din, dout, dy, steps);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  for (int i = 0; i < 5; i++)
    hipLaunchKernelGGL((k_step<V_SCHED, V_KEYS, V_GH, WAVES>), dim3(grid), dim3(64 * WAVES), lds, 0, drk, din, dout, dy, steps);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms; (void)hipEventElapsedTime(&ms, e0, e1);
  ms /= 5;
  const double blocks = (double)grid * WAVES * steps * 64;
  printf("%-28s waves=%2d: %.3f ms  %.2f CU-cyc/block@2.4  %.1f GB/s payload\n", name, WAVES, ms,
         256.0 * 2.4e9 * ms * 1e-3 / blocks, blocks * 16 / (ms * 1e-3) / 1e9);
}

int main() {
  uint32_t *drk, *dy;
  uint8_t *din, *dout;
  const size_t bytes = (size_t)256 * 12 * 64 * 1024;
  (void)hipMalloc(&drk, 4096);
  (void)hipMemset(drk, 0x3c, 4096);
  (void)hipMalloc(&din, bytes);
  (void)hipMalloc(&dout, bytes);
  (void)hipMemset(din, 0x5a, bytes);
  (void)hipMalloc(&dy, 256 * 1024 * 4);
  run<0, 0, 0, 12>("sched=cc keys=regs gh=cc", drk, din, dout, dy);
  run<1, 0, 0, 12>("sched=batch keys=regs gh=cc", drk, din, dout, dy);
  run<1, 0, 8, 12>("sched=batch keys=regs gh=w8", drk, din, dout, dy);
  run<1, 0, 16, 12>("sched=batch keys=regs gh=w16", drk, din, dout, dy);
  run<1, 1, 8, 12>("sched=batch keys=sload gh=w8", drk, din, dout, dy);
  run<1, 1, 16, 12>("sched=batch keys=sload gh=w16", drk, din, dout, dy);
  run<0, 1, 0, 12>("sched=cc keys=sload gh=cc", drk, din, dout, dy);
  run<0, 0, 8, 12>("sched=cc keys=regs gh=w8", drk, din, dout, dy);
  run<1, 0, 8, 8>("sched=batch keys=regs gh=w8", drk, din, dout, dy);
  return 0;
}
