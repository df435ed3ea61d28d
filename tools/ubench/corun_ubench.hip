// Microbenchmark: can the LDS-bound T-table AES-GCM step (step_ubench's k_step) and the
// VALU-bound bitsliced AES (aes_ubench's k_bs) share the CUs? Times each kernel alone and both
// launched together on two streams; if the pair takes about max(A, B) rather than A + B, a
// keystream kernel on the VALU beside the T-table kernel pays.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include "../../anothertls_amd/csrc/gcm_common.h"
#include "../bitsliced/sbox_bs.h"

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


__device__ __forceinline__ uint32_t rotr(uint32_t w, int n) { return n ? __builtin_amdgcn_alignbit(w, w, n) : w; }
typedef const __attribute__((address_space(4))) uint32_t cu32;

template <int G>
__device__ __forceinline__ void smark(uint32_t (&st)[G][4][8], cu32* m) {
#pragma unroll
  for (int g = 0; g < G; g++) {
    uint32_t (&a)[4][8] = st[g];
#pragma unroll
    for (int r = 1; r < 4; r++)
#pragma unroll
      for (int j = 0; j < 8; j++) a[r][j] = rotr(a[r][j], 8 * r);
    uint32_t u7[4];
#pragma unroll
    for (int r = 0; r < 4; r++) u7[r] = a[r][0] ^ a[(r + 1) & 3][0];
#pragma unroll
    for (int t = 7; t >= 0; t--) {
      const int j = 7 - t;
      uint32_t o[4];
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const uint32_t v = xor3(a[(r + 1) & 3][j], a[(r + 2) & 3][j], a[(r + 3) & 3][j]);
        const uint32_t k = m[8 * r + j];
        if (t == 0) o[r] = xor3(v, u7[r], k);
        else {
          const uint32_t u = a[r][j + 1] ^ a[(r + 1) & 3][j + 1];
          o[r] = (t == 1 || t == 3 || t == 4) ? xor3(xor3(v, u, u7[r]), k, 0u) : xor3(v, u, k);
        }
      }
#pragma unroll
      for (int r = 0; r < 4; r++) a[r][j] = o[r];
    }
  }
}

template <int G, int WPB>
__global__ __launch_bounds__(64 * WPB) __attribute__((amdgpu_waves_per_eu(G == 1 ? 8 : G == 2 ? 4 : 1))) void k_bs(const uint32_t* masks, uint32_t* out, int iters) {
  uint32_t st[G][4][8];
#pragma unroll
  for (int g = 0; g < G; g++)
#pragma unroll
    for (int r = 0; r < 4; r++)
#pragma unroll
      for (int j = 0; j < 8; j++) st[g][r][j] = threadIdx.x * 0x9E3779B9u + (g * 32 + r * 8 + j) * 0x85EBCA6Bu;
  for (int it = 0; it < iters; it++) {
#pragma unroll 1
    for (int rd = 1; rd <= 10; rd++) {
#pragma unroll
      for (int g = 0; g < G; g++)
#pragma unroll
        for (int r = 0; r < 4; r++) sbox_bs(st[g][r]);
      cu32* m = (cu32*)masks + 32 * rd;
      if (rd < 10) smark<G>(st, m);
      else {
#pragma unroll
        for (int g = 0; g < G; g++)
#pragma unroll
          for (int r = 0; r < 4; r++)
#pragma unroll
            for (int j = 0; j < 8; j++) st[g][r][j] = rotr(st[g][r][j], 8 * r) ^ m[8 * r + j];
      }
    }
  }
  uint32_t acc = 0;
#pragma unroll
  for (int g = 0; g < G; g++)
#pragma unroll
    for (int r = 0; r < 4; r++)
#pragma unroll
      for (int j = 0; j < 8; j++) acc ^= st[g][r][j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}


template <int WAVES>
void launchA(hipStream_t s, const uint32_t* drk, const uint8_t* din, uint8_t* dout, uint32_t* dy, int steps) {
  hipLaunchKernelGGL((k_step<0, 0, 0, WAVES>), dim3(256), dim3(64 * WAVES), 65536 + WAVES * 8192, s, drk, din, dout, dy, steps);
}
template <int G, int WPB>
void launchB(hipStream_t s, const uint32_t* dm, uint32_t* dout, int grid, int iters) {
  hipLaunchKernelGGL((k_bs<G, WPB>), dim3(grid), dim3(64 * WPB), 0, s, dm, dout, iters);
}

template <int WAVES, int G, int WPB>
void trial(const char* name, int stepsA, int gridB, int itersB, const uint32_t* drk, const uint8_t* din, uint8_t* dout,
           uint32_t* dy, const uint32_t* dm, uint32_t* dbo) {
  hipStream_t s1, s2;
  (void)hipStreamCreateWithFlags(&s1, hipStreamNonBlocking);
  (void)hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  float ta, tb, tab;
  launchA<WAVES>(s1, drk, din, dout, dy, 2); launchB<G, WPB>(s2, dm, dbo, gridB, 1); (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0, s1); launchA<WAVES>(s1, drk, din, dout, dy, stepsA); (void)hipEventRecord(e1, s1);
  (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ta, e0, e1);
  (void)hipEventRecord(e0, s2); launchB<G, WPB>(s2, dm, dbo, gridB, itersB); (void)hipEventRecord(e1, s2);
  (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&tb, e0, e1);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0, 0);
  (void)hipStreamWaitEvent(s1, e0, 0); (void)hipStreamWaitEvent(s2, e0, 0);
  launchA<WAVES>(s1, drk, din, dout, dy, stepsA);
  launchB<G, WPB>(s2, dm, dbo, gridB, itersB);
  hipEvent_t d1, d2;
  (void)hipEventCreate(&d1); (void)hipEventCreate(&d2);
  (void)hipEventRecord(d1, s1); (void)hipEventRecord(d2, s2);
  (void)hipStreamWaitEvent(0, d1, 0); (void)hipStreamWaitEvent(0, d2, 0);
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&tab, e0, e1);
  const double blkA = 256.0 * WAVES * stepsA * 64, blkB = (double)gridB * 64 * WPB * 8 * G * itersB;
  printf("%-22s A(tt %2dw) %.3f ms %.0f GB/s | B(bs G=%d) %.3f ms %.0f GB/s | together %.3f ms (A+B %.3f, max %.3f) -> %.0f GB/s\n",
         name, WAVES, ta, blkA * 16 / ta / 1e6, G, tb, blkB * 16 / tb / 1e6, tab, ta + tb, ta > tb ? ta : tb,
         (blkA + blkB) * 16 / tab / 1e6);
}

int main() {
  uint32_t *drk, *dy, *dm, *dbo;
  uint8_t *din, *dout;
  const size_t bytes = (size_t)256 * 12 * 64 * 1024;
  (void)hipMalloc(&drk, 4096); (void)hipMemset(drk, 0x3c, 4096);
  (void)hipMalloc(&din, bytes); (void)hipMalloc(&dout, bytes); (void)hipMemset(din, 0x5a, bytes);
  (void)hipMalloc(&dy, 256 * 1024 * 4);
  (void)hipMalloc(&dm, 4096); (void)hipMemset(dm, 0x5a, 4096);
  (void)hipMalloc(&dbo, 256 * 64 * 1024 * 4);
  trial<12, 2, 4>("tt12 + bs G2 x4w", 64, 256, 8, drk, din, dout, dy, dm, dbo);
  trial<8, 2, 4>("tt8 + bs G2 x4w", 64, 256, 8, drk, din, dout, dy, dm, dbo);
  trial<8, 1, 4>("tt8 + bs G1 x4w", 64, 512, 8, drk, din, dout, dy, dm, dbo);
  trial<8, 2, 4>("tt8 + bs G2 x4w (more B)", 64, 512, 8, drk, din, dout, dy, dm, dbo);
  trial<8, 4, 4>("tt8 + bs G4 x4w", 64, 256, 4, drk, din, dout, dy, dm, dbo);
  return 0;
}
