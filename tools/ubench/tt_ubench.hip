// Microbenchmark: T-table AES-128 rounds (2 tables x 32 bank copies in LDS, gcm.hip layout) and
// the 4-bit-table GHASH multiply (gcm_common.h) on gfx950, no HBM traffic. Reports CU-cycles per
// 16-B block at 2.4 GHz nominal, for several waves/CU and blocks/lane.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }
__device__ __forceinline__ uint32_t rot16(uint32_t x) { return (x << 16) | (x >> 16); }
__device__ __forceinline__ uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel) { return __builtin_amdgcn_perm(hi, lo, sel); }
__device__ __forceinline__ uint32_t lds_u32(uint32_t a) { return *reinterpret_cast<const __attribute__((address_space(3))) uint32_t*>(a); }
typedef uint32_t v4u32 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ v4u32 lds_u4(uint32_t a) { return *reinterpret_cast<const __attribute__((address_space(3))) v4u32*>(a); }
#define TA(w, sh) perm((w), lb, 0x0c0c0000u | ((4u + (sh) / 8u) << 8))

template <int NB>
__device__ __forceinline__ void aes_tt(uint32_t (&s)[NB][4], const uint32_t* rk, const uint32_t* rkr, uint32_t lb) {
#pragma unroll
  for (int b = 0; b < NB; b++)
#pragma unroll
    for (int i = 0; i < 4; i++) s[b][i] ^= rk[i];
#pragma unroll
  for (int r = 1; r < 10; r++) {
#pragma unroll
    for (int b = 0; b < NB; b++) {
      const uint32_t s0 = s[b][0], s1 = s[b][1], s2 = s[b][2], s3 = s[b][3];
      uint32_t t[4];
#pragma unroll
      for (int c = 0; c < 4; c++) {
        const uint32_t a = (c == 0 ? s0 : c == 1 ? s1 : c == 2 ? s2 : s3);
        const uint32_t bb = (c == 0 ? s1 : c == 1 ? s2 : c == 2 ? s3 : s0);
        const uint32_t cc = (c == 0 ? s2 : c == 1 ? s3 : c == 2 ? s0 : s1);
        const uint32_t dd = (c == 0 ? s3 : c == 1 ? s0 : c == 2 ? s1 : s2);
        const uint32_t u = xor3(lds_u32(TA(cc, 16)), lds_u32(TA(dd, 24) + 128), rkr[4 * r + c]);
        t[c] = xor3(lds_u32(TA(a, 0)), lds_u32(TA(bb, 8) + 128), rot16(u));
      }
#pragma unroll
      for (int c = 0; c < 4; c++) s[b][c] = t[c];
    }
  }
#pragma unroll
  for (int b = 0; b < NB; b++) {
    const uint32_t s0 = s[b][0], s1 = s[b][1], s2 = s[b][2], s3 = s[b][3];
    uint32_t t[4];
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const uint32_t a = (c == 0 ? s0 : c == 1 ? s1 : c == 2 ? s2 : s3);
      const uint32_t bb = (c == 0 ? s1 : c == 1 ? s2 : c == 2 ? s3 : s0);
      const uint32_t cc = (c == 0 ? s2 : c == 1 ? s3 : c == 2 ? s0 : s1);
      const uint32_t dd = (c == 0 ? s3 : c == 1 ? s0 : c == 2 ? s1 : s2);
      const uint32_t lo = perm(lds_u32(TA(bb, 8)), lds_u32(TA(a, 0)), 0x0c0c0501u);
      const uint32_t hi = perm(lds_u32(TA(dd, 24) + 128), lds_u32(TA(cc, 16) + 128), 0x07020c0cu);
      t[c] = __builtin_amdgcn_bitop3_b32(lo, hi, rk[40 + c], 0x56);
    }
#pragma unroll
    for (int c = 0; c < 4; c++) s[b][c] = t[c];
  }
}

__device__ __forceinline__ void ghash_mul_tab(uint32_t (&y)[4], uint32_t wb) {
  uint32_t a0 = 0, a1 = 0, a2 = 0, a3 = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const uint32_t hi4 = y[i] & 0xF0F0F0F0u, lo4 = (y[i] << 4) & 0xF0F0F0F0u;
#pragma unroll
    for (int b = 0; b < 4; b++) {
      const uint32_t byte = 4 * i + b;
      const uint32_t sel = 0x0c020100u | (4u + b);
      const v4u32 eh = lds_u4(perm(hi4, wb, sel) + (2 * byte) * 256);
      const v4u32 el = lds_u4(perm(lo4, wb, sel) + (2 * byte + 1) * 256);
      a0 = xor3(a0, eh.x, el.x); a1 = xor3(a1, eh.y, el.y); a2 = xor3(a2, eh.z, el.z); a3 = xor3(a3, eh.w, el.w);
    }
  }
  y[0] = a0; y[1] = a1; y[2] = a2; y[3] = a3;
}

// MODE 0: AES only, 1: GHASH only (Horner chain), 2: both
template <int MODE, int NB, int WAVES>
__global__ __launch_bounds__(64 * WAVES) void k(const uint32_t* rkg, uint32_t* out, int iters) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  for (int i = threadIdx.x; i < 16384; i += blockDim.x) smem[i] = i * 0x9E3779B9u;
  for (int i = threadIdx.x; i < WAVES * 2048; i += blockDim.x) smem[16384 + i] = i * 0x85EBCA6Bu;
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t lb = 4u * (lane & 31), wb = 65536u + wave * 8192u;
  uint32_t rk[44], rkr[44];
  const __attribute__((address_space(4))) uint32_t* rc = (const __attribute__((address_space(4))) uint32_t*)rkg;
#pragma unroll
  for (int i = 0; i < 44; i++) { rk[i] = rc[i]; rkr[i] = rot16(rk[i]); }
  uint32_t acc[4] = {0, 0, 0, 0}, y[4] = {lane * 3u, lane * 5u, lane * 7u, lane * 11u};
  for (int it = 0; it < iters; it++) {
    uint32_t st[NB][4];
#pragma unroll
    for (int b = 0; b < NB; b++) { st[b][0] = 0x11u; st[b][1] = 0x22u; st[b][2] = it; st[b][3] = (it * 64 + lane) * NB + b; }
    if (MODE != 1) aes_tt<NB>(st, rk, rkr, lb);
#pragma unroll
    for (int b = 0; b < NB; b++) {
      if (MODE != 0) {
        ghash_mul_tab(y, wb);
#pragma unroll
        for (int w = 0; w < 4; w++) y[w] ^= st[b][w];
      } else {
#pragma unroll
        for (int w = 0; w < 4; w++) acc[w] ^= st[b][w];
      }
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc[0] ^ acc[1] ^ acc[2] ^ acc[3] ^ y[0] ^ y[1] ^ y[2] ^ y[3];
}

template <int MODE, int NB, int WAVES>
void run(const uint32_t* drk, uint32_t* dout) {
  const int grid = 256 * 4, iters = 256;
  const size_t lds = 65536 + WAVES * 8192;
  hipLaunchKernelGGL((k<MODE, NB, WAVES>), dim3(grid), dim3(64 * WAVES), lds, 0, drk, dout, 4);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL((k<MODE, NB, WAVES>), dim3(grid), dim3(64 * WAVES), lds, 0, drk, dout, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms; (void)hipEventElapsedTime(&ms, e0, e1);
  const double blocks = (double)grid * 64 * WAVES * NB * iters;
  printf("mode=%s NB=%d waves/CU=%d: %.3f ms, %.2f CU-cycles/block @2.4GHz, %.1f GB/s\n",
         MODE == 0 ? "aes  " : MODE == 1 ? "ghash" : "both ", NB, WAVES, ms, 256.0 * 2.4e9 * ms * 1e-3 / blocks,
         blocks * 16 / (ms * 1e-3) / 1e9);
}

int main() {
  uint32_t *drk, *dout;
  (void)hipMalloc(&drk, 4096);
  (void)hipMemset(drk, 0x3c, 4096);
  (void)hipMalloc(&dout, 256 * 4 * 1024 * 4);
  run<0, 1, 8>(drk, dout);
  run<0, 1, 12>(drk, dout);
  run<0, 2, 8>(drk, dout);
  run<0, 2, 12>(drk, dout);
  run<1, 1, 8>(drk, dout);
  run<1, 1, 12>(drk, dout);
  run<1, 2, 12>(drk, dout);
  run<2, 1, 8>(drk, dout);
  run<2, 1, 12>(drk, dout);
  run<2, 2, 12>(drk, dout);
  return 0;
}
