// Microbenchmark: bitsliced AES-128 rounds (row-plane layout, aes_bs.h) on the VALU with
// wave-uniform round-key masks in SGPRs, G groups of 8 blocks per lane, no memory traffic.
// Prints CU-cycles per 16-B block at the nominal 2.4 GHz for each variant.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include "../bitsliced/sbox_bs.h"

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }
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

template <int G, int WPB>
void run(const uint32_t* dm, uint32_t* dout, int blocks_per_cu) {
  const int grid = 256 * blocks_per_cu, iters = 64;
  hipLaunchKernelGGL((k_bs<G, WPB>), dim3(grid), dim3(64 * WPB), 0, 0, dm, dout, 2);
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  hipEventRecord(a);
  hipLaunchKernelGGL((k_bs<G, WPB>), dim3(grid), dim3(64 * WPB), 0, 0, dm, dout, iters);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  const double blocks = (double)grid * 64 * WPB * 8 * G * iters;
  const double cyc = 256.0 * 2.4e9 * ms * 1e-3 / blocks;
  printf("bitsliced AES-128 G=%d waves/WG=%d WG/CU-ish=%d: %.3f ms, %.2f CU-cycles/block, %.1f GB/s keystream\n", G, WPB,
         blocks_per_cu, ms, cyc, blocks * 16 / (ms * 1e-3) / 1e9);
}

int main() {
  uint32_t *dm, *dout;
  hipMalloc(&dm, 4096);
  hipMemset(dm, 0x5a, 4096);
  hipMalloc(&dout, 256 * 64 * 1024 * 4);
  run<1, 4>(dm, dout, 8);
  run<2, 4>(dm, dout, 4);
  run<2, 4>(dm, dout, 8);
  run<2, 8>(dm, dout, 2);
  run<4, 4>(dm, dout, 2);
  run<4, 4>(dm, dout, 4);
  return 0;
}
