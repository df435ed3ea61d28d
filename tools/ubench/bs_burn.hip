// Burn kernel for co-residency experiments: aes_ubench's bitsliced AES rounds (VALU only, no
// memory traffic) callable from Python beside the engine (tools/corun_gcm.py).
#include <hip/hip_runtime.h>
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


extern "C" int bs_burn(void* stream, int g, int grid, int iters, const uint32_t* masks, uint32_t* out) {
  if (g == 1)
    hipLaunchKernelGGL((k_bs<1, 4>), dim3(grid), dim3(256), 0, (hipStream_t)stream, masks, out, iters);
  else
    hipLaunchKernelGGL((k_bs<2, 4>), dim3(grid), dim3(256), 0, (hipStream_t)stream, masks, out, iters);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
