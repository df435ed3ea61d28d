// Microbenchmark: does the vector-memory path (TA / TD / L1) add T-table lookup throughput beside
// the LDS? The AES-GCM kernel is bound by its LDS array (74.5 % busy, 133
// ds_read_b32 + 32 ds_read_b128 per block). Here each lane runs T-table AES-like rounds (16
// lookups per round from T0 / T1 by a byte of the state, combined with xor3 / rot16) with NG of the
// 16 lookups per round served by struct-buffer gathers from a 2 KiB table in global memory (L1-
// resident) and the rest by conflict-free ds_read_b32 from the kernel's 32x-replicated LDS tables.
// One 768-thread workgroup per CU (12 waves), as the record kernel. Prints ns per round per wave.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
__device__ int32_t buf_ld(i32x4 rsrc, int32_t vindex, int32_t voffset, int32_t soffset, int32_t aux)
    __asm("llvm.amdgcn.struct.buffer.load.i32");

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }
__device__ __forceinline__ uint32_t rot16(uint32_t x) { return (x << 16) | (x >> 16); }
__device__ __forceinline__ uint32_t lds_u32(uint32_t a) { return *reinterpret_cast<const __attribute__((address_space(3))) uint32_t*>(a); }
#define TA(w, sh) __builtin_amdgcn_perm((w), lb, 0x0c0c0000u | ((4u + (sh) / 8u) << 8))

// lookup i of a round (i = 4c + k: column c, byte k): global when G(i), else LDS
template <int NG>
__device__ __forceinline__ bool is_g(int i) { return NG > 0 && (i % (16 / NG)) == 0; }

template <int NG>
__device__ __forceinline__ uint32_t look(int i, uint32_t w, int sh, bool t1, uint32_t lb, i32x4 rs) {
  if (is_g<NG>(i)) return (uint32_t)buf_ld(rs, (int32_t)__builtin_amdgcn_ubfe(w, sh, 8) + (t1 ? 256 : 0), 0, 0, 0);
  return lds_u32(TA(w, sh) + (t1 ? 128u : 0u));
}

template <int NG>
__global__ __launch_bounds__(768) void k_rounds(const uint32_t* tab, uint32_t* out, int rounds) {
  extern __shared__ uint32_t sh_tt[];  // 256 rows x 64 words: T0 x32 | T1 x32
  for (int i = threadIdx.x; i < 256 * 64; i += blockDim.x) {
    const int e = i / 64, c = i % 64;
    sh_tt[i] = c < 32 ? tab[e] : tab[256 + e];
  }
  __syncthreads();
  const uint32_t lb = (threadIdx.x & 31) * 4;
  i32x4 rs;
  const uint64_t base = (uint64_t)tab;
  rs.x = (int32_t)(uint32_t)base;
  rs.y = (int32_t)((uint32_t)(base >> 32) | (4u << 16));  // stride 4 B
  rs.z = 512;                                            // records
  rs.w = 0x00020000;                                     // raw dword format bits as the compiler's default
  uint32_t s[4] = {threadIdx.x * 0x9e3779b9u, blockIdx.x * 0x7f4a7c15u + 1, threadIdx.x ^ 0x5bd1e995u, 0x27d4eb2fu};
  for (int r = 0; r < rounds; r++) {
    uint32_t v[16];
#pragma unroll
    for (int c = 0; c < 4; c++) {
      v[4 * c + 0] = look<NG>(4 * c + 0, s[c], 0, false, lb, rs);
      v[4 * c + 1] = look<NG>(4 * c + 1, s[(c + 1) & 3], 8, true, lb, rs);
      v[4 * c + 2] = look<NG>(4 * c + 2, s[(c + 2) & 3], 16, false, lb, rs);
      v[4 * c + 3] = look<NG>(4 * c + 3, s[(c + 3) & 3], 24, true, lb, rs);
    }
    s[0] = xor3(v[0], v[1], rot16(xor3(v[2], v[3], r)));
    s[1] = xor3(v[4], v[5], rot16(xor3(v[6], v[7], r * 3)));
    s[2] = xor3(v[8], v[9], rot16(xor3(v[10], v[11], r * 5)));
    s[3] = xor3(v[12], v[13], rot16(xor3(v[14], v[15], r * 7)));
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = s[0] ^ s[1] ^ s[2] ^ s[3];
}

template <int NG>
static void run(const uint32_t* tab, uint32_t* out, int ncu) {
  const int rounds = 4000;
  hipLaunchKernelGGL(k_rounds<NG>, dim3(ncu), dim3(768), 256 * 64 * 4, 0, tab, out, 16);
  (void)hipDeviceSynchronize();
  hipEvent_t a, b;
  (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  float best = 1e30f;
  for (int it = 0; it < 5; it++) {
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(k_rounds<NG>, dim3(ncu), dim3(768), 256 * 64 * 4, 0, tab, out, rounds);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms; (void)hipEventElapsedTime(&ms, a, b);
    if (ms < best) best = ms;
  }
  const double per_round_wave = best * 1e6 / rounds / 12.0;  // ns per round per wave slot of a CU
  printf("{\"global_lookups_per_round\": %d, \"lds_lookups_per_round\": %d, \"ms\": %.4f, \"ns_per_round_per_cu\": %.3f, \"ns_per_round_per_wave\": %.3f}\n",
         NG, 16 - NG, best, best * 1e6 / rounds, per_round_wave);
}

int main() {
  int ncu = 0;
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  uint32_t h[512];
  for (int i = 0; i < 512; i++) h[i] = (uint32_t)i * 0x01000193u ^ 0x811c9dc5u;
  uint32_t *tab, *out;
  (void)hipMalloc(&tab, sizeof h);
  (void)hipMemcpy(tab, h, sizeof h, hipMemcpyHostToDevice);
  (void)hipMalloc(&out, (size_t)ncu * 768 * 4);
  (void)hipFuncSetAttribute((const void*)k_rounds<0>, hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
  (void)hipFuncSetAttribute((const void*)k_rounds<2>, hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
  (void)hipFuncSetAttribute((const void*)k_rounds<4>, hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
  (void)hipFuncSetAttribute((const void*)k_rounds<8>, hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
  (void)hipFuncSetAttribute((const void*)k_rounds<16>, hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
  printf("{\"cus\": %d}\n", ncu);
  run<0>(tab, out, ncu);
  run<2>(tab, out, ncu);
  run<4>(tab, out, ncu);
  run<8>(tab, out, ncu);
  run<16>(tab, out, ncu);
  return 0;
}
