// Microbenchmark (round 6): what rate the LDS array gives the AES-GCM kernel's access patterns.
// gcm_kernel's fast step is 133 conflict-free random-row ds_read_b32 (T-table lookups, lane l always on bank
// l & 31) and 32 ds_read_b128 into 256-B GHASH table rows per 64 blocks, and SQ_LDS_IDX_ACTIVE puts the array at
// 0.72-0.75 of the launch's cycles. The question is whether the remaining quarter is idle because the kernel
// does not keep the array fed, or because random-row gathers cannot run at the documented 2 / 4 cycles per
// wave-instruction (MI355X_MICROARCH.md §LDS). Each pattern below issues 16 independent LDS reads per
// iteration per wave (one VALU op builds an address: a per-lane offset XOR a wave-uniform row select; with
// "dependent" the row select of the next iteration waits for this one's results, as an AES round's addresses
// wait for the round before), one
// workgroup per CU, 4-16 waves, and reports LDS-array cycles per wave-instruction from the waves' own
// s_memtime (shader clock) spans -- no HBM traffic, so nothing but the LDS and the issue of these few VALU ops.
//   b32_tt     : T-table layout (row = 32 x T0 | 32 x T1 words, 256 B), random row per lane, bank = lane & 31
//   b32_lin    : every lane a different bank of one row (a[l] = 4 l), rows walked in order
//   b32_bcast  : all lanes one address
//   b32_64bank : random row per lane, bank = lane (lanes 32-63 on banks 32-63; rows of 512 B)
//   b64_tt     : 8-byte entries, random row per lane, banks 2(l & 31), 2(l & 31) + 1
//   b128_gh    : GHASH 4-bit table: row = position (256 B), random nibble per lane (16-B entry)
//   mix        : 4 b32_tt + 1 b128_gh, in the fast step's proportion (133 : 32)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint32_t v2u32 __attribute__((ext_vector_type(2)));
typedef uint32_t v4u32 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint32_t ld32(uint32_t a) { return *reinterpret_cast<const __attribute__((address_space(3))) uint32_t*>(a); }
__device__ __forceinline__ v2u32 ld64(uint32_t a) { return *reinterpret_cast<const __attribute__((address_space(3))) v2u32*>(a); }
__device__ __forceinline__ v4u32 ld128(uint32_t a) { return *reinterpret_cast<const __attribute__((address_space(3))) v4u32*>(a); }
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }

enum { B32_TT, B32_LIN, B32_BCAST, B32_64BANK, B64_TT, B128_GH, MIX };
static const char* kNames[] = {"b32_tt", "b32_lin", "b32_bcast", "b32_64bank", "b64_tt", "b128_gh", "mix"};

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}

// per-lane offset of read k (fixed), and the row-select mask the wave-uniform value is applied with
template <int P>
__device__ __forceinline__ uint32_t base_off(int lane, int k) {
  const uint32_t h = hash32(lane * 131u + k * 7919u + 17u);
  switch (P) {
    case B32_TT: return (h & 255u) * 256u + ((k & 1) ? 128u : 0u) + 4u * (lane & 31);
    case B32_LIN: return 4u * lane;
    case B32_BCAST: return 0u;
    case B32_64BANK: return (h & 127u) * 512u + 4u * lane;  // 64 KiB: 128 rows of 512 B
    case B64_TT: return (h & 255u) * 256u + 8u * (lane & 31);
    case B128_GH: return (k & 31u) * 256u + (h & 15u) * 16u;
    default: return 0u;
  }
}
template <int P>
__device__ __forceinline__ uint32_t row_mask() {
  switch (P) {
    case B32_TT: return 0xff00u;     // XOR changes the row, keeps the bank
    case B32_LIN: return 0xff00u;    // walks rows; lane l stays on bank l (a row is 256 B = 64 banks x 4 B)
    case B32_BCAST: return 0xfffcu;
    case B32_64BANK: return 0xfe00u;
    case B64_TT: return 0xff00u;
    case B128_GH: return 0xf0u;      // changes the nibble: lanes of a group keep distinct / equal entries alike
    default: return 0u;
  }
}

template <int P, int WAVES, int DEP>
__global__ __launch_bounds__(64 * WAVES) void k(uint32_t* out, uint64_t* cyc, int iters) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  for (int i = threadIdx.x; i < 16384; i += blockDim.x) smem[i] = hash32(i);
  __syncthreads();
  const int lane = threadIdx.x & 63;
  uint32_t acc = lane;
  uint64_t t0 = 0;
  if (P == MIX) {
    uint32_t ob[16];
#pragma unroll
    for (int j = 0; j < 16; j++) ob[j] = (j % 5 == 4) ? base_off<B128_GH>(lane, j) : base_off<B32_TT>(lane, j);
    __syncthreads();
    t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; it++) {
      const uint32_t sel = DEP ? __builtin_amdgcn_readfirstlane(hash32(it + (acc & 1))) : hash32((uint32_t)it);
      uint32_t r[16];
#pragma unroll
      for (int j = 0; j < 16; j++) {
        if (j % 5 == 4) {
          const v4u32 v = ld128(ob[j] ^ (sel & 0xf0u));
          r[j] = v.x ^ v.w;
        } else {
          r[j] = ld32(ob[j] ^ (sel & 0xff00u));
        }
      }
#pragma unroll
      for (int j = 0; j < 16; j += 2) acc = xor3(acc, r[j], r[j + 1]);
    }
  } else {
    uint32_t ob[16];
#pragma unroll
    for (int j = 0; j < 16; j++) ob[j] = base_off<P>(lane, j);
    __syncthreads();
    t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; it++) {
      const uint32_t sel = (DEP ? __builtin_amdgcn_readfirstlane(hash32(it + (acc & 1))) : hash32((uint32_t)it)) & row_mask<P>();
      uint32_t r[16];
#pragma unroll
      for (int j = 0; j < 16; j++) {
        if (P == B64_TT) {
          const v2u32 v = ld64(ob[j] ^ sel);
          r[j] = v.x ^ v.y;
        } else if (P == B128_GH) {
          const v4u32 v = ld128(ob[j] ^ sel);
          r[j] = v.x ^ v.w;
        } else {
          r[j] = ld32(ob[j] ^ sel);
        }
      }
#pragma unroll
      for (int j = 0; j < 16; j += 2) acc = xor3(acc, r[j], r[j + 1]);
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  if (lane == 0) cyc[blockIdx.x * WAVES + (threadIdx.x >> 6)] = t1 - t0;
}

template <int P, int WAVES, int DEP>
void run(uint32_t* dout, uint64_t* dcyc, uint64_t* hcyc, int cus) {
  const int iters = 4096;
  const size_t lds = 160 * 1024;  // one workgroup per CU
  (void)hipFuncSetAttribute((const void*)k<P, WAVES, DEP>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL((k<P, WAVES, DEP>), dim3(cus), dim3(64 * WAVES), lds, 0, dout, dcyc, 64);  // warm-up
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL((k<P, WAVES, DEP>), dim3(cus), dim3(64 * WAVES), lds, 0, dout, dcyc, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  (void)hipMemcpy(hcyc, dcyc, sizeof(uint64_t) * cus * WAVES, hipMemcpyDeviceToHost);
  // the CU's span = its slowest wave's (all waves start together after the barrier)
  double span = 0;
  for (int c = 0; c < cus; c++) {
    uint64_t m = 0;
    for (int w = 0; w < WAVES; w++) m = hcyc[c * WAVES + w] > m ? hcyc[c * WAVES + w] : m;
    span += (double)m;
  }
  span /= cus;
  const double instr = (double)WAVES * iters * 16;  // LDS wave-instructions per CU
  const double doc = P == B128_GH ? 4.0 : P == MIX ? (12 * 2.0 + 4 * 4.0) / 16 : 2.0;
  printf("{\"pattern\": \"%s\", \"dependent\": %d, \"waves_per_cu\": %d, \"ms\": %.4f, \"cycles_per_lds_instr\": %.3f, "
         "\"documented\": %.2f, \"frac_of_documented_rate\": %.3f, \"sclk_MHz\": %.0f}\n",
         kNames[P], DEP, WAVES, ms, span / instr, doc, doc / (span / instr), span / (ms * 1e3));
  fflush(stdout);
}

template <int P>
void sweep(uint32_t* dout, uint64_t* dcyc, uint64_t* hcyc, int cus) {
  run<P, 4, 0>(dout, dcyc, hcyc, cus);
  run<P, 8, 0>(dout, dcyc, hcyc, cus);
  run<P, 12, 0>(dout, dcyc, hcyc, cus);
  run<P, 16, 0>(dout, dcyc, hcyc, cus);
  run<P, 12, 1>(dout, dcyc, hcyc, cus);
  run<P, 16, 1>(dout, dcyc, hcyc, cus);
}

int main() {
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, 0);
  const int cus = prop.multiProcessorCount;
  uint32_t* dout;
  uint64_t* dcyc;
  (void)hipMalloc(&dout, (size_t)cus * 1024 * 4);
  (void)hipMalloc(&dcyc, (size_t)cus * 16 * 8);
  uint64_t* hcyc = (uint64_t*)malloc((size_t)cus * 16 * 8);
  sweep<B32_TT>(dout, dcyc, hcyc, cus);
  sweep<B32_LIN>(dout, dcyc, hcyc, cus);
  sweep<B32_BCAST>(dout, dcyc, hcyc, cus);
  sweep<B32_64BANK>(dout, dcyc, hcyc, cus);
  sweep<B64_TT>(dout, dcyc, hcyc, cus);
  sweep<B128_GH>(dout, dcyc, hcyc, cus);
  sweep<MIX>(dout, dcyc, hcyc, cus);
  free(hcyc);
  return 0;
}
