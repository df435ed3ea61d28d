// Microbenchmark (round 3): VALU issue rates of the operations a ChaCha20 quarter-round and a
// Poly1305 product could be built from on gfx950, 16 independent chains per lane, 2 workgroups of
// 4 waves per CU (as valu_ubench.hip). Question: is a 16-bit half swap by `v_pk_add_u16` with
// op_sel (rotl16) cheaper than `v_alignbit_b32` (half rate), and what do v_add3 / v_xad / v_fma_f64
// cost next to v_mad_u64_u32 (quarter rate)?
// Second part: a whole ChaCha20 block (20 rounds, 16 words per lane, 2 blocks per lane for ILP) with
// the rotations as alignbit everywhere vs rotl16 as a packed half swap, same instruction stream
// otherwise, at 2 and 3 waves per SIMD.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

template <int OP>
__global__ __launch_bounds__(256) void k(uint32_t* out, int iters) {
  uint32_t a[16];
#pragma unroll
  for (int i = 0; i < 16; i++) a[i] = threadIdx.x * (i + 1) + blockIdx.x;
  uint32_t b = threadIdx.x ^ 0x1234567u, c = threadIdx.x * 77u;
  double f[8];
#pragma unroll
  for (int i = 0; i < 8; i++) f[i] = (double)(threadIdx.x + i);
  const double fb = 1.0000001, fc = 0.5;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int u = 0; u < 8; u++)
#pragma unroll
      for (int i = 0; i < 16; i++) {
        if (OP == 0) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
        if (OP == 1) asm volatile("v_pk_add_u16 %0, %0, 0 op_sel:[1,0] op_sel_hi:[0,1]" : "+v"(a[i]));
        if (OP == 2) asm volatile("v_alignbit_b32 %0, %0, %0, 16" : "+v"(a[i]));
        if (OP == 3) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
        if (OP == 4) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
        if (OP == 5) asm volatile("v_xad_u32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
        if (OP == 6) { if (i < 8) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(f[i]) : "v"(fb), "v"(fc)); }
        if (OP == 7) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(*(uint64_t*)&a[i & ~1]) : "v"(*(uint64_t*)&a[(i + 2) & 14]));
        if (OP == 8) asm volatile("v_mad_u32_u24 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
        if (OP == 9) asm volatile("v_lshlrev_b32 %0, 7, %0" : "+v"(a[i]));
        if (OP == 10) asm volatile("v_lshl_add_u32 %0, %0, 2, %1" : "+v"(a[i]) : "v"(b));
        if (OP == 11) asm volatile("v_bfi_b32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
        if (OP == 12) asm volatile("v_pk_lshlrev_b16 %0, 1, %0" : "+v"(a[i]));
        if (OP == 13) asm volatile("v_lshrrev_b32 %0, 25, %0" : "+v"(a[i]));
        if (OP == 14) { if (i < 8) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(f[i]) : "v"(fb)); }
        if (OP == 16) asm volatile("v_xor_b32_sdwa %0, %0, %1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0" : "+v"(a[i]) : "v"(b));
        if (OP == 17) asm volatile("v_add_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_0" : "+v"(a[i]) : "v"(b));
        if (OP == 15) { uint64_t t = ((uint64_t)a[(i + 1) & 15] << 32) | a[i];
                        asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(t) : "v"(b), "v"(c)); a[i] = (uint32_t)t; a[(i + 1) & 15] = (uint32_t)(t >> 32); }
      }
  }
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 16; i++) acc ^= a[i];
#pragma unroll
  for (int i = 0; i < 8; i++) acc ^= (uint32_t)(int64_t)f[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

__device__ __forceinline__ uint32_t rot_ab(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, 32 - n); }
__device__ __forceinline__ uint32_t rot16_pk(uint32_t x) {
  uint32_t r;
  asm("v_pk_add_u16 %0, %1, 0 op_sel:[1,0] op_sel_hi:[0,1]" : "=v"(r) : "v"(x));
  return r;
}
template <int MODE>
__device__ __forceinline__ uint32_t rot16(uint32_t x) { return MODE == 1 ? rot16_pk(x) : rot_ab(x, 16); }
// rotl16(d ^ a) as two SDWA xors (VOP2 encodings): the low half from the high halves, the high from the low
__device__ __forceinline__ uint32_t xrot16_sdwa(uint32_t d, uint32_t a) {
  uint32_t t;
  asm("v_xor_b32_sdwa %0, %1, %2 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_1\n\t"
      "v_xor_b32_sdwa %0, %1, %2 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0"
      : "=&v"(t) : "v"(d), "v"(a));
  return t;
}
template <int MODE>
__device__ __forceinline__ uint32_t xrot16(uint32_t d, uint32_t a) { return MODE == 2 ? xrot16_sdwa(d, a) : rot16<MODE>(d ^ a); }

#define QR(M, a, b, c, d)                  \
  a += b; d = xrot16<M>(d, a);              \
  c += d; b = rot_ab(b ^ c, 12);            \
  a += b; d = rot_ab(d ^ a, 8);             \
  c += d; b = rot_ab(b ^ c, 7);

// MODE 0: alignbit rotations; MODE 1: rotl16 as a packed half swap; MODE 2 (round 5): rotl16(d ^ a) as two
// SDWA xors.
template <int MODE, int MINW>
__global__ __launch_bounds__(256, MINW) void chacha_k(uint32_t* out, int iters) {
  uint32_t x[16], y[16];
#pragma unroll
  for (int i = 0; i < 16; i++) { x[i] = threadIdx.x * (i + 3) + blockIdx.x; y[i] = x[i] ^ 0x5a5a5a5au; }
  for (int it = 0; it < iters; it++) {
#pragma unroll 2
    for (int r = 0; r < 10; r++) {
      QR(MODE, x[0], x[4], x[8], x[12]) QR(MODE, x[1], x[5], x[9], x[13]) QR(MODE, x[2], x[6], x[10], x[14]) QR(MODE, x[3], x[7], x[11], x[15])
      QR(MODE, x[0], x[5], x[10], x[15]) QR(MODE, x[1], x[6], x[11], x[12]) QR(MODE, x[2], x[7], x[8], x[13]) QR(MODE, x[3], x[4], x[9], x[14])
    }
#pragma unroll
    for (int i = 0; i < 16; i++) x[i] += y[i];
  }
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 16; i++) acc ^= x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

static uint32_t* dout;

template <int OP>
void run(const char* name) {
  const int grid = 256 * 2, iters = 2000;
  hipLaunchKernelGGL(k<OP>, dim3(grid), dim3(256), 0, 0, dout, 10);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(k<OP>, dim3(grid), dim3(256), 0, 0, dout, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms; (void)hipEventElapsedTime(&ms, e0, e1);
  const int per = (OP == 6 || OP == 14) ? 8 : 16;
  const double inst = (double)grid * 4 * iters * 8 * per;  // wave-instructions
  printf("%-12s %.3f ms, %.3f wave-instr/CU/ns\n", name, ms, inst / 256 / (ms * 1e6));
}

template <int MODE, int MINW>
void run_chacha(const char* name, int wg_per_cu) {
  const int grid = 256 * wg_per_cu, iters = 200;
  hipLaunchKernelGGL((chacha_k<MODE, MINW>), dim3(grid), dim3(256), 0, 0, dout, 2);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL((chacha_k<MODE, MINW>), dim3(grid), dim3(256), 0, 0, dout, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms; (void)hipEventElapsedTime(&ms, e0, e1);
  const double blocks = (double)grid * 256 * iters;
  printf("%-22s wg/cu=%d: %.3f ms, %.1f CU-ns per 64 blocks, %.2f TB/s keystream\n", name, wg_per_cu, ms,
         ms * 1e6 * 256 / (blocks / 64), blocks * 64 / (ms * 1e-3) / 1e12);
}

int main() {
  (void)hipMalloc(&dout, 256 * 16 * 256 * 4);
  run<0>("xor");
  run<1>("pk_add_swap");
  run<2>("alignbit16");
  run<3>("add_u32");
  run<4>("add3_u32");
  run<5>("xad_u32");
  run<6>("fma_f64");
  run<14>("mul_f64");
  run<7>("lshl_add_u64");
  run<8>("mad_u32_u24");
  run<9>("lshlrev_b32");
  run<13>("lshrrev_b32");
  run<10>("lshl_add_u32");
  run<11>("bfi_b32");
  run<12>("pk_lshlrev16");
  run<15>("mad_u64_acc");
  run<16>("xor_sdwa_w1");
  run<17>("add_sdwa_w1w0");
  for (int w : {2, 3}) {
    run_chacha<0, 2>("chacha alignbit", w);
    run_chacha<1, 2>("chacha rot16 pk_add", w);
    run_chacha<2, 2>("chacha rot16 sdwa", w);
  }
  return 0;
}
