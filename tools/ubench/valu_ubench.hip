// Microbenchmark: VALU issue rate of v_xor_b32 (VOP2), v_bitop3_b32 / v_xor3 (VOP3) and
// v_alignbit_b32 on gfx950, 16 independent chains per lane, and the shader clock under load
// (s_memtime delta / wall time).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

template <int OP>
__global__ __launch_bounds__(256) void k(uint32_t* out, unsigned long long* clk, int iters) {
  uint32_t a[16];
#pragma unroll
  for (int i = 0; i < 16; i++) a[i] = threadIdx.x * (i + 1) + blockIdx.x;
  uint32_t b = threadIdx.x ^ 0x1234567u, c = threadIdx.x * 77u;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int u = 0; u < 8; u++)
#pragma unroll
      for (int i = 0; i < 16; i++) {
        if (OP == 0) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
        if (OP == 1) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a[i]) : "v"(b), "v"(c));
        if (OP == 2) asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(a[i]) : "v"(b));
        if (OP == 3) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
        if (OP == 5) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a[i]) : "v"(b));
        if (OP == 6) asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(a[i]) : "v"(b));
        if (OP == 7) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
        if (OP == 8) { uint64_t t; asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(t) : "v"(a[i]), "v"(b)); a[i] = (uint32_t)t ^ (uint32_t)(t >> 32); }
        if (OP == 9) asm volatile("v_bfe_i32 %0, %0, %1, 1" : "+v"(a[i]) : "v"(b));
        if (OP == 10) asm volatile("v_lshrrev_b64 %0, 3, %0" : "+v"(*(uint64_t*)&a[i & ~1]));
        if (OP == 11) asm volatile("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2" : "+v"(a[i]) : "v"(b));
        if (OP == 12) asm volatile("v_lshlrev_b32_sdwa %0, 4, %1 dst_sel:BYTE_0 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:BYTE_1" : "+v"(a[i]) : "v"(b));
        if (OP == 13) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
        if (OP == 14) asm volatile("v_lshl_or_b32 %0, %0, 3, %1" : "+v"(a[i]) : "v"(b));
        if (OP == 15) asm volatile("v_xor_b32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:WORD_1" : "+v"(a[i]) : "v"(b));
        if (OP == 4) { if (i & 1) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
                       else asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a[i]) : "v"(b), "v"(c)); }
      }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 16; i++) acc ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  if (threadIdx.x == 0 && blockIdx.x == 0) clk[0] = t1 - t0;
}

template <int OP>
void run(const char* name, uint32_t* dout, unsigned long long* dclk, int wg_per_cu) {
  const int grid = 256 * wg_per_cu, iters = 2000;
  hipLaunchKernelGGL(k<OP>, dim3(grid), dim3(256), 0, 0, dout, dclk, 10);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(k<OP>, dim3(grid), dim3(256), 0, 0, dout, dclk, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms; (void)hipEventElapsedTime(&ms, e0, e1);
  unsigned long long clk; (void)hipMemcpy(&clk, dclk, 8, hipMemcpyDeviceToHost);
  const double inst = (double)grid * 4 * iters * 8 * 16;  // wave-instructions
  const double per_cu_per_ns = inst / 256 / (ms * 1e6);
  printf("%-10s wg/cu=%d: %.3f ms, %.3f wave-instr/CU/ns, memtime %llu ticks (one wave) -> %.2f ticks/ns\n", name,
         wg_per_cu, ms, per_cu_per_ns, clk, clk / (ms * 1e6));
}

int main() {
  uint32_t* dout; unsigned long long* dclk;
  (void)hipMalloc(&dout, 256 * 16 * 256 * 4);
  (void)hipMalloc(&dclk, 64);
  for (int w : {2}) {
    run<0>("xor", dout, dclk, w);
    run<1>("bitop3", dout, dclk, w);
    run<2>("alignbit", dout, dclk, w);
    run<3>("perm", dout, dclk, w);
    run<5>("mul_u24", dout, dclk, w);
    run<6>("mulhi_u24", dout, dclk, w);
    run<7>("mul_lo_u32", dout, dclk, w);
    run<8>("mad_u64_u32", dout, dclk, w);
    run<9>("bfe_i32", dout, dclk, w);
    run<10>("lshr_b64", dout, dclk, w);
    run<11>("mov_sdwa", dout, dclk, w);
    run<12>("lshl_sdwa", dout, dclk, w);
    run<13>("and_or", dout, dclk, w);
    run<14>("lshl_or", dout, dclk, w);
    run<15>("xor_sdwa", dout, dclk, w);
  }
  return 0;
}
