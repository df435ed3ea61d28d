// Diagnostic kernels (not on the record path).
//
// The shader clock under load. MI355X lowers its clock under sustained load by how much energy a kernel
// spends per cycle (MI355X_MICROARCH.md "DVFS give-back"), so the record kernels' rooflines in cycles
// (the LDS array for AES-GCM) need the clock they actually ran at. clock_probe_kernel
// is one wave per workgroup that sleeps until delay_us has passed on the 100 MHz constant clock
// (s_memrealtime), then reads the shader-clock counter (s_memtime) and the constant clock around
// spin_us more of sleeping. It uses no LDS and few registers, so launched on a second stream it
// lands on CUs beside a running batch kernel (a gcm_kernel workgroup leaves 20 of a CU's 32 wave
// slots and a quarter of each SIMD's registers free) and samples the clock those kernels run at.
// Every wave leaves after delay_us + spin_us (both capped by the launcher).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/atls.h"

namespace atls {

__global__ __launch_bounds__(64) void clock_probe_kernel(uint32_t delay_us, uint32_t spin_us,
                                                         unsigned long long* __restrict__ out) {
  const unsigned long long start = __builtin_amdgcn_s_memrealtime();
  unsigned long long r = start;
  while (r - start < 100ull * delay_us) {
    __builtin_amdgcn_s_sleep(16);
    r = __builtin_amdgcn_s_memrealtime();
  }
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  r = r0;
  while (r - r0 < 100ull * spin_us) {
    __builtin_amdgcn_s_sleep(16);
    r = __builtin_amdgcn_s_memrealtime();
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = t1 - t0;
    out[2 * blockIdx.x + 1] = r1 - r0;
  }
}

}  // namespace atls

// wgs one-wave workgroups on stream s; out: 2 x wgs u64 (device memory).
extern "C" int atls_launch_clock_probe(uint32_t wgs, uint32_t delay_us, uint32_t spin_us, uint64_t* out,
                                       hipStream_t s) {
  hipLaunchKernelGGL(atls::clock_probe_kernel, dim3(wgs), dim3(64), 0, s, delay_us, spin_us,
                     (unsigned long long*)out);
  return hipGetLastError() == hipSuccess ? 0 : ATLS_INTERNAL_ERROR;
}
