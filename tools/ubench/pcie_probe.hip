// PCIe probe (round 3): what the host link gives a batch that starts and ends in pinned host memory.
// 1 GiB each way, pinned (hipHostMalloc) buffers:
//   dma_h2d / dma_d2h       one hipMemcpyAsync per direction, alone
//   dma_both                both directions at once on two streams
//   dma_chunk32             the engine's pipeline shape: 32 MiB chunks, H2D + D2H per chunk, alternating
//                           two streams (run_host_pipelined without the kernel)
//   zc_read / zc_write      a kernel reading host memory into HBM / writing HBM into host memory
//                           (16-B loads / stores per lane, mapped pinned memory)
//   zc_both                 both kernels at once on two streams
//   dma_d2h_2d / dma_h2d_2d C2's record layout (65,536 rows of 16,385 B at a 16,400-B pitch) copied
//                           with hipMemcpy2DAsync, one call, and in 32 MiB chunks (2,048 rows each)
// Rates are GB/s per direction (1e9 B/s).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ __launch_bounds__(256) void copy16(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n16) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += 4 * stride) {
    uint4 v[4];
#pragma unroll
    for (int u = 0; u < 4; u++) if (i + u * stride < n16) v[u] = src[i + u * stride];
#pragma unroll
    for (int u = 0; u < 4; u++) if (i + u * stride < n16) dst[i + u * stride] = v[u];
  }
}

static float timed(hipStream_t s0, hipStream_t s1, void (*fn)(void*), void* ctx) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a, s0));
  CK(hipStreamWaitEvent(s1, a, 0));
  fn(ctx);
  hipEvent_t c;
  CK(hipEventCreate(&c));
  CK(hipEventRecord(c, s1));
  CK(hipStreamWaitEvent(s0, c, 0));
  CK(hipEventRecord(b, s0));
  CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  return ms;
}

struct Ctx {
  uint8_t *h_in, *h_out, *d_in, *d_out, *hd_in, *hd_out;
  size_t n;
  hipStream_t s0, s1;
  int grid;
};
static Ctx C;

static void f_h2d(void*) { CK(hipMemcpyAsync(C.d_in, C.h_in, C.n, hipMemcpyHostToDevice, C.s0)); }
static void f_d2h(void*) { CK(hipMemcpyAsync(C.h_out, C.d_out, C.n, hipMemcpyDeviceToHost, C.s0)); }
static void f_both(void*) {
  CK(hipMemcpyAsync(C.d_in, C.h_in, C.n, hipMemcpyHostToDevice, C.s0));
  CK(hipMemcpyAsync(C.h_out, C.d_out, C.n, hipMemcpyDeviceToHost, C.s1));
}
static size_t g_chunk = 32u << 20;
static void f_chunk(void*) {
  int c = 0;
  for (size_t o = 0; o < C.n; o += g_chunk, c ^= 1) {
    hipStream_t s = c ? C.s1 : C.s0;
    const size_t m = C.n - o < g_chunk ? C.n - o : g_chunk;
    CK(hipMemcpyAsync(C.d_in + o, C.h_in + o, m, hipMemcpyHostToDevice, s));
    CK(hipMemcpyAsync(C.h_out + o, C.d_out + o, m, hipMemcpyDeviceToHost, s));
  }
}
static const size_t kW = 16385, kP = 16400, kRows = 65536;
static void f_d2h_2d(void*) { CK(hipMemcpy2DAsync(C.h_out, kP, C.d_out, kP, kW, kRows, hipMemcpyDeviceToHost, C.s0)); }
static void f_h2d_2d(void*) { CK(hipMemcpy2DAsync(C.d_in, kP, C.h_in, kP, kW, kRows, hipMemcpyHostToDevice, C.s0)); }
static void f_d2h_2d_chunk(void*) {
  for (size_t r = 0; r < kRows; r += 2048)
    CK(hipMemcpy2DAsync(C.h_out + r * kP, kP, C.d_out + r * kP, kP, kW, 2048, hipMemcpyDeviceToHost, C.s0));
}
static void f_zc_read(void*) {
  hipLaunchKernelGGL(copy16, dim3(C.grid), dim3(256), 0, C.s0, (const uint4*)C.hd_in, (uint4*)C.d_in, C.n / 16);
}
static void f_zc_write(void*) {
  hipLaunchKernelGGL(copy16, dim3(C.grid), dim3(256), 0, C.s0, (const uint4*)C.d_out, (uint4*)C.hd_out, C.n / 16);
}
static void f_zc_both(void*) {
  hipLaunchKernelGGL(copy16, dim3(C.grid), dim3(256), 0, C.s0, (const uint4*)C.hd_in, (uint4*)C.d_in, C.n / 16);
  hipLaunchKernelGGL(copy16, dim3(C.grid), dim3(256), 0, C.s1, (const uint4*)C.d_out, (uint4*)C.hd_out, C.n / 16);
}

int main() {
  C.n = (size_t)1 << 30;
  const size_t alloc = C.n + (16u << 20);  // the 2-D layout spans 65,536 x 16,400 B > 1 GiB
  static_assert(16400ull * 65536ull <= (1ull << 30) + (16ull << 20), "2-D layout fits the buffers");
  CK(hipHostMalloc(&C.h_in, alloc, hipHostMallocMapped));
  CK(hipHostMalloc(&C.h_out, alloc, hipHostMallocMapped));
  CK(hipMalloc(&C.d_in, alloc));
  CK(hipMalloc(&C.d_out, alloc));
  CK(hipHostGetDevicePointer((void**)&C.hd_in, C.h_in, 0));
  CK(hipHostGetDevicePointer((void**)&C.hd_out, C.h_out, 0));
  for (size_t i = 0; i < C.n; i += 4096) C.h_in[i] = (uint8_t)i;
  CK(hipMemset(C.d_out, 1, C.n));
  CK(hipStreamCreateWithFlags(&C.s0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&C.s1, hipStreamNonBlocking));
  struct { const char* name; void (*fn)(void*); int dirs; } T[] = {
      {"dma_h2d", f_h2d, 1}, {"dma_d2h", f_d2h, 1}, {"dma_both", f_both, 2}, {"dma_chunk32", f_chunk, 2},
      {"zc_read", f_zc_read, 1}, {"zc_write", f_zc_write, 1}, {"zc_both", f_zc_both, 2}};
  for (int grid : {256, 1024, 4096}) {
    C.grid = grid;
    for (auto& t : T) {
      if (grid != 1024 && t.name[0] == 'd') continue;
      timed(C.s0, C.s1, t.fn, nullptr);  // warm-up
      float best = 1e9f;
      for (int r = 0; r < 3; r++) { const float ms = timed(C.s0, C.s1, t.fn, nullptr); best = ms < best ? ms : best; }
      printf("%-12s grid=%-5d %8.3f ms  %6.1f GB/s per direction\n", t.name, grid, best, C.n / (best * 1e6));
    }
  }
  struct { const char* name; void (*fn)(void*); } T2[] = {
      {"dma_d2h_2d", f_d2h_2d}, {"dma_h2d_2d", f_h2d_2d}, {"dma_d2h_2dchunk", f_d2h_2d_chunk}};
  for (auto& t : T2) {
    timed(C.s0, C.s1, t.fn, nullptr);
    float best = 1e9f;
    for (int r = 0; r < 3; r++) { const float ms = timed(C.s0, C.s1, t.fn, nullptr); best = ms < best ? ms : best; }
    printf("%-16s %8.3f ms  %6.1f GB/s (record bytes)\n", t.name, best, kW * kRows / (best * 1e6));
  }
  for (size_t mb : {8, 16, 64, 128}) {
    g_chunk = mb << 20;
    timed(C.s0, C.s1, f_chunk, nullptr);
    float best = 1e9f;
    for (int r = 0; r < 3; r++) { const float ms = timed(C.s0, C.s1, f_chunk, nullptr); best = ms < best ? ms : best; }
    printf("dma_chunk%-3zu %8.3f ms  %6.1f GB/s per direction\n", mb, best, C.n / (best * 1e6));
  }
  return 0;
}
