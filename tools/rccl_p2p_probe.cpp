// Bracket the RCCL point-to-point size defect of round 4 (profiles/r04/multi_diag.log: a 2 GiB self
// send / recv came back wrong from byte 2^30 on). One GPU, a one-rank communicator (ncclCommInitAll),
// rank 0 sends to and receives from itself in one group, exactly as atls_multi's RCCL-self mode does;
// for every size the received bytes are compared with the sent ones on the device.
//
//   hipcc --offload-arch=gfx950 -O2 -std=c++17 -I/opt/rocm/include tools/rccl_p2p_probe.cpp -ldl -o tools/rccl_p2p_probe
//   tools/rccl_p2p_probe <librccl path> [size ...]     -> one JSON line per size
//
// The library path is explicit so both RCCLs of the image can be probed: the one PyTorch ships (which a
// process that imported torch resolves "librccl.so.1" to) and /opt/rocm's.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

namespace {

__global__ void fill(uint32_t* p, size_t n_words, uint32_t salt) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n_words; i += (size_t)gridDim.x * blockDim.x) {
    uint64_t x = (i + salt) * 0x9E3779B97F4A7C15ull;  // a different word at every offset
    x ^= x >> 29;
    p[i] = (uint32_t)x;
  }
}

// bad[0] = mismatching words, bad[1] = the first mismatching word index (or ~0)
__global__ void compare(const uint32_t* a, const uint32_t* b, size_t n_words, unsigned long long* bad) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n_words; i += (size_t)gridDim.x * blockDim.x)
    if (a[i] != b[i]) {
      atomicAdd(&bad[0], 1ull);
      atomicMin(&bad[1], (unsigned long long)i);
    }
}

#define CK(x)                                                         \
  do {                                                                \
    if ((x) != hipSuccess) {                                          \
      std::fprintf(stderr, "HIP error %d at line %d\n", (int)(x), __LINE__); \
      return 1;                                                       \
    }                                                                 \
  } while (0)

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s <librccl path> [bytes ...]\n", argv[0]);
    return 2;
  }
  void* h = dlopen(argv[1], RTLD_NOW | RTLD_LOCAL);
  if (!h) {
    std::fprintf(stderr, "dlopen %s: %s\n", argv[1], dlerror());
    return 1;
  }
  auto get_version = reinterpret_cast<decltype(&ncclGetVersion)>(dlsym(h, "ncclGetVersion"));
  auto init_all = reinterpret_cast<decltype(&ncclCommInitAll)>(dlsym(h, "ncclCommInitAll"));
  auto destroy = reinterpret_cast<decltype(&ncclCommDestroy)>(dlsym(h, "ncclCommDestroy"));
  auto gstart = reinterpret_cast<decltype(&ncclGroupStart)>(dlsym(h, "ncclGroupStart"));
  auto gend = reinterpret_cast<decltype(&ncclGroupEnd)>(dlsym(h, "ncclGroupEnd"));
  auto send = reinterpret_cast<decltype(&ncclSend)>(dlsym(h, "ncclSend"));
  auto recv = reinterpret_cast<decltype(&ncclRecv)>(dlsym(h, "ncclRecv"));
  if (!get_version || !init_all || !destroy || !gstart || !gend || !send || !recv) {
    std::fprintf(stderr, "missing RCCL symbols in %s\n", argv[1]);
    return 1;
  }
  int version = 0;
  get_version(&version);
  std::vector<size_t> sizes;
  for (int i = 2; i < argc; i++) sizes.push_back(std::strtoull(argv[i], nullptr, 0));
  if (sizes.empty()) {
    const size_t G = 1ull << 30;
    sizes = {G - 4096, G, G + 4096, G + (256ull << 20), G + (512ull << 20), 2 * G - 4096, 2 * G};
  }
  size_t max_size = 0;
  for (size_t s : sizes) max_size = s > max_size ? s : max_size;
  CK(hipSetDevice(0));
  uint32_t *src = nullptr, *dst = nullptr;
  unsigned long long* bad = nullptr;
  CK(hipMalloc(&src, max_size + 4));
  CK(hipMalloc(&dst, max_size + 4));
  CK(hipMalloc(&bad, 16));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  ncclComm_t comm;
  const int dev0 = 0;
  if (init_all(&comm, 1, &dev0) != ncclSuccess) {
    std::fprintf(stderr, "ncclCommInitAll failed\n");
    return 1;
  }
  int rc = 0;
  for (size_t n : sizes) {
    const size_t words = (n + 3) / 4;
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, s, src, words, (uint32_t)n);
    CK(hipMemsetAsync(dst, 0, words * 4, s));
    const unsigned long long init[2] = {0ull, ~0ull};
    CK(hipMemcpyAsync(bad, init, 16, hipMemcpyHostToDevice, s));
    CK(hipStreamSynchronize(s));
    ncclResult_t r1 = gstart();
    ncclResult_t r2 = send(src, n, ncclUint8, 0, comm, s);
    ncclResult_t r3 = recv(dst, n, ncclUint8, 0, comm, s);
    ncclResult_t r4 = gend();
    CK(hipStreamSynchronize(s));
    hipLaunchKernelGGL(compare, dim3(4096), dim3(256), 0, s, src, dst, n / 4, bad);  // whole words only
    unsigned long long hb[2];
    CK(hipMemcpyAsync(hb, bad, 16, hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    const bool ok = r1 == ncclSuccess && r2 == ncclSuccess && r3 == ncclSuccess && r4 == ncclSuccess && hb[0] == 0;
    std::printf("{\"rccl_version\": %d, \"bytes\": %zu, \"bytes_minus_2^30\": %lld, \"rc\": [%d, %d, %d, %d], "
                "\"bad_words\": %llu, \"first_bad_byte\": %lld, \"ok\": %s}\n",
                version, n, (long long)n - (1ll << 30), (int)r1, (int)r2, (int)r3, (int)r4, hb[0],
                hb[0] ? (long long)(hb[1] * 4) : -1ll, ok ? "true" : "false");
    std::fflush(stdout);
    if (!ok) rc = 3;
  }
  destroy(comm);
  (void)hipFree(src);
  (void)hipFree(dst);
  (void)hipFree(bad);
  return rc == 3 ? 0 : rc;  // a wrong transfer is a finding, not a tool failure
}
