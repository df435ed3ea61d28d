// Latency floor of one Cipher-trait call on this box, through the C ABI (no Python): the median
// microseconds of (a) an empty kernel launch + hipStreamSynchronize, (b) an empty kernel launch
// whose one lane writes a flag into mapped pinned memory that the host spins on, (c) the same flag
// written by hipStreamWriteValue32 behind the kernel, (d) a one-key install waited for by a stream sync
// and by atls_engine_sync, (e) atls_seal /
// atls_open of one record (ChaCha20-Poly1305 and AES-128-GCM, 1,537 and 16,385 B), (g) the round trip of a
// resident wave polling a doorbell in mapped memory. Prints JSON. Run with ATLS_SINGLE_RESIDENT=1 the
// ChaCha20-Poly1305 calls that fit the argument block go through the resident server.
// Build: hipcc --offload-arch=gfx950 -O2 -Iinclude tools/single_call_floor.hip -Lanothertls_amd -latls
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../include/atls.h"

__global__ void empty_kernel(volatile uint32_t* flag, uint32_t v) {
  if (flag && threadIdx.x == 0) {
    __threadfence_system();
    *flag = v;
  }
}

// (e) the same flag kernel with an argument block the size of the single-call kernels' (gcm_single /
// chacha_single: descriptor + 3,584 inline bytes): the cost of carrying the record in the launch
struct BigArgs {
  uint32_t* flag;
  uint32_t v;
  uint8_t bytes[3712];
};
__global__ void empty_kernel_big(BigArgs a) {
  if (threadIdx.x == 0) {
    __threadfence_system();
    *(volatile uint32_t*)a.flag = a.v + a.bytes[3711];
  }
}

// (g) a resident wave instead of a launch per call: the kernel stays on one CU polling a
// doorbell word in mapped, coherent host memory (s_sleep between polls); for request v it reads `nbytes`
// of request data from mapped host memory (the record a call would hand over), writes them back to a
// mapped reply area and raises the flag to v. It leaves on the stop value, or after `idle_ms` without a
// request -- an exit every wave reaches whatever the host does.
__global__ void doorbell_server(const uint32_t* bell, uint32_t* flag, const uint4* req, uint4* rep, uint32_t nbytes,
                                uint32_t idle_ms) {
  uint32_t last = 0;
  unsigned long long t_last = __builtin_amdgcn_s_memrealtime();
  for (;;) {
    const uint32_t v = __hip_atomic_load(bell, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
    if (v == 0xffffffffu) break;
    if (v == last) {
      if (__builtin_amdgcn_s_memrealtime() - t_last > 100000ull * idle_ms) break;  // 100 MHz ticks
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    last = v;
    for (uint32_t i = threadIdx.x; i < nbytes / 16; i += blockDim.x) rep[i] = req[i];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (threadIdx.x == 0) __hip_atomic_store(flag, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    t_last = __builtin_amdgcn_s_memrealtime();
  }
}

template <typename F>
double median_us(F f, int reps) {
  f();
  std::vector<double> t;
  for (int i = 0; i < reps; i++) {
    auto a = std::chrono::steady_clock::now();
    f();
    t.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count());
  }
  std::sort(t.begin(), t.end());
  return t[t.size() / 2];
}

int main() {
  hipStream_t s;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return 1;
  uint32_t* flag = nullptr;
  if (hipHostMalloc((void**)&flag, 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return 1;
  uint32_t* dflag = nullptr;
  (void)hipHostGetDevicePointer((void**)&dflag, flag, 0);
  *flag = 0;
  const double sync_us = median_us([&] {
    hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s, nullptr, 0u);
    (void)hipStreamSynchronize(s);
  }, 2000);
  uint32_t it = 0;
  const double spin_us = median_us([&] {
    ++it;
    hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s, dflag, it);
    while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != it) {
    }
  }, 2000);
  (void)hipStreamSynchronize(s);
  // (c) the flag written by the command processor after the kernel (hipStreamWriteValue32)
  const double wv_us = median_us([&] {
    ++it;
    hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s, nullptr, 0u);
    if (hipStreamWriteValue32(s, dflag, it, 0) != hipSuccess) abort();
    while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != it) {
    }
  }, 2000);
  (void)hipStreamSynchronize(s);
  BigArgs big;
  memset(&big, 0, sizeof big);
  big.flag = dflag;
  const double big_us = median_us([&] {
    ++it;
    big.v = it;
    hipLaunchKernelGGL(empty_kernel_big, dim3(1), dim3(64), 0, s, big);
    while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != it) {
    }
  }, 2000);
  (void)hipStreamSynchronize(s);
  printf("{\"empty_launch_sync_us\": %.1f, \"empty_launch_flag_spin_us\": %.1f, \"empty_launch_writevalue_spin_us\": %.1f, "
         "\"empty_launch_3712B_args_flag_spin_us\": %.1f",
         sync_us, spin_us, wv_us, big_us);
  // (g) the doorbell round trip of a resident wave: no payload, and a 1,552-byte record each way
  {
    uint8_t* blk = nullptr;  // [0] bell, [64] flag, [4096..] request, [8192..] reply
    if (hipHostMalloc((void**)&blk, 16384, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) abort();
    memset(blk, 0, 16384);
    uint8_t* dblk = nullptr;
    (void)hipHostGetDevicePointer((void**)&dblk, blk, 0);
    auto* bell = (uint32_t*)blk;
    auto* fl = (uint32_t*)(blk + 64);
    hipStream_t ps;
    if (hipStreamCreateWithFlags(&ps, hipStreamNonBlocking) != hipSuccess) abort();
    for (uint32_t nb : {0u, 1552u}) {
      __atomic_store_n(bell, 0u, __ATOMIC_RELEASE);
      __atomic_store_n(fl, 0u, __ATOMIC_RELEASE);
      hipLaunchKernelGGL(doorbell_server, dim3(1), dim3(64), 0, ps, (const uint32_t*)dblk, (uint32_t*)(dblk + 64),
                         (const uint4*)(dblk + 4096), (uint4*)(dblk + 8192), nb, 2000u);
      uint32_t v = 0;
      const double db = median_us([&] {
        ++v;
        for (uint32_t i = 0; i < nb; i += 64) blk[4096 + i] = (uint8_t)v;  // the request data changes per call
        __atomic_store_n(bell, v, __ATOMIC_RELEASE);
        auto t0 = std::chrono::steady_clock::now();
        while (__atomic_load_n(fl, __ATOMIC_ACQUIRE) != v) {
          if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(1)) abort();  // the server left
        }
      }, 2000);
      __atomic_store_n(bell, 0xffffffffu, __ATOMIC_RELEASE);
      if (hipStreamSynchronize(ps) != hipSuccess) abort();
      if (nb && blk[8192] != (uint8_t)v) abort();
      printf(", \"resident_wave_doorbell_%uB_us\": %.1f", nb, db);
    }
    (void)hipStreamDestroy(ps);
    (void)hipHostFree(blk);
  }
  // (f) a new key: atls_update_keys of one AES-128 / AES-256 slot (key-setup kernel, the key in the launch
  // arguments), then a wait on the engine stream -- the end-to-end cost of a connection's new key
  for (int kl : {16, 32}) {
    atls_engine* e = atls_engine_create(0);
    if (!e) abort();
    std::vector<atls_key> ks(64);
    for (size_t i = 0; i < ks.size(); i++) {
      memset(&ks[i], 0, sizeof ks[i]);
      ks[i].suite = kl == 16 ? ATLS_TLS_AES_128_GCM_SHA256 : ATLS_TLS_AES_256_GCM_SHA384;
      ks[i].key_len = (uint8_t)kl;
      ks[i].iv_len = 12;
      for (int b = 0; b < 32; b++) ks[i].key[b] = (uint8_t)(i * 31 + b);
    }
    if (atls_set_keys(e, ks.data(), (uint32_t)ks.size())) abort();
    hipStream_t es = (hipStream_t)atls_engine_stream(e);
    uint32_t slot = 0;
    const double up = median_us([&] {
      slot = (slot + 1) % 64;
      if (atls_update_keys(e, slot, &ks[slot], 1)) abort();
      (void)hipStreamSynchronize(es);
    }, 2000);
    printf("%s\"aes%d_update1_stream_sync_us\": %.1f", kl == 16 ? ", " : ", ", kl * 8, up);
    // the same through the engine's own wait (atls_engine_sync: a completion flag in mapped memory)
    const double upe = median_us([&] {
      slot = (slot + 1) % 64;
      if (atls_update_keys(e, slot, &ks[slot], 1)) abort();
      if (atls_engine_sync(e)) abort();
    }, 2000);
    printf(", \"aes%d_update1_engine_sync_us\": %.1f", kl * 8, upe);
    atls_engine_destroy(e);
  }
  std::vector<uint8_t> key(32, 7), iv(12, 1), aad = {0x17, 3, 3, 0x06, 0x11}, tag(16);
  for (uint16_t suite : {(uint16_t)ATLS_TLS_CHACHA20_POLY1305_SHA256, (uint16_t)ATLS_TLS_AES_128_GCM_SHA256}) {
    const size_t kl = suite == ATLS_TLS_AES_128_GCM_SHA256 ? 16 : 32;
    for (size_t n : {(size_t)1537, (size_t)16385}) {
      std::vector<uint8_t> pt(n, 0x5a), ct(n), back(n);
      const double seal = median_us([&] {
        if (atls_seal(suite, key.data(), kl, iv.data(), 12, aad.data(), 5, pt.data(), n, ct.data(), tag.data())) abort();
      }, 2000);
      const double open = median_us([&] {
        if (atls_open(suite, key.data(), kl, iv.data(), 12, aad.data(), 5, ct.data(), n, tag.data(), 16, back.data()))
          abort();
      }, 2000);
      if (back != pt) abort();
      printf(", \"%s_%zu_seal_us\": %.1f, \"%s_%zu_open_us\": %.1f", kl == 16 ? "aes128gcm" : "chacha20poly1305", n, seal,
             kl == 16 ? "aes128gcm" : "chacha20poly1305", n, open);
    }
  }
  const char* rm = getenv("ATLS_SINGLE_RESIDENT");
  printf(", \"single_resident\": %s}\n", rm && atoi(rm) ? "true" : "false");
  return 0;
}
