// The AES block cipher itself, AES::encrypt / AES::decrypt (crypto/aes/cipher.rs:175-215), over
// many independent 16-byte blocks under one key slot (ECB). Not on the record path -- GCM only
// ever encrypts -- but part of the reference's AES API, so it runs on the device
// too. One thread per block, byte-oriented rounds with the S-box and its inverse in LDS
// (FIPS-197 §5.1 / §5.3, the same round structure as cipher.rs), round keys from the key slot's
// schedule (keysetup.hip).
#include "aes_sbox.h"
#include "atls_dev.h"

namespace atls {

__device__ __forceinline__ uint8_t rk_byte(const uint32_t* rk, int r, int i) {
  return (uint8_t)(rk[4 * r + (i >> 2)] >> (8 * (i & 3)));
}

template <bool DEC>
__global__ __launch_bounds__(256) void aes_block_kernel(const KeySched* __restrict__ k, const uint8_t* __restrict__ in,
                                                        uint8_t* __restrict__ out, uint64_t nblocks,
                                                        uint32_t* __restrict__ err) {
  __shared__ uint8_t sbox[256], inv[256];
  {
    const int x = threadIdx.x;
    const uint8_t s = kSbox[x];
    sbox[x] = s;
    inv[s] = (uint8_t)x;  // InvSubBytes table (FIPS-197 Fig. 14)
  }
  __syncthreads();
  const uint32_t suite = k->suite;
  if (!k->valid || (suite != (uint32_t)kSuiteAes128 && suite != (uint32_t)kSuiteAes256)) {
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(err, 1u);
    return;
  }
  const int nr = (int)k->nr;
  const uint32_t* rk = k->rk;  // wave-uniform: scalar loads per round
  for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < nblocks;
       b += (uint64_t)gridDim.x * blockDim.x) {
    uint8_t s[16];
    const uint4 v = ld16(in + 16 * b);
    const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 16; i++) s[i] = (uint8_t)(w4[i >> 2] >> (8 * (i & 3)));
    if (!DEC) {  // cipher.rs:175-194
#pragma unroll
      for (int i = 0; i < 16; i++) s[i] ^= rk_byte(rk, 0, i);
      for (int r = 1; r <= nr; r++) {
        uint8_t t[16];
#pragma unroll
        for (int c = 0; c < 4; c++)  // SubBytes + ShiftRows
#pragma unroll
          for (int row = 0; row < 4; row++) t[4 * c + row] = sbox[s[4 * ((c + row) & 3) + row]];
        if (r < nr) {  // MixColumns
#pragma unroll
          for (int c = 0; c < 4; c++) {
            const uint8_t a0 = t[4 * c], a1 = t[4 * c + 1], a2 = t[4 * c + 2], a3 = t[4 * c + 3];
            const uint8_t x = a0 ^ a1 ^ a2 ^ a3;
            t[4 * c] = a0 ^ x ^ xtime(a0 ^ a1);
            t[4 * c + 1] = a1 ^ x ^ xtime(a1 ^ a2);
            t[4 * c + 2] = a2 ^ x ^ xtime(a2 ^ a3);
            t[4 * c + 3] = a3 ^ x ^ xtime(a3 ^ a0);
          }
        }
#pragma unroll
        for (int i = 0; i < 16; i++) s[i] = t[i] ^ rk_byte(rk, r, i);
      }
    } else {  // cipher.rs:196-215, the inverse cipher (FIPS-197 §5.3)
#pragma unroll
      for (int i = 0; i < 16; i++) s[i] ^= rk_byte(rk, nr, i);
      for (int r = nr - 1; r >= 0; r--) {
        uint8_t t[16];
#pragma unroll
        for (int c = 0; c < 4; c++)  // InvShiftRows + InvSubBytes
#pragma unroll
          for (int row = 0; row < 4; row++) t[4 * c + row] = inv[s[4 * ((c - row) & 3) + row]];
#pragma unroll
        for (int i = 0; i < 16; i++) t[i] ^= rk_byte(rk, r, i);
        if (r > 0) {  // InvMixColumns = MixColumns after the {04}-multiple pre-step
#pragma unroll
          for (int c = 0; c < 4; c++) {
            const uint8_t u = xtime(xtime(t[4 * c] ^ t[4 * c + 2]));
            const uint8_t w = xtime(xtime(t[4 * c + 1] ^ t[4 * c + 3]));
            const uint8_t a0 = t[4 * c] ^ u, a1 = t[4 * c + 1] ^ w, a2 = t[4 * c + 2] ^ u, a3 = t[4 * c + 3] ^ w;
            const uint8_t x = a0 ^ a1 ^ a2 ^ a3;
            t[4 * c] = a0 ^ x ^ xtime(a0 ^ a1);
            t[4 * c + 1] = a1 ^ x ^ xtime(a1 ^ a2);
            t[4 * c + 2] = a2 ^ x ^ xtime(a2 ^ a3);
            t[4 * c + 3] = a3 ^ x ^ xtime(a3 ^ a0);
          }
        }
#pragma unroll
        for (int i = 0; i < 16; i++) s[i] = t[i];
      }
    }
    uint32_t o[4] = {0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < 16; i++) o[i >> 2] |= (uint32_t)s[i] << (8 * (i & 3));
    st16(out + 16 * b, make_uint4(o[0], o[1], o[2], o[3]));
  }
}

}  // namespace atls

// nblocks blocks of in -> out under key slot ks (device pointers); err gets bit 0 when the slot
// is not an AES key. grid: workgroups (256 threads each).
extern "C" int atls_launch_aes_blocks(int decrypt, const void* ks, const uint8_t* in, uint8_t* out, uint64_t nblocks,
                                      uint32_t* err, int grid, hipStream_t s) {
  if (nblocks == 0) return 0;
  const uint64_t want = (nblocks + 255) / 256;
  const int g = (int)(want < (uint64_t)grid ? want : (uint64_t)grid);
  if (decrypt)
    hipLaunchKernelGGL(atls::aes_block_kernel<true>, dim3(g), dim3(256), 0, s, (const atls::KeySched*)ks, in, out,
                       nblocks, err);
  else
    hipLaunchKernelGGL(atls::aes_block_kernel<false>, dim3(g), dim3(256), 0, s, (const atls::KeySched*)ks, in, out,
                       nblocks, err);
  return hipGetLastError() == hipSuccess ? 0 : ATLS_INTERNAL_ERROR;
}
