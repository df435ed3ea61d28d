"""CPU check of the bitsliced AES core (anothertls_amd/csrc/aes_bs.h) that the GCM kernel runs
on the VALU: compiled for the host with software v_bitop3_b32 / v_perm_b32, 32 random blocks
per key for AES-128/192/256 round keys from the oracle's key expansion (one key per lane, and two
keys split 16/16 across the plane bits), compared against the
oracle (literal restatement of crypto/aes/cipher.rs) block by block."""
import os
import random
import subprocess
import tempfile

import oracle as ora

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SRC = r"""
#include <stdint.h>
#include <stdio.h>
#define __device__
#define __forceinline__ inline
static uint32_t __builtin_amdgcn_bitop3_b32(uint32_t a, uint32_t b, uint32_t c, uint32_t tt) {
  uint32_t r = 0;
  for (int i = 0; i < 32; i++) {
    unsigned idx = (((a >> i) & 1) << 2) | (((b >> i) & 1) << 1) | ((c >> i) & 1);
    r |= ((tt >> idx) & 1u) << i;
  }
  return r;
}
static uint32_t __builtin_amdgcn_perm(uint32_t s0, uint32_t s1, uint32_t sel) {
  uint64_t d = ((uint64_t)s0 << 32) | s1;
  uint32_t r = 0;
  for (int i = 0; i < 4; i++) {
    unsigned b = (sel >> (8 * i)) & 0xff, v;
    if (b == 12) v = 0; else if (b >= 13) v = 0xff; else v = (d >> (8 * b)) & 0xff;
    r |= v << (8 * i);
  }
  return r;
}
#include "aes_bs.h"
using namespace atls_bs;
static void keys(int two, const uint32_t* ra, const uint32_t* rb, int r, Key1& k1, Key2& k2) {
  for (int c = 0; c < 4; c++) { k1.w[c] = ra[4 * r + c]; k2.a[c] = ra[4 * r + c]; k2.b[c] = rb[4 * r + c]; }
  (void)two;
}
template <class KM>
static void rounds(uint32_t (&pl)[16][8], int nr, const uint32_t* ra, const uint32_t* rb) {
  Key1 k1; Key2 k2; KM* km;
  if constexpr (sizeof(KM) == sizeof(Key1)) km = (KM*)&k1; else km = (KM*)&k2;
  keys(0, ra, rb, 0, k1, k2);
  add_round_key(pl, *km);
  for (int r = 1; r < nr; r++) {
    sub_bytes(pl);
    keys(0, ra, rb, r, k1, k2);
    shift_mix_ark(pl, *km);
  }
  sub_bytes(pl);
  keys(0, ra, rb, nr, k1, k2);
  shift_ark(pl, *km);
}
int main(int argc, char** argv) {
  const int two = argc > 1;
  int nr; uint32_t rk[60], rk2[60]; uint32_t blk[4][32];
  if (scanf("%d", &nr) != 1) return 1;
  for (int i = 0; i < 4 * (nr + 1); i++) scanf("%x", &rk[i]);
  for (int i = 0; i < 4 * (nr + 1); i++) scanf("%x", &rk2[i]);
  for (int k = 0; k < 32; k++) for (int w = 0; w < 4; w++) scanf("%x", &blk[w][k]);
  uint32_t pl[16][8];
  for (int w = 0; w < 4; w++) {            // blocks -> planes (transpose is an involution)
    uint32_t x[32];
    for (int k = 0; k < 32; k++) x[k] = blk[w][k];
    transpose32(x);
    for (int b = 0; b < 4; b++) for (int t = 0; t < 8; t++) pl[4 * w + b][7 - t] = x[8 * b + t];
  }
  if (two) rounds<Key2>(pl, nr, rk, rk2); else rounds<Key1>(pl, nr, rk, rk);
  uint32_t out[4][32];
  planes_to_blocks(pl, out);
  for (int k = 0; k < 32; k++) { for (int w = 0; w < 4; w++) printf("%08x ", out[w][k]); printf("\n"); }
  return 0;
}
"""


def _expand(key):
    import ctypes
    buf = (ctypes.c_uint8 * 240)()
    assert ora.lib().ora_aes_expand_key((ctypes.c_uint8 * len(key)).from_buffer_copy(key), len(key), buf) == 0
    ek = bytes(buf)
    nr = len(key) // 4 + 6
    return nr, [int.from_bytes(ek[4 * i:4 * i + 4], "little") for i in range(4 * (nr + 1))]


def test_bitsliced_aes_matches_oracle():
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "t.cpp")
        exe = os.path.join(d, "t")
        open(c, "w").write(SRC)
        subprocess.check_call(["g++", "-O1", "-I", os.path.join(ROOT, "anothertls_amd", "csrc"), c, "-o", exe])
        rng = random.Random(99)
        for two in (False, True):
            for klen in (16, 24, 32):
                keys = [bytes(rng.getrandbits(8) for _ in range(klen)) for _ in range(2)]
                nr, rka = _expand(keys[0])
                _, rkb = _expand(keys[1])
                blocks = [bytes(rng.getrandbits(8) for _ in range(16)) for _ in range(32)]
                words = [int.from_bytes(b[4 * w:4 * w + 4], "little") for b in blocks for w in range(4)]
                inp = (f"{nr}\n" + " ".join(f"{x:08x}" for x in rka + rkb) + "\n" +
                       " ".join(f"{x:08x}" for x in words) + "\n")
                out = subprocess.check_output([exe] + (["2"] if two else []), input=inp.encode()).decode().split("\n")
                for k, b in enumerate(blocks):
                    got = b"".join(int(x, 16).to_bytes(4, "little") for x in out[k].split())
                    key = keys[1] if (two and k >= 16) else keys[0]
                    rc, want = ora.aes_encrypt_block(key, b)
                    assert rc == 0 and got == want, (two, klen, k)
