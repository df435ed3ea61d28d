"""CPU check of the bitsliced AES core (tools/bitsliced/aes_bs.h, the bitsliced AES of the round-1/2 hybrid experiments) as it would run
on the VALU: compiled for the host with software v_bitop3_b32 / v_perm_b32, 32 random blocks
per key for AES-128/192/256 round keys from the oracle's key expansion, in the row-plane layout, compared against the
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
// v_perm_b32: selector 0-7 picks a byte of {S0:S1}, 8-11 replicate bit 15/31/47/63, 12 -> 0x00,
// 13-15 -> 0xFF (the compiler folds perm(0x80000000, 0x8000, 0x0b0a0908) to 0xff0000ff)
static uint32_t __builtin_amdgcn_perm(uint32_t s0, uint32_t s1, uint32_t sel) {
  uint64_t d = ((uint64_t)s0 << 32) | s1;
  uint32_t r = 0;
  for (int i = 0; i < 4; i++) {
    unsigned b = (sel >> (8 * i)) & 0xff, v;
    if (b == 12) v = 0;
    else if (b >= 13) v = 0xff;
    else if (b >= 8) v = ((d >> (16 * (b - 8) + 15)) & 1) ? 0xff : 0;
    else v = (d >> (8 * b)) & 0xff;
    r |= v << (8 * i);
  }
  return r;
}
static uint32_t __builtin_amdgcn_alignbit(uint32_t a, uint32_t b, uint32_t s) {
  return (uint32_t)((((uint64_t)a << 32) | b) >> (s & 31));
}
#include "aes_bs.h"
using namespace atls_bs;
int main(void) {
  int nr; uint32_t rk[60]; uint32_t blk[32][4];
  if (scanf("%d", &nr) != 1) return 1;
  for (int i = 0; i < 4 * (nr + 1); i++) scanf("%x", &rk[i]);
  for (int k = 0; k < 32; k++) for (int w = 0; w < 4; w++) scanf("%x", &blk[k][w]);
  State st;
  for (int g = 0; g < 4; g++) {
    uint32_t x[32];
    for (int c = 0; c < 4; c++) for (int b = 0; b < 8; b++) x[8 * c + b] = blk[8 * g + b][c];
    blocks_to_group(x, st[g]);
  }
  Masks m;
  { uint32_t w[4] = {rk[0], rk[1], rk[2], rk[3]}; make_masks(w, m); }
  add_round_key(st, m);
  for (int r = 1; r <= nr; r++) {
    sub_bytes(st);
    uint32_t w[4] = {rk[4 * r], rk[4 * r + 1], rk[4 * r + 2], rk[4 * r + 3]};
    make_masks(w, m);
    if (r < nr) shift_mix_ark(st, m); else shift_ark(st, m);
  }
  for (int g = 0; g < 4; g++) {
    uint32_t x[32];
    group_to_blocks(st[g], x);
    for (int b = 0; b < 8; b++) { for (int c = 0; c < 4; c++) printf("%08x ", x[8 * c + b]); printf("\n"); }
  }
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
        subprocess.check_call(["g++", "-O1", "-I", os.path.join(ROOT, "tools", "bitsliced"), c, "-o", exe])
        rng = random.Random(99)
        for klen in (16, 24, 32):
            for _ in range(2):
                key = bytes(rng.getrandbits(8) for _ in range(klen))
                nr, rkw = _expand(key)
                blocks = [bytes(rng.getrandbits(8) for _ in range(16)) for _ in range(32)]
                words = [int.from_bytes(b[4 * w:4 * w + 4], "little") for b in blocks for w in range(4)]
                inp = f"{nr}\n" + " ".join(f"{x:08x}" for x in rkw) + "\n" + " ".join(f"{x:08x}" for x in words) + "\n"
                out = subprocess.check_output([exe], input=inp.encode()).decode().split("\n")
                for k, b in enumerate(blocks):
                    got = b"".join(int(x, 16).to_bytes(4, "little") for x in out[k].split())
                    rc, want = ora.aes_encrypt_block(key, b)
                    assert rc == 0 and got == want, (klen, k)
