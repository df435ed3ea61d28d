"""CPU check of the generated bitsliced S-box (tools/bitsliced/sbox_bs.h): compile it for the
host with a software v_bitop3_b32 (result bit = tt[(a<<2)|(b<<1)|c], the gfx950 operand order
observed in hipcc's own lowering) and compare all 256 inputs with the FIPS-197 S-box."""
import os
import subprocess
import tempfile

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
#include "sbox_bs.h"
int main(void) {
  for (int base = 0; base < 256; base += 32) {
    uint32_t x[8] = {0};
    for (int s = 0; s < 32; s++)
      for (int j = 0; j < 8; j++) x[j] |= (uint32_t)(((base + s) >> (7 - j)) & 1) << s;
    sbox_bs(x);
    for (int s = 0; s < 32; s++) {
      int v = 0;
      for (int j = 0; j < 8; j++) v |= ((x[j] >> s) & 1) << (7 - j);
      printf("%02x", v);
    }
  }
  printf("\n");
  return 0;
}
"""

SBOX_HEX = ("637c777bf26b6fc53001672bfed7ab76ca82c97dfa5947f0add4a2af9ca472c0b7fd9326363ff7cc34a5e5f171d8311504c723c31896059a071280e2eb27b275"
            "09832c1a1b6e5aa0523bd6b329e32f8453d100ed20fcb15b6acbbe394a4c58cfd0efaafb434d338545f9027f503c9fa851a3408f929d38f5bcb6da2110fff3d2"
            "cd0c13ec5f974417c4a77e3d645d197360814fdc222a908846eeb814de5e0bdbe0323a0a4906245cc2d3ac629195e479e7c8376d8dd54ea96c56f4ea657aae08"
            "ba78252e1ca6b4c6e8dd741f4bbd8b8a703eb5664803f60e613557b986c11d9ee1f8981169d98e949b1e87e9ce5528df8ca1890dbfe6426841992d0fb054bb16")


def test_generated_sbox_matches_fips197():
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "t.cpp")
        exe = os.path.join(d, "t")
        open(c, "w").write(SRC)
        subprocess.check_call(["g++", "-O1", "-I", os.path.join(ROOT, "tools", "bitsliced"), c, "-o", exe])
        out = subprocess.check_output([exe]).decode().strip()
    assert out == SBOX_HEX
