"""C-ABI library: loads, exports every symbol include/atls.h declares, struct layouts match,
and without a GPU every compute entry point fails loudly (no CPU fallback)."""
import os
import re
import subprocess
import tempfile

import pytest

import anothertls_amd as atls

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "atls.h")


def declared_functions():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[\w\s\*]*?\b(atls_\w+)\s*\(", text, re.M)))


def test_exports_every_declared_symbol():
    names = declared_functions()
    assert len(names) >= 12, names
    lib = atls.library()
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_product_build_has_no_experiment_switches():
    """The library the package loads is the product build: no ATLS_DBG_* timing switch (those
    drop work and give wrong results), no alternative GHASH / counter-cache variant."""
    lib = atls.library()
    lib.atls_build_flags.restype = __import__("ctypes").c_uint
    assert lib.atls_build_flags() == 0


def test_abi_version_and_arch():
    assert atls.abi_version() == 1
    assert atls.library().atls_device_arch() == b"gfx950"


def test_struct_layout_matches_header():
    src = """
#include <stdio.h>
#include <stddef.h>
#include "atls.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu %zu %zu\\n", sizeof(atls_key), sizeof(atls_rec), sizeof(atls_open_result),
         offsetof(atls_rec, len), offsetof(atls_rec, aad_len), offsetof(atls_key, static_iv),
         offsetof(atls_open_result, status));
  return 0;
}
"""
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "t.c")
        exe = os.path.join(d, "t")
        open(c, "w").write(src)
        subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o", exe])
        got = [int(x) for x in subprocess.check_output([exe]).split()]
    K, R, O = atls.KEY_DTYPE, atls.REC_DTYPE, atls.OPEN_RESULT_DTYPE
    assert got == [K.itemsize, R.itemsize, O.itemsize, R.fields["len"][1], R.fields["aad_len"][1],
                   K.fields["static_iv"][1], O.fields["status"][1]]


def test_cipher_suite_mirror():
    CS = atls.CipherSuite
    assert CS.new(0x1301).get_key_and_iv_len() == (16, 12)
    assert CS.new(0x1302).get_key_and_iv_len() == (32, 12)
    assert CS.new(0x1303).get_key_and_iv_len() == (32, 12)
    assert isinstance(CS(0x1301).get_cipher(), atls.Gcm)
    assert isinstance(CS(0x1303).get_cipher(), atls.Poly1305)
    with pytest.raises(atls.TlsError) as e:
        CS.new(0x1304)
    assert e.value.code == 71
    with pytest.raises(atls.TlsError) as e:
        CS.TLS_EMPTY_RENEGOTIATION_INFO_SCSV.get_cipher()
    assert e.value.code == 71


def test_parameter_errors_before_device():
    # Validation happens at the boundary, before any device work (reference panics here).
    with pytest.raises(atls.TlsError) as e:
        atls.Gcm().encrypt(b"k" * 15, b"i" * 12, b"x")
    assert e.value.code == 47
    with pytest.raises(atls.TlsError) as e:
        atls.Poly1305().encrypt(b"k" * 32, b"i" * 8, b"x")
    assert e.value.code == 47
    with pytest.raises(atls.TlsError) as e:
        atls.Gcm().decrypt(b"k" * 16, b"i" * 12, b"x", b"", b"short")
    assert e.value.code == 20
    with pytest.raises(atls.TlsError) as e:  # AES::init with a key that is not the block size
        atls.AES.init(b"k" * 16, 256)
    assert e.value.code == 47


@pytest.mark.skipif(atls.device_available(), reason="a GPU is present")
def test_no_gpu_fails_loudly():
    with pytest.raises(atls.TlsError) as e:
        atls.Gcm().encrypt(b"k" * 16, b"i" * 12, b"hello")
    assert e.value.code == 80
    with pytest.raises(atls.TlsError) as e:
        atls.Engine(0)
    assert e.value.code == 80
    with pytest.raises(atls.TlsError) as e:
        atls.AES.init(b"k" * 16).encrypt(bytes(16))
    assert e.value.code == 80
