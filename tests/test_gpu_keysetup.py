"""The key-setup kernel (anothertls_amd/csrc/keysetup.hip, one wave per key slot) against a host model
of every KeySched field (tests/keysched_model.py: the oracle's AES key expansion and E_K(0), GF(2^128)
products in gcm.rs's bit order). Both install paths: keys staged by one copy (set_keys of many slots)
and keys in the kernel arguments (update_keys / set_keys of at most 4 slots, the single call's cache
miss). Reference: crypto/aes/cipher.rs:216-249, crypto/aes/gcm.rs:21-56, chacha20/cipher.rs:29-31."""
import ctypes
import os

import numpy as np
import pytest

import keysched_model as km

RNG = np.random.default_rng(0x4B53)


def _keys(spec):
    import anothertls_amd as atls

    arr = np.zeros(len(spec), dtype=atls.KEY_DTYPE)
    for i, (suite, klen) in enumerate(spec):
        arr[i]["suite"], arr[i]["key_len"], arr[i]["iv_len"] = suite, klen, 12
        arr[i]["key"] = RNG.integers(0, 256, 32, dtype=np.uint8)
        arr[i]["static_iv"] = RNG.integers(0, 256, 12, dtype=np.uint8)
    return arr


# ---- CPU: the model itself -----------------------------------------------------------------------

def test_model_product_equals_oracle_gmult():
    """The model's GF(2^128) product is the reference's gmult (gcm.rs:21-40, the oracle's restatement)."""
    import oracle as ora

    for _ in range(20):
        a, b = RNG.integers(0, 256, 16, dtype=np.uint8).tobytes(), RNG.integers(0, 256, 16, dtype=np.uint8).tobytes()
        want = int.from_bytes(ora.gcm_gmult(a, b), "big")
        assert km.gf_mul(int.from_bytes(a, "big"), int.from_bytes(b, "big")) == want


def _mulxk64(v, m):
    """gcm_common.h gf_mulxk64, restated on a Python int (1 <= m <= 64): shift, and the m bits pushed
    past x^127 folded back as S ^ S>>1 ^ S>>2 ^ S>>7."""
    mask = (1 << 128) - 1
    s = (v << (128 - m)) & mask
    return (v >> m) ^ s ^ (s >> 1) ^ (s >> 2) ^ (s >> 7)


def test_one_step_multiply_by_x_power_equals_repeated_mulx():
    for _ in range(30):
        v = int.from_bytes(RNG.integers(0, 256, 16, dtype=np.uint8).tobytes(), "big")
        for m in (1, 2, 4, 7, 31, 32, 33, 60, 63, 64):
            assert _mulxk64(v, m) == km.gf_mulxk(v, m), m
        for m in (65, 100, 124, 127):  # gf_mulxk: 64 first, then the rest
            assert _mulxk64(_mulxk64(v, 64), m - 64) == km.gf_mulxk(v, m), m


# ---- GPU ------------------------------------------------------------------------------------------

def _dump(atls, eng, slot):
    lib = atls.library()
    lib.atls_debug_key_sched.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t]
    buf = np.zeros(1, dtype=km.KEYSCHED_DTYPE)
    assert lib.atls_debug_key_sched(eng._e, slot, buf.ctypes.data, buf.nbytes) == buf.nbytes
    return buf[0]


SPEC = [(0x1301, 16), (0x1302, 32), (0x1301, 24), (0x1303, 32), (0x1302, 16), (0x1301, 32), (0x1302, 24),
        (0x1303, 16), (0x00FF, 16), (0x1301, 20), (0x1301, 16)]


@pytest.mark.gpu
def test_staged_install_matches_model():
    import anothertls_amd as atls

    keys = _keys(SPEC)
    eng = atls.Engine(int(os.environ.get("ATLS_DEVICE", "0")))
    try:
        with pytest.raises(atls.TlsError):  # the invalid slots are reported, the others installed
            eng.set_keys(keys)
        for i, k in enumerate(keys):
            bad = km.compare(_dump(atls, eng, i), km.expected(k))
            assert not bad, (i, SPEC[i], bad)
    finally:
        eng.close()


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 2, 3, 4])
def test_inline_install_matches_model(n):
    """n <= 4 keys travel in the kernel arguments (no staging copy, no host wait); an update after
    them, and batches after it, see them."""
    import anothertls_amd as atls

    base = _keys([(0x1301, 16)] * 6)
    eng = atls.Engine(int(os.environ.get("ATLS_DEVICE", "0")))
    try:
        eng.set_keys(base)
        new = _keys([SPEC[(n + j) % 7] for j in range(n)])
        eng.update_keys(2, new)
        eng.update_keys(6, new[:1])  # grows the table by one slot (a reallocation) after the inline launch
        for i in range(7):
            want = km.expected(new[i - 2] if 2 <= i < 2 + n else new[0] if i == 6 else base[i])
            bad = km.compare(_dump(atls, eng, i), want)
            assert not bad, (n, i, bad)
    finally:
        eng.close()


@pytest.mark.gpu
def test_many_keys_one_launch_match_model():
    """C2's 4,096 connections in one install (1,024 workgroups of 4 waves): a sample of slots."""
    import anothertls_amd as atls
    from anothertls_amd import workload

    b = workload.config_batch("c2_aes128gcm_64Ki_x_16KiB", n=4096)
    keys = b["keys"].copy()
    keys[1::3]["key_len"], keys[1::3]["suite"] = 32, 0x1302
    eng = atls.Engine(int(os.environ.get("ATLS_DEVICE", "0")))
    try:
        eng.set_keys(keys)
        for i in list(range(0, 4096, 257)) + [4095]:
            bad = km.compare(_dump(atls, eng, i), km.expected(keys[i]))
            assert not bad, (i, bad)
    finally:
        eng.close()


def _square(v):
    """gcm_common.h gf_square, restated on a Python int: coefficient x^i -> x^(2i) (bit b of each 64-bit
    half -> bit 2b + 1), the high half's image O(x) folded back as O * (1 + x + x^2 + x^7)."""
    def spread(x):
        return sum(((x >> b) & 1) << (2 * b + 1) for b in range(64))

    lo, hi = v >> 64, v & ((1 << 64) - 1)  # x^0..x^63 in the high 64 bits of the number
    o = spread(hi)
    return spread(lo) ^ o ^ _mulxk64(o, 1) ^ _mulxk64(o, 2) ^ _mulxk64(o, 7)


def test_one_step_square_equals_product():
    for _ in range(30):
        v = int.from_bytes(RNG.integers(0, 256, 16, dtype=np.uint8).tobytes(), "big")
        assert _square(v) == km.gf_mul(v, v)
