"""Host model of the device key schedule (anothertls_amd/csrc/atls_dev.h KeySched), test-only.

What the key-setup kernel (csrc/keysetup.hip) must write for one key slot, from the reference's
definitions: AES key expansion (crypto/aes/cipher.rs:216-249, through the oracle's
ora_aes_expand_key), H = E_K(0^128) (crypto/aes/gcm.rs:56, through the oracle's AES), and GF(2^128)
products in GCM's bit order (gcm.rs:21-40 gmult: the coefficient of x^i is bit 127 - i of the
block read big-endian) for H^1..H^64 and the GHASH table seeds x^(4p) * H^e.
"""
import ctypes

import numpy as np

KEYSCHED_DTYPE = np.dtype([
    ("suite", "<u4"), ("nr", "<u4"), ("key_len", "<u4"), ("valid", "<u4"),
    ("rk", "<u4", 60), ("kw", "<u4", 8), ("siv", "<u4", 4), ("h_be", "<u4", 4),
    ("hpow_be", "<u4", (64, 4)), ("p4_be", "<u4", (32, 4)), ("rkr", "<u4", 60), ("pad", "<u4", 4),
    ("p4g_be", "<u4", (3, 32, 4)),
])
assert KEYSCHED_DTYPE.itemsize == 3648

R = 0xE1 << 120


def gf_mulx(v):
    """v * x (gf_mulx_be): shift toward x^127, reduce by 1 + x + x^2 + x^7."""
    return (v >> 1) ^ (R if v & 1 else 0)


def gf_mul(x, y):
    """x * y in GF(2^128), GCM bit order (NIST SP 800-38D Algorithm 1, the product gcm.rs gmult computes)."""
    z, v = 0, y
    for i in range(128):
        if (x >> (127 - i)) & 1:
            z ^= v
        v = gf_mulx(v)
    return z


def gf_mulxk(v, k):
    for _ in range(k):
        v = gf_mulx(v)
    return v


def be_words(v):
    return [(v >> (96 - 32 * w)) & 0xFFFFFFFF for w in range(4)]


def expected(key_row, ora=None):
    """Dict of the KeySched fields the kernel must write for one atls_key row (KEY_DTYPE)."""
    suite, klen = int(key_row["suite"]), int(key_row["key_len"])
    kb = bytes(key_row["key"])
    out = {"suite": suite, "key_len": klen,
           "kw": [int(w) for w in np.frombuffer(kb, "<u4")],
           "siv": [int(w) for w in np.frombuffer(bytes(key_row["static_iv"]) + b"\0" * 4, "<u4")]}
    aes = suite in (0x1301, 0x1302) and klen in (16, 24, 32)
    if not aes:
        out.update(nr=0, valid=int(suite == 0x1303 and klen == 32))
        return out
    if ora is None:
        import oracle as ora
    nr = klen // 4 + 6
    ek = (ctypes.c_uint8 * 240)()
    assert ora.lib().ora_aes_expand_key(bytes(kb[:klen]), ctypes.c_size_t(klen), ek) == 0
    ekb = bytes(ek)[:16 * (nr + 1)]
    rk = [int(w) for w in np.frombuffer(ekb, "<u4")] + [0] * (60 - 4 * (nr + 1))
    rc, hb = ora.aes_encrypt_block(kb[:klen], b"\0" * 16)
    assert rc == 0
    h = int.from_bytes(hb, "big")
    pw, p = [], h
    for _ in range(64):
        pw.append(p)
        p = gf_mul(p, h)
    out.update(nr=nr, valid=1, rk=rk, rkr=[((w << 16) | (w >> 16)) & 0xFFFFFFFF for w in rk],
               h_be=be_words(h), hpow_be=[be_words(x) for x in pw],
               p4_be=[be_words(gf_mulxk(pw[63], 4 * j)) for j in range(32)],
               p4g_be=[[be_words(gf_mulxk(pw[(8 << t) - 1], 4 * j)) for j in range(32)] for t in range(3)])
    return out


def compare(dev_row, want):
    """Names of the KeySched fields of dev_row (KEYSCHED_DTYPE) that differ from `want`."""
    bad = []
    for k, v in want.items():
        got = np.asarray(dev_row[k]).astype(np.uint64).ravel()
        exp = np.asarray(v, dtype=np.uint64).ravel()
        if got.shape != exp.shape or not np.array_equal(got, exp):
            bad.append(k)
    return bad
