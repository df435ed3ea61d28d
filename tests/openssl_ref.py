"""Independent cross-check: OpenSSL 3 libcrypto EVP AEADs through ctypes (test-only).

Valid oracle for AES-GCM with any IV length and for ChaCha20-Poly1305 only
where the reference's F4 quirk does not fire (AEAD input length % 64 != 0).
"""
import ctypes
import ctypes.util

_lib = None


def available():
    try:
        _load()
        return True
    except OSError:
        return False


def _load():
    global _lib
    if _lib is None:
        name = ctypes.util.find_library("crypto") or "libcrypto.so.3"
        _lib = ctypes.CDLL(name)
        for fn in ("EVP_CIPHER_CTX_new", "EVP_aes_128_gcm", "EVP_aes_192_gcm", "EVP_aes_256_gcm",
                   "EVP_chacha20_poly1305"):
            getattr(_lib, fn).restype = ctypes.c_void_p
        _lib.EVP_CIPHER_CTX_free.argtypes = [ctypes.c_void_p]
        _lib.EVP_CIPHER_CTX_ctrl.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        for fn in ("EVP_EncryptInit_ex", "EVP_DecryptInit_ex"):
            getattr(_lib, fn).argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_char_p,
                                          ctypes.c_char_p]
        for fn in ("EVP_EncryptUpdate", "EVP_DecryptUpdate"):
            getattr(_lib, fn).argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int),
                                          ctypes.c_char_p, ctypes.c_int]
        for fn in ("EVP_EncryptFinal_ex", "EVP_DecryptFinal_ex"):
            getattr(_lib, fn).argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]
    return _lib


EVP_CTRL_AEAD_SET_IVLEN = 0x9
EVP_CTRL_AEAD_GET_TAG = 0x10
EVP_CTRL_AEAD_SET_TAG = 0x11


def _cipher(kind, key_len):
    lib = _load()
    if kind == "gcm":
        return {16: lib.EVP_aes_128_gcm, 24: lib.EVP_aes_192_gcm, 32: lib.EVP_aes_256_gcm}[key_len]()
    return lib.EVP_chacha20_poly1305()


def seal(kind, key, iv, pt, aad=b""):
    lib = _load()
    ctx = lib.EVP_CIPHER_CTX_new()
    try:
        assert lib.EVP_EncryptInit_ex(ctx, _cipher(kind, len(key)), None, None, None) == 1
        assert lib.EVP_CIPHER_CTX_ctrl(ctx, EVP_CTRL_AEAD_SET_IVLEN, len(iv), None) == 1
        assert lib.EVP_EncryptInit_ex(ctx, None, None, bytes(key), bytes(iv)) == 1
        outl = ctypes.c_int(0)
        if aad:
            assert lib.EVP_EncryptUpdate(ctx, None, ctypes.byref(outl), bytes(aad), len(aad)) == 1
        out = ctypes.create_string_buffer(len(pt) + 32)
        assert lib.EVP_EncryptUpdate(ctx, out, ctypes.byref(outl), bytes(pt), len(pt)) == 1
        n = outl.value
        fin = ctypes.create_string_buffer(32)
        assert lib.EVP_EncryptFinal_ex(ctx, fin, ctypes.byref(outl)) == 1
        tag = ctypes.create_string_buffer(16)
        assert lib.EVP_CIPHER_CTX_ctrl(ctx, EVP_CTRL_AEAD_GET_TAG, 16, tag) == 1
        return out.raw[:n], tag.raw
    finally:
        lib.EVP_CIPHER_CTX_free(ctx)


_XC = None


def _xcheck():
    """tests/native/build/libxcheck.so (OpenSSL batch sealer; built by `make -C tests/native`)."""
    global _XC
    if _XC is None:
        import os
        import subprocess

        here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native")
        path = os.path.join(here, "build", "libxcheck.so")
        if not os.path.exists(path):
            subprocess.check_call(["make", "-s", "-C", here])
        _XC = ctypes.CDLL(path)
        _XC.xc_seal_tls_batch.argtypes = [ctypes.c_void_p] * 2 + [ctypes.c_uint32] + [ctypes.c_void_p] * 4 + \
            [ctypes.c_int]
    return _XC


def seal_tls_batch(keys, recs, inbuf, out_bytes, nthreads=16):
    """OpenSSL seal of every TLS-mode record of a batch (numpy KEY_DTYPE / REC_DTYPE arrays,
    inbuf a uint8 array). Returns (out, tags, skipped): skipped[i] = 1 for ChaCha20-Poly1305
    records that hit the reference's last-block quirk, which OpenSSL cannot check."""
    import numpy as np

    keys = np.ascontiguousarray(keys)
    recs = np.ascontiguousarray(recs)
    inbuf = np.ascontiguousarray(inbuf)
    out = np.zeros(max(out_bytes, 16), np.uint8)
    tags = np.zeros(16 * len(recs), np.uint8)
    skipped = np.zeros(max(len(recs), 1), np.uint8)
    rc = _xcheck().xc_seal_tls_batch(keys.ctypes.data, recs.ctypes.data, len(recs), inbuf.ctypes.data,
                                     out.ctypes.data, tags.ctypes.data, skipped.ctypes.data, nthreads)
    assert rc == 0, "OpenSSL batch seal failed"
    return out, tags, skipped[:len(recs)]


def open_(kind, key, iv, ct, aad, tag):
    """Returns plaintext or None on authentication failure."""
    lib = _load()
    ctx = lib.EVP_CIPHER_CTX_new()
    try:
        assert lib.EVP_DecryptInit_ex(ctx, _cipher(kind, len(key)), None, None, None) == 1
        assert lib.EVP_CIPHER_CTX_ctrl(ctx, EVP_CTRL_AEAD_SET_IVLEN, len(iv), None) == 1
        assert lib.EVP_DecryptInit_ex(ctx, None, None, bytes(key), bytes(iv)) == 1
        outl = ctypes.c_int(0)
        if aad:
            assert lib.EVP_DecryptUpdate(ctx, None, ctypes.byref(outl), bytes(aad), len(aad)) == 1
        out = ctypes.create_string_buffer(len(ct) + 32)
        assert lib.EVP_DecryptUpdate(ctx, out, ctypes.byref(outl), bytes(ct), len(ct)) == 1
        n = outl.value
        t = ctypes.create_string_buffer(bytes(tag), 16)
        assert lib.EVP_CIPHER_CTX_ctrl(ctx, EVP_CTRL_AEAD_SET_TAG, 16, t) == 1
        fin = ctypes.create_string_buffer(32)
        ok = lib.EVP_DecryptFinal_ex(ctx, fin, ctypes.byref(outl))
        return out.raw[:n] if ok == 1 else None
    finally:
        lib.EVP_CIPHER_CTX_free(ctx)
