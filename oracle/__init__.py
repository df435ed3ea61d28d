"""TEST INFRASTRUCTURE ONLY: ctypes binding to the parity oracle (oracle/build/libatls_oracle.so).

The oracle is a literal C restatement of otsmr/AnotherTLS's AEAD path (ref_restatement.c).
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module; the product package anothertls_amd never does.
"""
import ctypes
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "libatls_oracle.so")
_lib = None

SHA256, SHA384 = 32, 48
MODE_TLS, MODE_RAW, MODE_WIRE = 0, 1, 2


class OraKey(ctypes.Structure):
    _fields_ = [("suite", ctypes.c_uint16), ("key_len", ctypes.c_uint8), ("iv_len", ctypes.c_uint8),
                ("key", ctypes.c_uint8 * 32), ("static_iv", ctypes.c_uint8 * 12),
                ("reserved", ctypes.c_uint8 * 16)]


class OraRec(ctypes.Structure):
    _fields_ = [("in_off", ctypes.c_uint64), ("out_off", ctypes.c_uint64), ("aux_off", ctypes.c_uint64),
                ("seq", ctypes.c_uint64), ("len", ctypes.c_uint32), ("key_slot", ctypes.c_uint32),
                ("aad_len", ctypes.c_uint16), ("content_type", ctypes.c_uint8), ("mode", ctypes.c_uint8),
                ("iv_len", ctypes.c_uint8), ("reserved", ctypes.c_uint8 * 3)]


class OraOpenResult(ctypes.Structure):
    _fields_ = [("content_len", ctypes.c_uint32), ("status", ctypes.c_uint8),
                ("content_type", ctypes.c_uint8), ("reserved", ctypes.c_uint8 * 2)]


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = ctypes.CDLL(LIB_PATH)
    return _lib


def _buf(b):
    b = bytes(b)
    return (ctypes.c_uint8 * max(len(b), 1)).from_buffer_copy(b if b else b"\0"), len(b)


def _out(n):
    return (ctypes.c_uint8 * max(n, 1))()


def aes_encrypt_block(key, block):
    k, kl = _buf(key)
    i, _ = _buf(block)
    o = _out(16)
    rc = lib().ora_aes_encrypt_block(k, ctypes.c_size_t(kl), i, o)
    return rc, bytes(o)


def aes_decrypt_block(key, block):
    k, kl = _buf(key)
    i, _ = _buf(block)
    o = _out(16)
    rc = lib().ora_aes_decrypt_block(k, ctypes.c_size_t(kl), i, o)
    return rc, bytes(o)


def _aead(fn, key, iv, data, aad):
    k, kl = _buf(key)
    v, vl = _buf(iv)
    d, n = _buf(data)
    a, m = _buf(aad)
    o = _out(n)
    t = _out(16)
    S = ctypes.c_size_t
    rc = fn(k, S(kl), v, S(vl), d, S(n), a, S(m), o, t)
    return rc, bytes(o)[:n], bytes(t)


def _aead_open(fn, key, iv, data, aad, tag):
    k, kl = _buf(key)
    v, vl = _buf(iv)
    d, n = _buf(data)
    a, m = _buf(aad)
    tg, tl = _buf(tag)
    o = _out(n)
    S = ctypes.c_size_t
    rc = fn(k, S(kl), v, S(vl), d, S(n), a, S(m), tg, S(tl), o)
    return rc, bytes(o)[:n]


def gcm_encrypt(key, iv, pt, aad=b""):
    return _aead(lib().ora_gcm_encrypt, key, iv, pt, aad)


def gcm_decrypt(key, iv, ct, aad, tag):
    return _aead_open(lib().ora_gcm_decrypt, key, iv, ct, aad, tag)


def chacha_poly_encrypt(key, iv, pt, aad=b""):
    return _aead(lib().ora_chacha_poly_encrypt, key, iv, pt, aad)


def chacha_poly_decrypt(key, iv, ct, aad, tag):
    return _aead_open(lib().ora_chacha_poly_decrypt, key, iv, ct, aad, tag)


def cipher_encrypt(suite, key, iv, pt, aad=b""):
    f = lib().ora_cipher_encrypt
    k, kl = _buf(key)
    v, vl = _buf(iv)
    d, n = _buf(pt)
    a, m = _buf(aad)
    o, t = _out(n), _out(16)
    S = ctypes.c_size_t
    rc = f(ctypes.c_uint16(suite), k, S(kl), v, S(vl), d, S(n), a, S(m), o, t)
    return rc, bytes(o)[:n], bytes(t)


def cipher_decrypt(suite, key, iv, ct, aad, tag):
    f = lib().ora_cipher_decrypt
    k, kl = _buf(key)
    v, vl = _buf(iv)
    d, n = _buf(ct)
    a, m = _buf(aad)
    tg, tl = _buf(tag)
    o = _out(n)
    S = ctypes.c_size_t
    rc = f(ctypes.c_uint16(suite), k, S(kl), v, S(vl), d, S(n), a, S(m), tg, S(tl), o)
    return rc, bytes(o)[:n]


def chacha20_encrypt(key, iv, data, counter):
    d, n = _buf(data)
    k, kl = _buf(key)
    v, vl = _buf(iv)
    o = _out(n)
    S = ctypes.c_size_t
    rc = lib().ora_chacha20_encrypt(d, S(n), k, S(kl), v, S(vl), S(counter), o)
    return rc, bytes(o)[:n]


def poly1305_mac(key, msg):
    k, _ = _buf(key)
    m, n = _buf(msg)
    t = _out(16)
    lib().ora_poly1305_mac(k, m, ctypes.c_size_t(n), t)
    return bytes(t)


def poly1305_key_gen(key, iv):
    k, kl = _buf(key)
    v, vl = _buf(iv)
    o = _out(32)
    rc = lib().ora_poly1305_key_gen(k, ctypes.c_size_t(kl), v, ctypes.c_size_t(vl), o)
    return rc, bytes(o)


def gcm_gmult(a, b):
    x, _ = _buf(a)
    y, _ = _buf(b)
    o = _out(16)
    lib().ora_gcm_gmult(x, y, o)
    return bytes(o)


def sha(hash_len, msg):
    m, n = _buf(msg)
    o = _out(hash_len)
    (lib().ora_sha384 if hash_len == SHA384 else lib().ora_sha256)(m, ctypes.c_size_t(n), o)
    return bytes(o)


def hmac(hash_len, key, msg):
    k, kl = _buf(key)
    m, n = _buf(msg)
    o = _out(hash_len)
    lib().ora_hmac(hash_len, k, ctypes.c_size_t(kl), m, ctypes.c_size_t(n), o)
    return bytes(o)


def hkdf_extract(hash_len, salt, ikm):
    s, sl = _buf(salt)
    i, il = _buf(ikm)
    o = _out(hash_len)
    lib().ora_hkdf_extract(hash_len, s, ctypes.c_size_t(sl), i, ctypes.c_size_t(il), o)
    return bytes(o)


def hkdf_expand(hash_len, prk, info, out_len):
    p, pl = _buf(prk)
    i, il = _buf(info)
    o = _out(out_len)
    rc = lib().ora_hkdf_expand(hash_len, p, ctypes.c_size_t(pl), i, ctypes.c_size_t(il), o,
                               ctypes.c_size_t(out_len))
    return None if rc else bytes(o)[:out_len]


def key_from_secret(hash_len, secret, key_len, iv_len=12):
    s, sl = _buf(secret)
    k, v = _out(key_len), _out(iv_len)
    rc = lib().ora_key_from_secret(hash_len, s, ctypes.c_size_t(sl), ctypes.c_size_t(key_len),
                                   ctypes.c_size_t(iv_len), k, v)
    return rc, bytes(k)[:key_len], bytes(v)[:iv_len]


def key_schedule(hash_len, shared, hello_hash, handshake_hash=None):
    """key_schedule.rs:170-222 + :87-114 -> (c_hs, s_hs, master, c_ap, s_ap) secrets."""
    s, sl = _buf(shared)
    h, _ = _buf(hello_hash)
    f = _buf(handshake_hash)[0] if handshake_hash is not None else None
    o = _out(5 * hash_len)
    rc = lib().ora_key_schedule(hash_len, s, ctypes.c_size_t(sl), h, f, o)
    assert rc == 0
    b = bytes(o)
    return tuple(b[i * hash_len:(i + 1) * hash_len] for i in range(5 if handshake_hash is not None else 3))


def per_record_nonce(iv, seq):
    v, _ = _buf(iv)
    o = _out(12)
    lib().ora_per_record_nonce(v, ctypes.c_uint64(seq), o)
    return bytes(o)


def record_seal(suite, key, iv, seq, content_type, frag):
    k, kl = _buf(key)
    v, _ = _buf(iv)
    f, fl = _buf(frag)
    w = _out(fl + 1 + 5 + 16)
    wl = ctypes.c_size_t(0)
    rc = lib().ora_record_seal(ctypes.c_uint16(suite), k, ctypes.c_size_t(kl), v, ctypes.c_uint64(seq),
                               ctypes.c_uint8(content_type), f, ctypes.c_size_t(fl), w, ctypes.byref(wl))
    return rc, bytes(w)[:wl.value]


def record_open(suite, key, iv, seq, wire):
    k, kl = _buf(key)
    v, _ = _buf(iv)
    w, wl = _buf(wire)
    c = _out(wl)
    cl = ctypes.c_size_t(0)
    ct = ctypes.c_uint8(0)
    rc = lib().ora_record_open(ctypes.c_uint16(suite), k, ctypes.c_size_t(kl), v, ctypes.c_uint64(seq), w,
                               ctypes.c_size_t(wl), c, ctypes.byref(cl), ctypes.byref(ct))
    return rc, bytes(c)[:cl.value], ct.value


def _ptr(arr):
    """numpy uint8 array -> ctypes pointer"""
    return arr.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


def seal_batch(keys, recs, inbuf, aux, out, tags, nthreads=1):
    """keys: OraKey array; recs: OraRec array; inbuf/aux/out/tags: numpy uint8 arrays."""
    return lib().ora_seal_batch(keys, recs, ctypes.c_uint32(len(recs)), _ptr(inbuf), _ptr(aux), _ptr(out),
                                _ptr(tags), ctypes.c_int(nthreads))


def open_batch(keys, recs, inbuf, aux, tags, out, results, nthreads=1):
    return lib().ora_open_batch(keys, recs, ctypes.c_uint32(len(recs)), _ptr(inbuf), _ptr(aux), _ptr(tags),
                                _ptr(out), results, ctypes.c_int(nthreads))
