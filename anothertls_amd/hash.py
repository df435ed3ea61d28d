"""The reference's hash module on the device (otsmr/AnotherTLS anothertls/src/hash/*.rs and the
key-schedule parts of net/key_schedule.rs), mirrored with the same names and argument meaning:

* ``HashType`` (hash/mod.rs:18-22), ``sha256`` / ``sha384`` / ``sha_x`` (sha256.rs:188-192,
  sha384.rs:202-206, mod.rs:37-42)
* ``Hmac(hash, key).update(buf).result()`` (hmac.rs:10-78; keys > 64 bytes hashed for both hashes)
* ``Hkdf.extract`` / ``Hkdf.from_prk`` / ``Hkdf.expand`` (hkdf.rs:24-65; expand returns None past
  255 * HashLen)
* ``get_hkdf_expand_label`` (key_schedule.rs:20-29), ``Key.from_hkdf`` (:40-50),
  ``KeySchedule.do_key_schedule`` (:170-222) and ``application_secrets`` (:87-114)

Every computation runs on the GPU through the C ABI (atls_hash_batch, atls_key_schedule); the
``*_batch`` functions hash many items per launch, which is how a server with many connections
would use them. There is no CPU fallback."""
import ctypes
import enum
import os

import numpy as np

from . import Engine, TlsError, _check, _lib

_lib.atls_hash_batch.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t,
                                 ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]
_lib.atls_key_schedule.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                   ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]
SPAN_DTYPE = np.dtype([("off", "<u8"), ("len", "<u4"), ("reserved", "<u4")])
OP_SHA, OP_HMAC, OP_HKDF_EXTRACT, OP_HKDF_EXPAND = 0, 1, 2, 3


class HashType(enum.IntEnum):
    """hash/mod.rs:18-22 (the value is the digest length)."""

    SHA256 = 32
    SHA384 = 48


_ENGINE = None


def _engine():
    global _ENGINE
    if _ENGINE is None:
        _ENGINE = Engine(int(os.environ.get("ATLS_DEVICE", "0")))
    return _ENGINE


def _pack(*lists):
    """Concatenate byte strings of several parallel lists into one buffer + one span array per list."""
    data, spans, pos = [], [], 0
    for items in lists:
        sp = np.zeros(len(items), SPAN_DTYPE)
        for i, b in enumerate(items):
            b = bytes(b)
            sp[i]["off"], sp[i]["len"] = pos, len(b)
            data.append(b)
            pos += len(b)
        spans.append(sp)
    buf = np.frombuffer(b"".join(data) + b"\0", np.uint8).copy()
    return buf, spans


def _run(op, hash_type, keys, msgs, out_len):
    hl = int(hash_type)
    n = len(msgs)
    if keys is None:
        buf, (ms,) = _pack(msgs)
        ks = None
    else:
        buf, (ks, ms) = _pack(keys, msgs)
    out = np.zeros(max(n * out_len, 1), np.uint8)
    _check(_lib.atls_hash_batch(_engine()._e, op, hl, buf.ctypes.data, len(buf) - 1,
                                None if ks is None else ks.ctypes.data, ms.ctypes.data, n, out_len, out.ctypes.data))
    return [out[i * out_len:(i + 1) * out_len].tobytes() for i in range(n)]


def sha_batch(hash_type, msgs):
    return _run(OP_SHA, hash_type, None, msgs, int(hash_type))


def hmac_batch(hash_type, keys, msgs):
    return _run(OP_HMAC, hash_type, keys, msgs, int(hash_type))


def hkdf_extract_batch(hash_type, salts, ikms):
    return _run(OP_HKDF_EXTRACT, hash_type, salts, ikms, int(hash_type))


def hkdf_expand_batch(hash_type, prks, infos, out_len):
    return _run(OP_HKDF_EXPAND, hash_type, prks, infos, out_len)


def sha256(data):
    return sha_batch(HashType.SHA256, [data])[0]


def sha384(data):
    return sha_batch(HashType.SHA384, [data])[0]


def sha_x(hash_type, data):
    return sha_batch(hash_type, [data])[0]


class Hmac:
    """hash/hmac.rs:10-78."""

    def __init__(self, hash_type, key):
        self.hash = HashType(hash_type)
        self.key = bytes(key)
        self.input = bytearray()

    def update(self, buf):
        self.input += bytes(buf)
        return self

    def result(self):
        return hmac_batch(self.hash, [self.key], [bytes(self.input)])[0]


class Hkdf:
    """hash/hkdf.rs:13-65."""

    def __init__(self, hash_type, pseudo_random_key):
        self.hash = HashType(hash_type)
        self.pseudo_random_key = bytes(pseudo_random_key)

    @classmethod
    def from_prk(cls, hash_type, pseudo_random_key):
        return cls(hash_type, pseudo_random_key)

    @classmethod
    def extract(cls, hash_type, salt, ikm):
        return cls(hash_type, hkdf_extract_batch(hash_type, [salt], [ikm])[0])

    def expand(self, info, out_len):
        if out_len > int(self.hash) * 255:  # hkdf.rs:38
            return None
        return hkdf_expand_batch(self.hash, [self.pseudo_random_key], [info], out_len)[0]


def get_hkdf_expand_label(label, context, out_len):
    """net/key_schedule.rs:20-29."""
    label, context = bytes(label), bytes(context)
    return bytes([(out_len >> 8) & 255, out_len & 255, 6 + len(label)]) + b"tls13 " + label + \
        bytes([len(context)]) + context


class Key:
    """net/key_schedule.rs:31-65 (the traffic key of one direction)."""

    def __init__(self, traffic_secret, key, iv):
        self.traffic_secret, self.key, self.iv = traffic_secret, key, iv
        self.sequence_number = 0

    @classmethod
    def from_hkdf(cls, hkdf, key_len, iv_len):
        key = hkdf.expand(get_hkdf_expand_label(b"key", b"", key_len), key_len)
        iv = hkdf.expand(get_hkdf_expand_label(b"iv", b"", iv_len), iv_len)
        if key is None or iv is None:
            return None
        return cls(hkdf.pseudo_random_key, key, iv)

    def get_per_record_nonce(self):
        out = bytearray(self.iv)
        for i in range(8):
            out[11 - i] ^= (self.sequence_number >> (8 * i)) & 255
        self.sequence_number += 1
        return bytes(out)


def key_schedule_batch(hash_type, shared_secrets, hello_hashes, handshake_hashes=None):
    """atls_key_schedule: per connection (c_hs, s_hs, master, c_ap, s_ap) secrets."""
    hl = int(hash_type)
    n = len(shared_secrets)
    sl = len(shared_secrets[0]) if n else 0
    if any(len(s) != sl for s in shared_secrets):
        raise TlsError(TlsError.ILLEGAL_PARAMETER)
    sh = np.frombuffer(b"".join(bytes(s) for s in shared_secrets) or b"\0", np.uint8).copy()
    hh = np.frombuffer(b"".join(bytes(h) for h in hello_hashes) or b"\0", np.uint8).copy()
    fh = None if handshake_hashes is None else np.frombuffer(b"".join(bytes(h) for h in handshake_hashes),
                                                             np.uint8).copy()
    out = np.zeros(max(5 * hl * n, 1), np.uint8)
    _check(_lib.atls_key_schedule(_engine()._e, hl, sh.ctypes.data, sl, hh.ctypes.data,
                                  None if fh is None else fh.ctypes.data, n, out.ctypes.data))
    return [tuple(out[(5 * i + j) * hl:(5 * i + j + 1) * hl].tobytes() for j in range(5)) for i in range(n)]


class KeySchedule:
    """net/key_schedule.rs:116-222 after the X25519 step: ``do_key_schedule(hash, hello_hash,
    shared_secret)`` gives the handshake traffic secrets and the master secret (Hkdf objects)."""

    def __init__(self, c_hs, s_hs, master):
        self.client_handshake_traffic_secret = c_hs
        self.server_handshake_traffic_secret = s_hs
        self.hkdf_master_secret = master

    @classmethod
    def do_key_schedule(cls, hash_type, hello_hash, shared_secret):
        c, s, m, _, _ = key_schedule_batch(hash_type, [shared_secret], [hello_hash])[0]
        h = HashType(hash_type)
        return cls(Hkdf.from_prk(h, c), Hkdf.from_prk(h, s), Hkdf.from_prk(h, m))


def application_secrets(hkdf_master_secret, handshake_hash):
    """WriteKeys::application_keys_from_master_secret (key_schedule.rs:87-114): the client and
    server application traffic secrets 0 as Hkdf objects."""
    h = hkdf_master_secret.hash
    hl = int(h)
    info_c = get_hkdf_expand_label(b"c ap traffic", handshake_hash, hl)
    info_s = get_hkdf_expand_label(b"s ap traffic", handshake_hash, hl)
    c, s = hkdf_expand_batch(h, [hkdf_master_secret.pseudo_random_key] * 2, [info_c, info_s], hl)
    return Hkdf.from_prk(h, c), Hkdf.from_prk(h, s)
