"""anothertls_amd — MI355X-native TLS 1.3 record-layer AEAD engine (host-side Python mirror).

The product is the C-ABI library ``libatls.so`` (include/atls.h): hand-written gfx950 HIP
kernels for AES-GCM and ChaCha20-Poly1305 plus a C++ engine. This module binds it with
ctypes and mirrors the reference's cipher interface (otsmr/AnotherTLS, paths relative to
anothertls/src):

* ``CipherSuite`` / ``get_cipher()`` / ``get_key_and_iv_len()`` — crypto/ciphersuite.rs:33-87
* ``Gcm`` / ``Poly1305`` with ``encrypt(key, iv, plaintext, aad) -> (ct, tag)`` and
  ``decrypt(key, iv, ct, aad, tag) -> pt`` raising ``TlsError`` — the ``Cipher`` trait,
  crypto/ciphersuite.rs:12-31 (gcm.rs:131-162, poly1305.rs:69-104)
* ``Engine`` — the batched record API (atls_engine_*, atls_*_batch) used by the record layer
  and the benchmark.

There is no CPU fallback: importing works without a GPU, but every compute call raises
``TlsError(INTERNAL_ERROR)`` when no HIP device is usable, and importing fails loudly if the
library has not been built (``python -m anothertls_amd._build``).
"""
import ctypes
import enum
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ATLS_LIB") or os.path.join(_HERE, "libatls.so")  # ATLS_LIB: tuning variants

if not os.path.exists(LIB_PATH):
    raise ImportError(f"anothertls_amd: {LIB_PATH} is missing; build it with `python anothertls_amd/_build.py`")

# One HIP runtime per process: PyTorch-ROCm bundles its own libamdhip64 (same SONAME). If torch is
# installed, load it first so libatls.so binds to that already-loaded runtime instead of pulling a
# second copy from /opt/rocm (two runtimes in one process cannot both open the device). torch is
# used only as plumbing by callers that pass device tensors; the library itself does not need it.
if os.environ.get("ATLS_NO_TORCH_RUNTIME") != "1":
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
_lib = ctypes.CDLL(LIB_PATH)

_c = ctypes
_u8p = _c.POINTER(_c.c_uint8)
_lib.atls_seal.argtypes = [_c.c_uint16, _c.c_void_p, _c.c_size_t, _c.c_void_p, _c.c_size_t, _c.c_void_p,
                           _c.c_size_t, _c.c_void_p, _c.c_size_t, _c.c_void_p, _c.c_void_p]
_lib.atls_open.argtypes = [_c.c_uint16, _c.c_void_p, _c.c_size_t, _c.c_void_p, _c.c_size_t, _c.c_void_p,
                           _c.c_size_t, _c.c_void_p, _c.c_size_t, _c.c_void_p, _c.c_size_t, _c.c_void_p]
_lib.atls_engine_create.restype = _c.c_void_p
_lib.atls_engine_create.argtypes = [_c.c_int]
_lib.atls_engine_destroy.argtypes = [_c.c_void_p]
_lib.atls_engine_sync.argtypes = [_c.c_void_p]
_lib.atls_engine_join.argtypes = [_c.c_void_p]
_lib.atls_engine_stream.restype = _c.c_void_p
_lib.atls_engine_stream.argtypes = [_c.c_void_p]
_lib.atls_set_keys.argtypes = [_c.c_void_p, _c.c_void_p, _c.c_uint32]
_lib.atls_update_keys.argtypes = [_c.c_void_p, _c.c_uint32, _c.c_void_p, _c.c_uint32]
_lib.atls_seal_batch.argtypes = [_c.c_void_p, _c.c_void_p, _c.c_uint32, _c.c_void_p, _c.c_void_p, _c.c_void_p,
                                 _c.c_void_p, _c.c_uint32]
_lib.atls_open_batch.argtypes = [_c.c_void_p, _c.c_void_p, _c.c_uint32, _c.c_void_p, _c.c_void_p, _c.c_void_p,
                                 _c.c_void_p, _c.c_void_p, _c.c_uint32]
_lib.atls_derive_keys.argtypes = [_c.c_void_p, _c.c_uint16, _c.c_void_p, _c.c_size_t, _c.c_uint32, _c.c_void_p]
_lib.atls_aes_blocks.argtypes = [_c.c_void_p, _c.c_int, _c.c_uint32, _c.c_void_p, _c.c_void_p, _c.c_size_t,
                                 _c.c_uint32]
_lib.atls_aes_block.argtypes = [_c.c_int, _c.c_void_p, _c.c_size_t, _c.c_void_p, _c.c_void_p]
_lib.atls_device_arch.restype = _c.c_char_p
_lib.atls_multi_create.restype = _c.c_void_p
_lib.atls_multi_create.argtypes = [_c.c_void_p, _c.c_int]
_lib.atls_multi_destroy.argtypes = [_c.c_void_p]
_lib.atls_multi_devices.argtypes = [_c.c_void_p]
_lib.atls_multi_uses_rccl.argtypes = [_c.c_void_p]
_lib.atls_multi_rccl_version.argtypes = [_c.c_void_p]
_lib.atls_multi_max_message.argtypes = [_c.c_void_p]
_lib.atls_multi_max_message.restype = _c.c_size_t
_lib.atls_multi_set_keys.argtypes = [_c.c_void_p, _c.c_void_p, _c.c_uint32]
_lib.atls_multi_seal_batch.argtypes = _lib.atls_seal_batch.argtypes
_lib.atls_multi_open_batch.argtypes = _lib.atls_open_batch.argtypes
_lib.atls_partition.restype = None
_lib.atls_clock_probe.argtypes = [_c.c_void_p, _c.c_void_p, _c.c_uint32, _c.c_uint32, _c.c_uint32, _c.c_void_p]
_lib.atls_partition.argtypes = [_c.c_void_p, _c.c_uint32, _c.c_int, _c.c_uint32, _c.c_void_p]


class TlsError(Exception):
    """net/alert.rs:18-45 TlsError; ``code`` is the u8 discriminant."""

    OK = 0
    BAD_RECORD_MAC = 20
    ILLEGAL_PARAMETER = 47
    DECRYPT_ERROR = 50
    DECODE_ERROR = 51
    INSUFFICIENT_SECURITY = 71
    INTERNAL_ERROR = 80
    _names = {20: "BadRecordMac", 47: "IllegalParameter", 50: "DecryptError", 51: "DecodeError",
              71: "InsufficientSecurity", 80: "InternalError"}

    def __init__(self, code):
        self.code = int(code)
        super().__init__(f"TlsError::{self._names.get(self.code, self.code)} ({self.code})")


def _check(rc):
    if rc != 0:
        raise TlsError(rc)


# ---- numpy mirrors of the C structs (include/atls.h) ----------------------------------------
KEY_DTYPE = np.dtype([("suite", "<u2"), ("key_len", "u1"), ("iv_len", "u1"), ("key", "u1", 32),
                      ("static_iv", "u1", 12), ("reserved", "u1", 16)])
REC_DTYPE = np.dtype([("in_off", "<u8"), ("out_off", "<u8"), ("aux_off", "<u8"), ("seq", "<u8"),
                      ("len", "<u4"), ("key_slot", "<u4"), ("aad_len", "<u2"), ("content_type", "u1"),
                      ("mode", "u1"), ("iv_len", "u1"), ("reserved", "u1", 3)])
OPEN_RESULT_DTYPE = np.dtype([("content_len", "<u4"), ("status", "u1"), ("content_type", "u1"),
                              ("reserved", "u1", 2)])
assert KEY_DTYPE.itemsize == 64 and REC_DTYPE.itemsize == 48 and OPEN_RESULT_DTYPE.itemsize == 8

MODE_TLS, MODE_RAW, MODE_WIRE = 0, 1, 2
FLAG_DEVICE_PTRS, FLAG_DEVICE_RECS, FLAG_NO_SYNC, FLAG_LAZY_JOIN = 1, 2, 4, 8


class CipherSuite(enum.IntEnum):
    """crypto/ciphersuite.rs:33-40."""

    TLS_AES_256_GCM_SHA384 = 0x1302
    TLS_CHACHA20_POLY1305_SHA256 = 0x1303
    TLS_AES_128_GCM_SHA256 = 0x1301
    TLS_EMPTY_RENEGOTIATION_INFO_SCSV = 0x00FF

    @classmethod
    def new(cls, x):  # ciphersuite.rs:43-51
        try:
            return cls(x)
        except ValueError:
            raise TlsError(TlsError.INSUFFICIENT_SECURITY) from None

    def as_u16(self):
        return int(self)

    def get_key_and_iv_len(self):  # ciphersuite.rs:69-77
        return (16, 12) if self == CipherSuite.TLS_AES_128_GCM_SHA256 else (32, 12)

    def get_hash_len(self):  # ciphersuite.rs:60-68 (get_tshash): SHA-384 for 0x1302, else SHA-256
        if self == CipherSuite.TLS_EMPTY_RENEGOTIATION_INFO_SCSV:
            raise TlsError(TlsError.INSUFFICIENT_SECURITY)
        return 48 if self == CipherSuite.TLS_AES_256_GCM_SHA384 else 32

    def get_cipher(self):  # ciphersuite.rs:78-87
        if self in (CipherSuite.TLS_AES_256_GCM_SHA384, CipherSuite.TLS_AES_128_GCM_SHA256):
            return Gcm(self)
        if self == CipherSuite.TLS_CHACHA20_POLY1305_SHA256:
            return Poly1305()
        raise TlsError(TlsError.INSUFFICIENT_SECURITY)


def _bytes_arg(b):
    b = bytes(b)
    return ctypes.create_string_buffer(b, max(len(b), 1)), len(b)


class _DeviceCipher:
    """The Cipher trait over atls_seal / atls_open (GPU; one record per call)."""

    _suite = None

    def get_cipher_suite(self):
        return self._suite

    def encrypt(self, key, iv, plaintext, additional_data=b""):
        k, kl = _bytes_arg(key)
        v, vl = _bytes_arg(iv)
        a, al = _bytes_arg(additional_data)
        p, n = _bytes_arg(plaintext)
        out = ctypes.create_string_buffer(max(n, 1))
        tag = ctypes.create_string_buffer(16)
        _check(_lib.atls_seal(int(self._suite), k, kl, v, vl, a, al, p, n, out, tag))
        return out.raw[:n], tag.raw

    def decrypt(self, key, iv, ciphertext, additional_data, auth_tag):
        k, kl = _bytes_arg(key)
        v, vl = _bytes_arg(iv)
        a, al = _bytes_arg(additional_data)
        c, n = _bytes_arg(ciphertext)
        t, tl = _bytes_arg(auth_tag)
        out = ctypes.create_string_buffer(max(n, 1))
        _check(_lib.atls_open(int(self._suite), k, kl, v, vl, a, al, c, n, t, tl, out))
        return out.raw[:n]


class Gcm(_DeviceCipher):
    """crypto/aes/gcm.rs:15-162 — AES-GCM; AES-128/192/256 chosen by key length (gcm.rs:49)."""

    def __init__(self, cs=CipherSuite.TLS_AES_128_GCM_SHA256):
        self._suite = CipherSuite(cs)


class Poly1305(_DeviceCipher):
    """crypto/chacha20/poly1305.rs:15-104 — ChaCha20-Poly1305 (RFC 8439, with the reference's
    last-block behaviour when len % 64 == 0)."""

    _suite = CipherSuite.TLS_CHACHA20_POLY1305_SHA256


class AES:
    """crypto/aes/cipher.rs:159-215 ``AES``: ``AES.init(key, blocksize)`` then ``encrypt`` /
    ``decrypt`` of one 16-byte block, on the device (atls_aes_block). ``blocksize`` is the key
    size in bits (cipher.rs:141-156 Blocksize); a key of another length is ILLEGAL_PARAMETER
    where the reference would index out of bounds."""

    def __init__(self, key, blocksize=None):
        self.key = bytes(key)
        bits = len(self.key) * 8 if blocksize is None else int(blocksize)
        if bits not in (128, 192, 256) or bits != len(self.key) * 8:
            raise TlsError(TlsError.ILLEGAL_PARAMETER)

    @classmethod
    def init(cls, key, blocksize=None):
        return cls(key, blocksize)

    def _run(self, decrypt, block):
        block = bytes(block)
        if len(block) != 16:
            raise TlsError(TlsError.ILLEGAL_PARAMETER)
        out = _c.create_string_buffer(16)
        _check(_lib.atls_aes_block(int(decrypt), self.key, len(self.key), block, out))
        return out.raw

    def encrypt(self, block):  # cipher.rs:175-194
        return self._run(False, block)

    def decrypt(self, block):  # cipher.rs:196-215
        return self._run(True, block)


def device_available():
    """True when the HIP runtime sees a device the engine can open."""
    e = _lib.atls_engine_create(int(os.environ.get("ATLS_DEVICE", "0")))
    if not e:
        return False
    _lib.atls_engine_destroy(e)
    return True


def make_keys(entries):
    """entries: iterable of (suite, key_bytes, static_iv_bytes) -> KEY_DTYPE array."""
    entries = list(entries)
    arr = np.zeros(len(entries), dtype=KEY_DTYPE)
    for i, (suite, key, iv) in enumerate(entries):
        arr[i]["suite"] = int(suite)
        arr[i]["key_len"] = len(key)
        arr[i]["iv_len"] = len(iv)
        arr[i]["key"][: len(key)] = np.frombuffer(bytes(key), np.uint8)
        arr[i]["static_iv"][: len(iv)] = np.frombuffer(bytes(iv), np.uint8)
    return arr


def _ptr(x):
    """numpy array -> host pointer; torch tensor (any device) -> data_ptr; int -> as is."""
    if x is None:
        return None
    if isinstance(x, int):
        return x
    if isinstance(x, np.ndarray):
        return x.ctypes.data
    if hasattr(x, "data_ptr"):
        return x.data_ptr()
    raise TypeError(type(x))


class Engine:
    """One HIP device: key slots + batched seal/open (include/atls.h engine API)."""

    def __init__(self, device=0):
        self._e = _lib.atls_engine_create(int(device))
        if not self._e:
            raise TlsError(TlsError.INTERNAL_ERROR)
        self.device = device

    def close(self):
        if self._e:
            _lib.atls_engine_destroy(self._e)
            self._e = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def stream(self):
        return _lib.atls_engine_stream(self._e)

    def sync(self):
        _check(_lib.atls_engine_sync(self._e))

    def join(self):
        """atls_engine_join: the engine stream waits for the side kernels of FLAG_LAZY_JOIN batches."""
        _check(_lib.atls_engine_join(self._e))

    def set_keys(self, keys):
        keys = np.ascontiguousarray(keys, dtype=KEY_DTYPE)
        _check(_lib.atls_set_keys(self._e, keys.ctypes.data, len(keys)))

    def clock_probe(self, out, wgs=8, delay_us=0, spin_us=1000, stream=None):
        """Enqueue the shader-clock probe (atls_clock_probe): `out` a device tensor of >= 2 * wgs int64, on
        `stream` (a hipStream_t handle; None = the engine's stream). SCLK MHz = 100 * out[2w] / out[2w+1]."""
        _check(_lib.atls_clock_probe(self._e, stream, int(wgs), int(delay_us), int(spin_us), _ptr(out)))

    def update_keys(self, first, keys):
        """Install key slots [first, first + len(keys)), keeping the other slots."""
        keys = np.ascontiguousarray(keys, dtype=KEY_DTYPE)
        _check(_lib.atls_update_keys(self._e, int(first), keys.ctypes.data, len(keys)))

    def derive_keys(self, suite, secrets):
        """Key::from_hkdf for each traffic secret (bytes-like, n * hash_len) -> KEY_DTYPE array."""
        hl = CipherSuite(suite).get_hash_len()
        buf = np.frombuffer(bytes(secrets), np.uint8)
        n = len(buf) // hl
        out = np.zeros(n, dtype=KEY_DTYPE)
        _check(_lib.atls_derive_keys(self._e, int(suite), buf.ctypes.data, hl, n, out.ctypes.data))
        return out

    def _after_torch(self, *xs):
        """Device tensors from PyTorch: the engine's stream waits for the work already queued on
        torch's current stream (e.g. the fill of a fresh torch.zeros output), without a host sync.
        The event and the engine-stream wrapper are made once per engine (a batch call then costs
        one event record and one stream wait)."""
        for x in xs:
            if getattr(x, "is_cuda", False):
                import torch

                if getattr(self, "_torch_sync", None) is None or self._torch_sync[0] != x.device:
                    self._torch_sync = (x.device, torch.cuda.Event(),
                                        torch.cuda.ExternalStream(self.stream, device=x.device))
                _, ev, ext = self._torch_sync
                ev.record(torch.cuda.current_stream(x.device))
                ext.wait_event(ev)
                return

    def seal_batch(self, recs, inp, aux, out, tags, flags=0, n=None):
        n = len(recs) if n is None else n
        self._after_torch(recs, inp, aux, out, tags)
        _check(_lib.atls_seal_batch(self._e, _ptr(recs), n, _ptr(inp), _ptr(aux), _ptr(out), _ptr(tags), flags))

    def aes_blocks(self, decrypt, key_slot, inp, out, flags=0, nblocks=None):
        """AES::encrypt / decrypt of every 16-byte block of inp under key slot key_slot."""
        self._after_torch(inp, out)
        nb = (inp.nbytes if hasattr(inp, "nbytes") else inp.numel()) // 16 if nblocks is None else nblocks
        _check(_lib.atls_aes_blocks(self._e, int(decrypt), int(key_slot), _ptr(inp), _ptr(out), nb, flags))

    def open_batch(self, recs, inp, aux, tags, out, results, flags=0, n=None):
        n = len(recs) if n is None else n
        self._after_torch(recs, inp, aux, tags, out, results)
        _check(_lib.atls_open_batch(self._e, _ptr(recs), n, _ptr(inp), _ptr(aux), _ptr(tags), _ptr(out),
                                    _ptr(results), flags))


def partition(recs, parts, open_=False):
    """atls_partition: record boundaries [first[p], first[p+1]) of `parts` contiguous ranges
    balanced by cumulative bytes (read + written + 16-byte tag per record). Host-only."""
    recs = np.ascontiguousarray(recs, dtype=REC_DTYPE)
    first = np.zeros(parts + 1, np.uint32)
    _lib.atls_partition(recs.ctypes.data, len(recs), int(bool(open_)), parts, first.ctypes.data)
    return first


class MultiEngine:
    """Several HIP devices in one process (atls_multi_*): a batch is split by cumulative bytes
    into one contiguous record range per device; device-resident buffers live on devices[0] and
    the other ranges travel over RCCL (distinct devices) or device copies (repeated devices)."""

    def __init__(self, devices):
        self.devices = [int(d) for d in devices]
        arr = (_c.c_int * len(self.devices))(*self.devices)
        self._m = _lib.atls_multi_create(arr, len(self.devices))
        if not self._m:
            raise TlsError(TlsError.INTERNAL_ERROR)

    @property
    def uses_rccl(self):
        return bool(_lib.atls_multi_uses_rccl(self._m))

    @property
    def rccl_version(self):
        """ncclGetVersion of the RCCL in use (e.g. 22606 = 2.26.6), 0 without RCCL."""
        return int(_lib.atls_multi_rccl_version(self._m))

    @property
    def max_message(self):
        """Largest RCCL point-to-point message in bytes (0 without RCCL)."""
        return int(_lib.atls_multi_max_message(self._m))

    def close(self):
        if self._m:
            _lib.atls_multi_destroy(self._m)
            self._m = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_keys(self, keys):
        keys = np.ascontiguousarray(keys, dtype=KEY_DTYPE)
        _check(_lib.atls_multi_set_keys(self._m, keys.ctypes.data, len(keys)))

    def _after_torch(self, *xs):
        for x in xs:
            if getattr(x, "is_cuda", False):
                import torch

                torch.cuda.synchronize(x.device)
                return

    def seal_batch(self, recs, inp, aux, out, tags, flags=0):
        recs = np.ascontiguousarray(recs, dtype=REC_DTYPE)
        self._after_torch(inp, aux, out, tags)
        _check(_lib.atls_multi_seal_batch(self._m, recs.ctypes.data, len(recs), _ptr(inp), _ptr(aux), _ptr(out),
                                          _ptr(tags), flags))

    def open_batch(self, recs, inp, aux, tags, out, results, flags=0):
        recs = np.ascontiguousarray(recs, dtype=REC_DTYPE)
        self._after_torch(inp, aux, tags, out, results)
        _check(_lib.atls_multi_open_batch(self._m, recs.ctypes.data, len(recs), _ptr(inp), _ptr(aux), _ptr(tags),
                                          _ptr(out), _ptr(results), flags))


def abi_version():
    return _lib.atls_abi_version()


def library():
    """The loaded ctypes library (for the ABI tests)."""
    return _lib
