"""Synthetic TLS record batches (BASELINE.json configs) as engine descriptors.

A batch is: key slots (one per connection, KEY_DTYPE), record descriptors (REC_DTYPE), and
the byte sizes of the input/output buffers. Payload bytes are generated separately (host
numpy for tests, device tensors for the benchmark). Records are laid out back to back at
16-byte aligned offsets; TLS seal output holds content||type ciphertext (len + 1 bytes).
Connections are assigned round-robin (record i -> slot i % n_keys) and each connection's
records carry consecutive sequence numbers, as a record layer's writes would.
"""
import numpy as np

from . import KEY_DTYPE, MODE_TLS, MODE_WIRE, REC_DTYPE, CipherSuite

SEEDS = {"payload": 0x5EED0001, "keys": 0x5EED0002, "layout": 0x5EED0003}

CONFIGS = {
    # name: (suite or "mixed", n_records, content_len or (lo, hi)), BASELINE.json configs[1..4]
    "c2_aes128gcm_64Ki_x_16KiB": (CipherSuite.TLS_AES_128_GCM_SHA256, 65536, 16384),
    "c3_chacha20poly1305_64Ki_x_1.5KiB": (CipherSuite.TLS_CHACHA20_POLY1305_SHA256, 65536, 1536),
    "c4_aes256gcm_1Mi_x_16KiB": (CipherSuite.TLS_AES_256_GCM_SHA384, 1048576, 16384),
    "c5_mixed_256Ki_x_64B-16KiB": ("mixed", 262144, (64, 16384)),
}


def _round16(x):
    return (x + 15) & ~np.uint64(15) if isinstance(x, np.ndarray) else (x + 15) & ~15


def make_keys(n_keys, suites, seed=SEEDS["keys"], key_lens=None):
    """n_keys slots; suites: array of suite per slot. key_len from the suite unless given."""
    rng = np.random.default_rng(seed)
    keys = np.zeros(n_keys, dtype=KEY_DTYPE)
    keys["suite"] = suites
    if key_lens is None:
        key_lens = np.where(np.asarray(suites) == int(CipherSuite.TLS_AES_128_GCM_SHA256), 16, 32)
    keys["key_len"] = key_lens
    keys["iv_len"] = 12
    keys["key"] = rng.integers(0, 256, size=(n_keys, 32), dtype=np.uint8)
    keys["static_iv"] = rng.integers(0, 256, size=(n_keys, 12), dtype=np.uint8)
    return keys


def tls_batch(n, lens, suites_per_key, n_keys=4096, content_type=23, seq_base=0, first=0, shrink_keys=True):
    """n TLS-mode records; lens: int or array (content lengths). The records are entries
    first .. first+n-1 of a record stream in which entry g uses slot g % n_keys with sequence
    number seq_base + g // n_keys (a shard of a larger batch when first > 0)."""
    if shrink_keys:  # small ad-hoc batches: no more key slots than records
        n_keys = min(n_keys, first + n) if n else 1
    lens = np.broadcast_to(np.asarray(lens, dtype=np.uint64), (n,)).copy()
    recs = np.zeros(n, dtype=REC_DTYPE)
    in_sz = _round16(lens)
    out_sz = _round16(lens + 1)
    recs["in_off"] = np.concatenate([[0], np.cumsum(in_sz)[:-1]]).astype(np.uint64) if n else []
    recs["out_off"] = np.concatenate([[0], np.cumsum(out_sz)[:-1]]).astype(np.uint64) if n else []
    recs["len"] = lens.astype(np.uint32)
    g = np.arange(first, first + n, dtype=np.uint64)
    recs["key_slot"] = (g % np.uint64(n_keys)).astype(np.uint32)
    recs["seq"] = seq_base + g // np.uint64(n_keys)
    recs["content_type"] = content_type
    recs["mode"] = MODE_TLS
    keys = make_keys(n_keys, suites_per_key(n_keys) if callable(suites_per_key) else
                     np.full(n_keys, int(suites_per_key), dtype=np.uint16))
    return dict(keys=keys, recs=recs, in_bytes=int(in_sz.sum()) if n else 0,
                out_bytes=int(out_sz.sum()) if n else 0, payload=int(lens.sum() + n))


def wire_batch(b):
    """The batch b with its records sealed as one contiguous wire stream (ATLS_MODE_WIRE): record
    i's header || ciphertext || tag at out_off, 5 + len + 1 + 16 bytes, back to back as
    RecordPayloadProtection::encrypt's outputs go on the socket (record.rs:162-198)."""
    recs = b["recs"].copy()
    wl = recs["len"].astype(np.uint64) + np.uint64(22)
    recs["out_off"] = np.concatenate([[0], np.cumsum(wl)[:-1]]).astype(np.uint64) if len(recs) else []
    recs["mode"] = MODE_WIRE
    return dict(b, recs=recs, out_bytes=int(wl.sum()) if len(recs) else 0)


def wire_open_descs(sealed):
    """Open descriptors for a wire stream sealed with `sealed` (wire_batch records): each record
    read at its wire offset with len = ciphertext bytes, plaintext out 16-byte aligned."""
    recs = sealed.copy()
    L = recs["len"].astype(np.uint64) + np.uint64(1)
    recs["in_off"] = sealed["out_off"]
    recs["len"] = L.astype(np.uint32)
    recs["out_off"] = np.concatenate([[0], np.cumsum(_round16(L))[:-1]]).astype(np.uint64) if len(recs) else []
    return recs, int(_round16(L).sum()) if len(recs) else 0


def config_batch(name, n=None, first=0, n_keys=None):
    """Descriptors for a BASELINE config: records first .. first+n-1 of it (default: all).
    n_keys overrides the config's 4,096 connections (n_keys = records: a key per record, the
    SURVEY §8d worst case)."""
    suite, n_full, lens = CONFIGS[name]
    n = n_full - first if n is None else n
    nk = min(4096, n_full) if n_keys is None else int(n_keys)
    if suite == "mixed":
        rng = np.random.default_rng(SEEDS["layout"])
        lo, hi = lens
        L = rng.integers(lo, hi + 1, size=max(n_full, first + n), dtype=np.uint64)[first:first + n]

        def suites(k):
            r = np.random.default_rng(SEEDS["layout"] + 1)
            return np.where(r.random(k) < 0.5, int(CipherSuite.TLS_AES_128_GCM_SHA256),
                            int(CipherSuite.TLS_CHACHA20_POLY1305_SHA256)).astype(np.uint16)

        return tls_batch(n, L, suites, n_keys=nk, first=first, shrink_keys=False)
    return tls_batch(n, lens, int(suite), n_keys=nk, first=first, shrink_keys=False)


# Configs BASELINE.json quotes on 8 GPUs: their records are split evenly over 8 ranks, and a rank
# keeps that share whatever the GPU count (weak scaling). The others run whole on every GPU.
EIGHT_GPU_CONFIGS = ("c4_aes256gcm_1Mi_x_16KiB", "c5_mixed_256Ki_x_64B-16KiB")


def records_per_rank(name):
    n_full = CONFIGS[name][1]
    return n_full // 8 if name in EIGHT_GPU_CONFIGS else n_full


def capped(b, cap):
    """The batch b with every content length cut to at most `cap` bytes and the records re-packed
    (same records, keys, slots and sequence numbers). For CPU rehearsals of whole-config exchanges
    (bench.py --dry-run): C4's 1 Mi records at 16 KiB are 34 GB of buffers, at 64 B 150 MB."""
    recs = b["recs"].copy()
    lens = np.minimum(recs["len"].astype(np.uint64), np.uint64(cap))
    in_sz, out_sz = _round16(lens), _round16(lens + np.uint64(1))
    n = len(recs)
    recs["len"] = lens.astype(np.uint32)
    recs["in_off"] = np.concatenate([[0], np.cumsum(in_sz)[:-1]]).astype(np.uint64) if n else []
    recs["out_off"] = np.concatenate([[0], np.cumsum(out_sz)[:-1]]).astype(np.uint64) if n else []
    return dict(b, recs=recs, in_bytes=int(in_sz.sum()) if n else 0, out_bytes=int(out_sz.sum()) if n else 0,
                payload=int(lens.sum() + n))


def shard_batch(name, rank, n=None, n_keys=None):
    """Rank `rank`'s shard: records rank*n .. rank*n+n-1 of the config's record stream (key slots,
    sequence numbers and lengths as in the unsharded batch). n defaults to records_per_rank()."""
    n = records_per_rank(name) if n is None else n
    return config_batch(name, n=n, first=rank * n, n_keys=n_keys)
