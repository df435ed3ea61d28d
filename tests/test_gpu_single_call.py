"""The Cipher-trait drop-in (atls_seal / atls_open) as the reference's record layer uses it: one
call per record, from any thread (Arc<dyn Cipher + Send + Sync>, crypto/ciphersuite.rs:78-87,
net/record.rs:191-193): concurrent calls from several threads (more threads than the bounded pool of
call contexts, ATLS_SINGLE_CONTEXTS = 8), records read in place from mapped pinned memory (up to
1 MiB) and copied once (longer), the key cache across
evictions, the ChaCha20 f32 block-count limit (chacha20/cipher.rs:94), and atls_update_keys."""
import os
import random
import threading

import numpy as np
import pytest

import anothertls_amd as atls
import oracle as ora
from anothertls_amd import workload

pytestmark = pytest.mark.gpu


def _case(rng, keys):
    suite, key = rng.choice(keys)
    n = rng.choice([0, 1, 15, 16, 17, 63, 64, 127, 1536, 1537, 4096, 16385])
    iv = bytes(rng.getrandbits(8) for _ in range(12))
    aad = bytes(rng.getrandbits(8) for _ in range(rng.choice([0, 5, 13])))
    pt = bytes(rng.getrandbits(8) for _ in range(n))
    return suite, key, iv, aad, pt


@pytest.mark.parametrize("n_threads", [8, 20])  # 20 > the 8 pooled contexts: callers wait for one
def test_concurrent_threads_vs_oracle(n_threads):
    rng0 = random.Random(5)
    keys = [(s, bytes(rng0.getrandbits(8) for _ in range(kl))) for s, kl in
            [(0x1301, 16), (0x1301, 16), (0x1302, 32), (0x1301, 24), (0x1303, 32), (0x1303, 32)]]
    errors = []

    def worker(t):
        rng = random.Random(100 + t)
        try:
            for _ in range(40):
                suite, key, iv, aad, pt = _case(rng, keys)
                c = atls.CipherSuite(suite).get_cipher()
                ct, tag = c.encrypt(key, iv, pt, aad)
                rc, ect, etag = ora.cipher_encrypt(suite, key, iv, pt, aad)
                assert rc == 0 and ct == ect and tag == etag, (t, suite, len(pt))
                assert c.decrypt(key, iv, ct, aad, tag) == pt
                with pytest.raises(atls.TlsError) as e:
                    c.decrypt(key, iv, ct, aad, bytes([tag[0] ^ 1]) + tag[1:])
                assert e.value.code == 20
        except BaseException as exc:  # noqa: BLE001 -- reported by the main thread
            errors.append(exc)

    threads = [threading.Thread(target=worker, args=(t,)) for t in range(n_threads)]
    for th in threads:
        th.start()
    for th in threads:
        th.join(120)
    assert not errors, errors[:3]


def test_key_cache_eviction_cycles():
    rng = random.Random(9)
    keys = [bytes(rng.getrandbits(8) for _ in range(16)) for _ in range(40)]  # > 16 cached slots
    c = atls.Gcm()
    for rnd in range(2):
        for i, k in enumerate(keys):
            pt = bytes([i, rnd]) * 100
            iv = bytes([rnd]) * 12
            ct, tag = c.encrypt(k, iv, pt, b"hdr")
            rc, ect, etag = ora.gcm_encrypt(k, iv, pt, b"hdr")
            assert rc == 0 and (ct, tag) == (ect, etag), (rnd, i)


def test_chacha_f32_block_count_limit():
    key, iv = bytes(range(32)), bytes(12)
    c = atls.Poly1305()
    with pytest.raises(atls.TlsError) as e:  # 2^24 + 1: the reference's f32 ceil drops the last byte
        c.encrypt(key, iv, bytes(2**24 + 1))
    assert e.value.code == 47
    # the largest accepted length is exact in f32 and matches the oracle
    pt = np.random.default_rng(1).integers(0, 256, 2**24 - 1, dtype=np.uint8).tobytes()
    ct, tag = c.encrypt(key, iv, pt, b"")
    rc, ect, etag = ora.chacha_poly_encrypt(key, iv, pt, b"")
    assert rc == 0 and ct == ect and tag == etag
    # batch path: a TLS seal of 2^24 - 1 content bytes is a 2^24-byte AEAD input -> refused
    eng = atls.Engine(0)
    b = workload.tls_batch(2, np.array([100, 2**24 - 1], np.uint64), 0x1303, n_keys=1)
    eng.set_keys(b["keys"])
    inbuf = np.zeros(b["in_bytes"] + 16, np.uint8)
    out = np.zeros(b["out_bytes"] + 16, np.uint8)
    with pytest.raises(atls.TlsError) as e:
        eng.seal_batch(b["recs"], inbuf, np.zeros(16, np.uint8), out, np.zeros(32, np.uint8))
    assert e.value.code == 47
    eng.close()


def test_update_keys_keeps_other_slots():
    from test_gpu_parity import fill_payload, oracle_keys, oracle_recs

    def suites(k):
        return np.array([0x1301, 0x1303, 0x1302, 0x1301][:k], np.uint16)

    b = workload.tls_batch(8, 3000, suites, n_keys=4)
    eng = atls.Engine(0)
    eng.set_keys(b["keys"][:3])
    new = workload.make_keys(2, np.array([0x1302, 0x1301], np.uint16), seed=77)
    eng.update_keys(2, new)  # replaces slot 2, appends slot 3
    keys = b["keys"].copy()
    keys[2:4] = new
    inbuf = fill_payload(b, 4)
    out = np.zeros(b["out_bytes"] + 16, np.uint8)
    tags = np.zeros(16 * 8, np.uint8)
    eng.seal_batch(b["recs"], inbuf, np.zeros(16, np.uint8), out, tags)
    oout, otags = np.zeros_like(out), np.zeros_like(tags)
    assert ora.seal_batch(oracle_keys(keys), oracle_recs(b["recs"]), inbuf, np.zeros(16, np.uint8), oout, otags, 4) == 0
    assert np.array_equal(tags, otags) and np.array_equal(out, oout)
    with pytest.raises(atls.TlsError):
        eng.update_keys(9, new)  # would leave a gap
    eng.close()


@pytest.mark.parametrize("suite,klen", [(0x1301, 16), (0x1302, 24), (0x1302, 32), (0x1303, 32)])
def test_argument_block_boundary_vs_oracle(suite, klen):
    """Single calls whose IV || AAD || input (|| tag on open) fit the launch's argument block (3,584 B,
    csrc/plan.h kSingleInline: gcm_single / chacha_single) and the first ones that do not (pinned-block
    kernels), each side of the boundary, with 12- and 16-byte IVs (GCM) and 0..40-byte AADs."""
    rng = random.Random(klen * 7 + suite)
    key = bytes(rng.getrandbits(8) for _ in range(klen))
    c = atls.CipherSuite(suite if suite != 0x1302 or klen == 32 else 0x1301).get_cipher()
    for iv_len in ([12, 16] if suite != 0x1303 else [12]):
        for aad_len in (0, 5, 40):
            head = (iv_len + aad_len + 15) // 16 * 16
            for n in (3584 - head - 32, 3584 - head - 17, 3584 - head - 16, 3584 - head - 1, 3584 - head, 3600):
                iv = bytes(rng.getrandbits(8) for _ in range(iv_len))
                aad = bytes(rng.getrandbits(8) for _ in range(aad_len))
                pt = bytes(rng.getrandbits(8) for _ in range(n))
                ct, tag = c.encrypt(key, iv, pt, aad)
                rc, ect, etag = ora.cipher_encrypt(suite, key, iv, pt, aad)
                assert rc == 0 and ct == ect and tag == etag, (iv_len, aad_len, n)
                assert c.decrypt(key, iv, ct, aad, tag) == pt
                with pytest.raises(atls.TlsError) as e:
                    c.decrypt(key, iv, ct, aad, tag[:15] + bytes([tag[15] ^ 0x80]))
                assert e.value.code == 20


@pytest.mark.parametrize("suite,klen", [(0x1301, 16), (0x1302, 32)])
def test_single_first_step_boundary_vs_oracle(suite, klen):
    """The single-call kernel's branch-free first step (gcm.hip ATLS_SINGLE_FAST_FIRST: lane 0 E_K(J0),
    lane 1 the AAD block, lanes 2-63 data) takes records with one AAD block (1..16 B), a 96-bit IV and at
    least 62 whole data blocks; both sides of that boundary, seal and open, against the oracle."""
    rng = random.Random(klen * 13 + suite)
    key = bytes(rng.getrandbits(8) for _ in range(klen))
    c = atls.CipherSuite(suite).get_cipher()
    for aad_len in (0, 1, 5, 13, 16, 17):
        for n in (975, 991, 992, 993, 1008, 1009, 1024, 2047, 3000):
            iv = bytes(rng.getrandbits(8) for _ in range(12))
            aad = bytes(rng.getrandbits(8) for _ in range(aad_len))
            pt = bytes(rng.getrandbits(8) for _ in range(n))
            ct, tag = c.encrypt(key, iv, pt, aad)
            rc, ect, etag = ora.cipher_encrypt(suite, key, iv, pt, aad)
            assert rc == 0 and ct == ect and tag == etag, (aad_len, n)
            assert c.decrypt(key, iv, ct, aad, tag) == pt
            with pytest.raises(atls.TlsError):
                c.decrypt(key, iv, ct, aad, bytes([tag[0] ^ 1]) + tag[1:])


@pytest.mark.parametrize("suite,klen", [(0x1301, 16), (0x1302, 32)])
def test_four_wave_step_boundaries_vs_oracle(suite, klen):
    """The AES-GCM single call spreads a record over four waves (gcm.hip gcm_record LN = 256: 256 slots per
    step, H^256 Horner, combine multipliers up to H^256): records whose slot count lands on each side of
    256 / 512 / 1,024, in the argument block and from the pinned block, 12- and 16-byte IVs, AADs of 0-40
    bytes; seal, open and a tampered tag against the oracle."""
    rng = random.Random(klen * 31 + suite)
    key = bytes(rng.getrandbits(8) for _ in range(klen))
    c = atls.CipherSuite(suite).get_cipher()
    for iv_len in (12, 16):
        for aad_len in (0, 5, 40):
            for n in (976, 992, 1008, 3520, 4064, 4080, 4096, 8160, 8176, 8192, 16336, 16352, 16368, 16385):
                iv = bytes(rng.getrandbits(8) for _ in range(iv_len))
                aad = bytes(rng.getrandbits(8) for _ in range(aad_len))
                pt = bytes(rng.getrandbits(8) for _ in range(n))
                ct, tag = c.encrypt(key, iv, pt, aad)
                rc, ect, etag = ora.cipher_encrypt(suite, key, iv, pt, aad)
                assert rc == 0 and ct == ect and tag == etag, (iv_len, aad_len, n)
                assert c.decrypt(key, iv, ct, aad, tag) == pt
                with pytest.raises(atls.TlsError):
                    c.decrypt(key, iv, ct, aad, tag[:8] + bytes([tag[8] ^ 4]) + tag[9:])


def test_chacha_four_wave_record_vs_oracle():
    """The ChaCha20-Poly1305 single call on four waves (chacha.hip chacha_record G = 256: slot j on thread
    j mod 256, per-wave power scans with the wave factor r^(256 w), the Horner factor r^1024, partial tags
    and content-type maxima meeting in LDS): lengths from empty to past one 256-slot step (16,305 B and
    up take two), the F4 quirk lengths (n % 64 == 0, cipher.rs:99-102), AADs of 0-40 bytes; seal, open
    and a tampered tag against the oracle."""
    rng = random.Random(0xC4A)
    key = bytes(rng.getrandbits(8) for _ in range(32))
    c = atls.CipherSuite(0x1303).get_cipher()
    for aad_len in (0, 5, 40):
        for n in (0, 1, 63, 64, 65, 1536, 1537, 3500, 4096, 8191, 16304, 16320, 16336, 16383, 16384, 16385):
            iv = bytes(rng.getrandbits(8) for _ in range(12))
            aad = bytes(rng.getrandbits(8) for _ in range(aad_len))
            pt = bytes(rng.getrandbits(8) for _ in range(n))
            ct, tag = c.encrypt(key, iv, pt, aad)
            rc, ect, etag = ora.cipher_encrypt(0x1303, key, iv, pt, aad)
            assert rc == 0 and ct == ect and tag == etag, (aad_len, n)
            assert c.decrypt(key, iv, ct, aad, tag) == pt
            with pytest.raises(atls.TlsError):
                c.decrypt(key, iv, ct, aad, tag[:15] + bytes([tag[15] ^ 0x40]))


@pytest.mark.parametrize("suite,klen", [(0x1301, 16), (0x1302, 32), (0x1303, 32)])
def test_long_single_calls_vs_oracle(suite, klen):
    """Single calls far past the argument block: AES-GCM records around the counter cache's
    limit (16,384 slots = 262,144 B of slots: past it gcm_record runs without the cache) and just past the
    1 MiB read-in-place limit (the record is copied into device memory first), 12- and 16-byte IVs, AADs of
    0 / 5 / 40 bytes; ChaCha20-Poly1305 across the same 1 MiB limit. Seal, open and a tampered tag against
    the oracle (crypto/aes/gcm.rs:42-162, crypto/chacha20/poly1305.rs:69-104)."""
    rng = np.random.default_rng(klen * 101 + suite)
    key = rng.integers(0, 256, klen, dtype=np.uint8).tobytes()
    c = atls.CipherSuite(suite).get_cipher()
    gcm = suite != 0x1303
    lens = (262096, 262112, 262128, 262145, 1048560, 1048577) if gcm else (1048512, 1048576, 1048577)
    for iv_len in ((12, 16) if gcm else (12,)):
        for aad_len in (0, 5, 40):
            for n in lens:
                iv = rng.integers(0, 256, iv_len, dtype=np.uint8).tobytes()
                aad = rng.integers(0, 256, aad_len, dtype=np.uint8).tobytes()
                pt = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
                ct, tag = c.encrypt(key, iv, pt, aad)
                rc, ect, etag = ora.cipher_encrypt(suite, key, iv, pt, aad)
                assert rc == 0 and ct == ect and tag == etag, (iv_len, aad_len, n)
                assert c.decrypt(key, iv, ct, aad, tag) == pt
                with pytest.raises(atls.TlsError) as e:
                    c.decrypt(key, iv, ct, aad, tag[:3] + bytes([tag[3] ^ 0x10]) + tag[4:])
                assert e.value.code == 20
