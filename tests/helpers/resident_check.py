"""Run by tests/test_gpu_single_resident.py in its own process (the mode is read once per process):
Cipher-trait single calls with the resident server on (ATLS_SINGLE_RESIDENT=1: ChaCha20-Poly1305 calls through
it; =2: AES-GCM calls too, gcm.hip single_resident<true>) against the oracle: ChaCha20-Poly1305 at lengths across the F4 quirk
(chacha20/cipher.rs:99-102) and the argument-block limit; AES-128/-192/-256-GCM (gcm.rs:42-162) with 12-byte
and other IVs; AADs of 0-40 bytes; seal / open / tampered tag; suites interleaved; batch launches between
calls (the server steps aside and comes back, building its AES tables again); calls after the server left on
its idle timeout; 8 threads at once; and 8 threads of calls without a pause beside a thread sealing batches,
each batch within a bound."""
import os
import random
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import anothertls_amd as atls  # noqa: E402
import oracle as ora  # noqa: E402

CHACHA, AES128, AES256 = 0x1303, 0x1301, 0x1302


def one(ciphers, rng, suite, key, n, aad_len, iv_len=12):
    c = ciphers[suite]
    iv = bytes(rng.getrandbits(8) for _ in range(iv_len))
    aad = bytes(rng.getrandbits(8) for _ in range(aad_len))
    pt = bytes(rng.getrandbits(8) for _ in range(n))
    ct, tag = c.encrypt(key, iv, pt, aad)
    rc, ect, etag = ora.cipher_encrypt(suite, key, iv, pt, aad)
    assert rc == 0 and ct == ect and tag == etag, (hex(suite), len(key), n, aad_len, iv_len)
    assert c.decrypt(key, iv, ct, aad, tag) == pt, (hex(suite), n)
    try:
        c.decrypt(key, iv, ct, aad, tag[:7] + bytes([tag[7] ^ 2]) + tag[8:])
    except atls.TlsError as e:
        assert e.code == 20
    else:
        raise AssertionError("tampered tag accepted")


def batch_launch():
    """A batch on an engine of this process: the server must step aside (its hardware queue) and return."""
    from anothertls_amd import workload
    eng = atls.Engine(0)
    b = workload.tls_batch(16, 1024, 0x1301, n_keys=4)
    eng.set_keys(b["keys"])
    h_in = np.random.default_rng(1).integers(0, 256, b["in_bytes"] + 16, dtype=np.uint8)
    out, tags = np.zeros(b["out_bytes"] + 16, np.uint8), np.zeros(16 * 16, np.uint8)
    eng.seal_batch(b["recs"], h_in, np.zeros(16, np.uint8), out, tags)
    eng.close()


def main():
    assert os.environ.get("ATLS_SINGLE_RESIDENT") in ("1", "2")  # 2: AES-GCM calls through the server too
    rng = random.Random(0x5E5)
    ciphers = {s: atls.CipherSuite(s).get_cipher() for s in (CHACHA, AES128, AES256)}
    keys = {CHACHA: [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(3)],
            AES128: [bytes(rng.getrandbits(8) for _ in range(16)) for _ in range(3)],
            AES256: [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(3)]}
    print("first calls", flush=True)
    one(ciphers, rng, CHACHA, keys[CHACHA][0], 1537, 5)
    one(ciphers, rng, AES128, keys[AES128][0], 1537, 5)
    print("first calls OK", flush=True)
    lens = (0, 1, 15, 16, 17, 63, 64, 65, 127, 128, 1023, 1024, 1536, 1537, 3000, 3455, 3456, 3500, 3600, 16385)
    for aad_len in (0, 5, 40):
        for n in lens:
            one(ciphers, rng, CHACHA, keys[CHACHA][n % 3], n, aad_len)
            one(ciphers, rng, AES128, keys[AES128][n % 3], n, aad_len)
            one(ciphers, rng, AES256, keys[AES256][n % 3], n, aad_len)
        print("aad", aad_len, "OK", flush=True)
    for iv_len in (1, 8, 16, 60):  # GCM's J0 from GHASH(IV) (gcm.rs:59-70)
        for n in (0, 16, 1537):
            one(ciphers, rng, AES128, keys[AES128][1], n, 13, iv_len)
            one(ciphers, rng, AES256, keys[AES256][2], n, 0, iv_len)
    # AES-192 keys through the AES-128 suite's cipher (the key length picks the rounds, gcm.rs:49)
    k192 = bytes(rng.getrandbits(8) for _ in range(24))
    for n in (0, 100, 1537):
        one(ciphers, rng, AES128, k192, n, 5)
    print("ivs and key sizes OK", flush=True)
    for _ in range(2):  # a batch launch in between: the server stops for it, the next call starts a new one
        batch_launch()
        one(ciphers, rng, AES256, keys[AES256][0], 1537, 5)
        one(ciphers, rng, CHACHA, keys[CHACHA][0], 1537, 5)
    for _ in range(3):  # the server leaves after ATLS_SINGLE_RESIDENT_IDLE_MS without a call; the next call relaunches it
        time.sleep(0.05)
        one(ciphers, rng, AES128, keys[AES128][0], 1537, 5)
        one(ciphers, rng, CHACHA, keys[CHACHA][0], 1537, 5)
    print("relaunches OK", flush=True)
    errors = []

    def worker(t):
        r = random.Random(t)
        try:
            for i in range(40):
                s = (CHACHA, AES128, AES256)[(t + i) % 3]
                one(ciphers, r, s, keys[s][(t + i) % 3], r.choice([0, 1, 64, 700, 1537, 2048, 3000]), r.choice([0, 5, 13]))
        except BaseException as ex:  # noqa: BLE001
            errors.append(ex)

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    for th in ths:
        th.start()
    for th in ths:
        th.join(120)
    assert not errors, errors[:2]
    print("8 threads OK", flush=True)
    batches_beside_calls(ciphers, keys)
    print("resident OK")


def batches_beside_calls(ciphers, keys, n_batches=40, bound_s=1.0):
    """8 threads of single calls through the server without a pause while another thread seals
    batches on its own engine. Every batch must finish within bound_s (a batch enqueued behind a server kept
    alive by the calls would wait until they stop), equal the first batch byte for byte, which equals the oracle
    (crypto/aes/gcm.rs:42-162 via net/record.rs:162-198); every call is checked against the oracle by one()."""
    import ctypes

    from anothertls_amd import workload
    eng = atls.Engine(0)
    b = workload.tls_batch(256, 16384, AES128, n_keys=8)
    recs = b["recs"]
    eng.set_keys(b["keys"])
    h_in = np.random.default_rng(7).integers(0, 256, b["in_bytes"] + 16, dtype=np.uint8)
    aux = np.zeros(16, np.uint8)
    ref_out, ref_tags = np.zeros(b["out_bytes"] + 16, np.uint8), np.zeros(16 * len(recs), np.uint8)
    eng.seal_batch(recs, h_in, aux, ref_out, ref_tags)
    o_out, o_tags = np.zeros_like(ref_out), np.zeros_like(ref_tags)
    okeys = (ora.OraKey * len(b["keys"])).from_buffer_copy(b["keys"].tobytes())
    orecs = (ora.OraRec * len(recs)).from_buffer_copy(recs.tobytes())
    ora.seal_batch(okeys, orecs, h_in, aux, o_out, o_tags, 8)
    assert np.array_equal(ref_out, o_out) and np.array_equal(ref_tags, o_tags), "batch != oracle"
    lib = atls.library()
    lib.atls_debug_resident_fallbacks.restype = ctypes.c_ulonglong
    fb0 = lib.atls_debug_resident_fallbacks()
    stop, errors, calls, times = threading.Event(), [], [0] * 8, []

    def caller(t):
        r = random.Random(100 + t)
        t_end = time.monotonic() + 60.0
        try:
            while not stop.is_set() and time.monotonic() < t_end:
                s = (CHACHA, AES128, AES256)[(t + calls[t]) % 3]
                one(ciphers, r, s, keys[s][calls[t] % 3], r.choice([0, 17, 700, 1537, 3000]), r.choice([0, 5]))
                calls[t] += 1
        except BaseException as ex:  # noqa: BLE001
            errors.append(ex)

    def batcher():
        try:
            out, tags = np.zeros_like(ref_out), np.zeros_like(ref_tags)
            time.sleep(0.2)  # the callers are running
            for _ in range(n_batches):
                out[:] = 0
                t0 = time.perf_counter()
                eng.seal_batch(recs, h_in, aux, out, tags)
                times.append(time.perf_counter() - t0)
                assert np.array_equal(out, ref_out) and np.array_equal(tags, ref_tags), "batch beside calls differs"
        except BaseException as ex:  # noqa: BLE001
            errors.append(ex)
        finally:
            stop.set()

    ths = [threading.Thread(target=caller, args=(t,)) for t in range(8)] + [threading.Thread(target=batcher)]
    for th in ths:
        th.start()
    for th in ths:
        th.join(120)
    eng.close()
    assert not errors, errors[:2]
    assert len(times) == n_batches, times
    fb = lib.atls_debug_resident_fallbacks() - fb0
    print(f"batches beside calls: {n_batches} batches, max {max(times) * 1e3:.1f} ms, median "
          f"{sorted(times)[len(times) // 2] * 1e3:.1f} ms; {sum(calls)} calls, {fb} of them launched while a batch "
          f"held the server", flush=True)
    assert max(times) < bound_s, times
    assert sum(calls) > 8 * 10, calls


if __name__ == "__main__":
    main()
