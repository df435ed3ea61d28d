"""Run by tests/test_gpu_single_resident.py in its own process (the mode is read once per process):
Cipher-trait single calls with the resident server on (ATLS_SINGLE_RESIDENT=1: ChaCha20-Poly1305 calls through
it; =2: AES-GCM calls too, gcm.hip single_resident<true>) against the oracle: ChaCha20-Poly1305 at lengths across the F4 quirk
(chacha20/cipher.rs:99-102) and the argument-block limit; AES-128/-192/-256-GCM (gcm.rs:42-162) with 12-byte
and other IVs; AADs of 0-40 bytes; seal / open / tampered tag; suites interleaved; batch launches between
calls (the server steps aside and comes back, building its AES tables again); calls after the server left on
its idle timeout; and 8 threads at once."""
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
    print("resident OK")


if __name__ == "__main__":
    main()
