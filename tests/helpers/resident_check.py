"""Run by tests/test_gpu_single_resident.py in its own process (the mode is read once per process):
ChaCha20-Poly1305 single calls through the resident server (ATLS_SINGLE_RESIDENT=1) against the oracle --
lengths across the F4 quirk (chacha20/cipher.rs:99-102) and the argument-block limit, AADs of 0-40 bytes,
seal / open / tampered tag, calls after the server left on its idle timeout, and 8 threads at once."""
import os
import random
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import anothertls_amd as atls  # noqa: E402
import oracle as ora  # noqa: E402


def one(c, rng, key, n, aad_len):
    iv = bytes(rng.getrandbits(8) for _ in range(12))
    aad = bytes(rng.getrandbits(8) for _ in range(aad_len))
    pt = bytes(rng.getrandbits(8) for _ in range(n))
    ct, tag = c.encrypt(key, iv, pt, aad)
    rc, ect, etag = ora.cipher_encrypt(0x1303, key, iv, pt, aad)
    assert rc == 0 and ct == ect and tag == etag, (n, aad_len)
    assert c.decrypt(key, iv, ct, aad, tag) == pt
    try:
        c.decrypt(key, iv, ct, aad, tag[:7] + bytes([tag[7] ^ 2]) + tag[8:])
    except atls.TlsError as e:
        assert e.code == 20
    else:
        raise AssertionError("tampered tag accepted")


def main():
    assert os.environ.get("ATLS_SINGLE_RESIDENT") == "1"
    rng = random.Random(0x5E5)
    c = atls.CipherSuite(0x1303).get_cipher()
    keys = [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(3)]
    print("first call", flush=True)
    one(c, rng, keys[0], 1537, 5)
    print("first call OK", flush=True)
    for aad_len in (0, 5, 40):
        for n in (0, 1, 15, 16, 63, 64, 65, 127, 128, 1023, 1024, 1536, 1537, 3000, 3455, 3456, 3500, 3600, 16385):
            one(c, rng, keys[n % 3], n, aad_len)
        print("aad", aad_len, "OK", flush=True)
    for _ in range(3):  # the server leaves after ATLS_SINGLE_RESIDENT_IDLE_MS without a call; the next call relaunches it
        time.sleep(0.05)
        one(c, rng, keys[0], 1537, 5)
    errors = []

    def worker(t):
        r = random.Random(t)
        try:
            for i in range(60):
                one(c, r, keys[(t + i) % 3], r.choice([0, 1, 64, 700, 1537, 2048, 3000]), r.choice([0, 5, 13]))
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
