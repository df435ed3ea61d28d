"""Per-call latency of the Cipher-trait drop-in (atls_seal / atls_open through the ctypes mirror,
one record per call as net/record.rs:191-193 calls Cipher::encrypt), beside the oracle (the
reference's per-record CPU algorithm) for the same call, and the aggregate rate of 8 threads
calling concurrently. Prints one JSON object. Needs a GPU."""
import json
import os
import statistics
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import anothertls_amd as atls  # noqa: E402
import oracle as ora  # noqa: E402


def _median_us(fn, reps):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return round(statistics.median(ts) * 1e6, 1)


def main():
    out = {"what": "median microseconds per call, one record per call, host buffers"}
    key16, key32, iv = bytes(range(16)), bytes(range(32)), bytes(12)
    for suite, key, name in [(0x1301, key16, "aes128gcm"), (0x1303, key32, "chacha20poly1305")]:
        c = atls.CipherSuite(suite).get_cipher()
        for n in (1537, 16385):
            pt = os.urandom(n)
            ct, tag = c.encrypt(key, iv, pt, b"\x17\x03\x03\x40\x11")
            out[f"{name}_{n}_seal_us"] = _median_us(lambda: c.encrypt(key, iv, pt, b"\x17\x03\x03\x40\x11"), 200)
            out[f"{name}_{n}_open_us"] = _median_us(lambda: c.decrypt(key, iv, ct, b"\x17\x03\x03\x40\x11", tag), 200)
            out[f"{name}_{n}_oracle_seal_us"] = _median_us(
                lambda: ora.cipher_encrypt(suite, key, iv, pt, b"\x17\x03\x03\x40\x11"), 5 if n > 2000 else 20)
    # a fresh key on every call (the reference expands the key and computes H on every call, gcm.rs:49-56):
    # 256 keys in turn, more than a context's 16 cached slots, so every call installs its key first
    # (key-setup kernel, its key in the launch arguments) and then seals
    aad = b"\x17\x03\x03\x06\x11"
    for suite, klen, name in [(0x1301, 16, "aes128gcm"), (0x1302, 32, "aes256gcm"), (0x1303, 32, "chacha20poly1305")]:
        c = atls.CipherSuite(suite).get_cipher()
        keys = [os.urandom(klen) for _ in range(256)]
        pt = os.urandom(1537)
        it = {"i": 0}

        def call():
            it["i"] += 1
            c.encrypt(keys[it["i"] % 256], iv, pt, aad)

        out[f"{name}_1537_newkey_seal_us"] = _median_us(call, 400)
        out[f"{name}_1537_oracle_newkey_seal_us"] = _median_us(
            lambda: ora.cipher_encrypt(suite, keys[0], iv, pt, aad), 20)
        ct, tag = c.encrypt(keys[5], iv, pt, aad)
        assert ora.cipher_encrypt(suite, keys[5], iv, pt, aad)[1:] == (ct, tag)
    # 8 threads, each its own key, 16385-B AES-128-GCM seals
    calls, secs = 200, []
    pt = os.urandom(16385)

    def worker(t):
        k = bytes([t]) * 16
        g = atls.Gcm()
        g.encrypt(k, iv, pt)
        t0 = time.perf_counter()
        for _ in range(calls):
            g.encrypt(k, iv, pt)
        secs.append(time.perf_counter() - t0)

    th = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    t0 = time.perf_counter()
    for x in th:
        x.start()
    for x in th:
        x.join()
    wall = time.perf_counter() - t0
    out["threads8_aes128gcm_16385_calls_per_s"] = round(8 * calls / wall, 1)
    out["threads8_aes128gcm_16385_MBps"] = round(8 * calls * 16385 / wall / 1e6, 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
