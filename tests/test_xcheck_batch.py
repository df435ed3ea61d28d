"""CPU: the OpenSSL batch cross-check (tests/native/openssl_batch.c) agrees with the oracle on
TLS-mode batches of every suite, and flags exactly the ChaCha20 last-block-quirk records
(AEAD length % 64 == 0, chacha20/cipher.rs:99-102) as unchecked. The GPU config tests
(test_gpu_configs.py) rely on it for whole-batch comparisons."""
import numpy as np

import openssl_ref
import oracle as ora
from anothertls_amd import workload


def test_openssl_batch_matches_oracle():
    lens = np.array([0, 1, 15, 16, 17, 62, 63, 64, 126, 127, 1535, 1536, 4095, 16383, 16384] * 4, np.uint64)
    n = len(lens)

    def suites(k):
        return np.array([0x1301, 0x1302, 0x1303] * k, np.uint16)[:k]

    b = workload.tls_batch(n, lens, suites, n_keys=7)
    b["recs"]["seq"] += np.uint64(2**40 - 3)
    inbuf = np.random.default_rng(5).integers(0, 256, b["in_bytes"] + 16, dtype=np.uint8)
    out, tags, skipped = openssl_ref.seal_tls_batch(b["keys"], b["recs"], inbuf, b["out_bytes"], 4)
    okeys = (ora.OraKey * len(b["keys"])).from_buffer_copy(b["keys"].tobytes())
    orecs = (ora.OraRec * n).from_buffer_copy(b["recs"].tobytes())
    oout, otags = np.zeros_like(out), np.zeros_like(tags)
    assert ora.seal_batch(okeys, orecs, inbuf, np.zeros(16, np.uint8), oout, otags, 4) == 0
    chacha = b["keys"]["suite"][b["recs"]["key_slot"]] == 0x1303
    quirk = chacha & ((lens + 1) % 64 == 0)
    assert np.array_equal(skipped.astype(bool), quirk) and quirk.sum() > 0
    for i in range(n):
        r = b["recs"][i]
        o, L = int(r["out_off"]), int(r["len"]) + 1
        same = out[o:o + L].tobytes() == oout[o:o + L].tobytes() and tags[16 * i:16 * i + 16].tobytes() == \
            otags[16 * i:16 * i + 16].tobytes()
        assert same != bool(quirk[i]), (i, int(lens[i]), bool(quirk[i]))
