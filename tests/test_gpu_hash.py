"""Row a15 on the device: SHA-256/384, HMAC, HKDF extract/expand and the TLS 1.3 secret chain,
through the C ABI (atls_hash_batch, atls_key_schedule) and the reference-named Python mirror
(anothertls_amd.hash). Pinned by the reference's own KATs (hash/sha256.rs:208-222,
sha384.rs:228-255, hmac.rs:99-143, hkdf.rs:82-121, extracted to tests/golden/reference_kats.json),
RFC 8448 §3's key-schedule values, Python hashlib / hmac as an independent implementation, and the
oracle (which also restates the reference's HMAC long-key quirk, hmac.rs:41-49)."""
import hashlib
import hmac as pyhmac
import json
import os
import random

import pytest

import oracle as ora
from anothertls_amd import hash as H

pytestmark = pytest.mark.gpu
KATS = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_kats.json")))
B = bytes.fromhex
HT = {"sha256": H.HashType.SHA256, "sha384": H.HashType.SHA384}


@pytest.mark.parametrize("v", KATS["sha"], ids=lambda v: v["src"])
def test_sha_kats(v):
    assert H.sha_x(HT[v["hash"]], B(v["msg"])).hex() == v["digest"]


@pytest.mark.parametrize("v", KATS["hmac"], ids=lambda v: v["src"])
def test_hmac_kats(v):
    assert H.Hmac(HT[v["hash"]], B(v["key"])).update(B(v["data"])).result().hex() == v["mac"]


@pytest.mark.parametrize("v", KATS["hkdf"], ids=lambda v: v["src"])
def test_hkdf_kats(v):
    h = HT[v["hash"]]
    prk = H.Hkdf.extract(h, B(v["salt"]), B(v["ikm"]))
    assert prk.expand(B(v["info"]), len(B(v["okm"]))).hex() == v["okm"]


def test_sha_batch_lengths_vs_hashlib():
    rng = random.Random(3)
    lens = [0, 1, 55, 56, 63, 64, 65, 111, 112, 119, 120, 127, 128, 129, 1000, 4097]
    msgs = [bytes(rng.getrandbits(8) for _ in range(n)) for n in lens]
    assert H.sha_batch(H.HashType.SHA256, msgs) == [hashlib.sha256(m).digest() for m in msgs]
    assert H.sha_batch(H.HashType.SHA384, msgs) == [hashlib.sha384(m).digest() for m in msgs]


def test_hmac_batch_vs_hashlib_and_long_key_quirk():
    rng = random.Random(4)
    for ht, name in [(H.HashType.SHA256, "sha256"), (H.HashType.SHA384, "sha384")]:
        keys = [bytes(rng.getrandbits(8) for _ in range(k)) for k in (0, 1, 32, 48, 64, 65, 100, 128, 129, 200)]
        msgs = [bytes(rng.getrandbits(8) for _ in range(rng.choice([0, 10, 200]))) for _ in keys]
        got = H.hmac_batch(ht, keys, msgs)
        for k, m, g in zip(keys, msgs, got):
            assert g == ora.hmac(int(ht), k, m)  # the reference's HMAC, quirk included
            # RFC 2104 agrees except SHA-384 keys of 65..128 bytes, which the reference hashes first
            std = pyhmac.new(k, m, name).digest()
            assert (g == std) == (not (ht == H.HashType.SHA384 and 64 < len(k) <= 128)), (name, len(k))


def test_hkdf_expand_lengths_and_limit():
    rng = random.Random(5)
    for ht in H.HashType:
        prk = bytes(rng.getrandbits(8) for _ in range(int(ht)))
        info = b"ctx" * 7
        for L in (1, int(ht), int(ht) + 1, 100, 255 * int(ht)):
            assert H.Hkdf.from_prk(ht, prk).expand(info, L) == ora.hkdf_expand(int(ht), prk, info, L)
        assert H.Hkdf.from_prk(ht, prk).expand(info, 255 * int(ht) + 1) is None


RFC8448 = dict(  # RFC 8448 §3 (simple 1-RTT handshake), TLS_AES_128_GCM_SHA256
    shared="8bd4054fb55b9d63fdfbacf9f04b9f0d35e6d63f537563efd46272900f89492d",
    hello="860c06edc07858ee8e78f0e7428c58edd6b43f2ca3e6e95f02ed063cf0e1cad8",
    c_hs="b3eddb126e067f35a780b3abf45e2d8f3b1a950738f52e9600746a0e27a55a21",
    s_hs="b67b7d690cc16c4e75e54213cb2d37b4e9c912bcded9105d42befd59d391ad38",
    master="18df06843d13a08bf2a449844c5f8a478001bc4d4c627984d5a41da8d0402919")


def test_key_schedule_rfc8448_and_traffic_keys():
    ks = H.KeySchedule.do_key_schedule(H.HashType.SHA256, B(RFC8448["hello"]), B(RFC8448["shared"]))
    assert ks.client_handshake_traffic_secret.pseudo_random_key.hex() == RFC8448["c_hs"]
    assert ks.server_handshake_traffic_secret.pseudo_random_key.hex() == RFC8448["s_hs"]
    assert ks.hkdf_master_secret.pseudo_random_key.hex() == RFC8448["master"]
    k = H.Key.from_hkdf(ks.server_handshake_traffic_secret, 16, 12)  # RFC 8448 server handshake key / iv
    assert k.key.hex() == "3fce516009c21727d0f2e4e86ee403bc" and k.iv.hex() == "5d313eb2671276ee13000b30"


def test_key_schedule_batch_vs_oracle():
    rng = random.Random(6)
    for ht in H.HashType:
        hl = int(ht)
        n = 64
        shared = [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(n)]
        hello = [bytes(rng.getrandbits(8) for _ in range(hl)) for _ in range(n)]
        fin = [bytes(rng.getrandbits(8) for _ in range(hl)) for _ in range(n)]
        got = H.key_schedule_batch(ht, shared, hello, fin)
        for i in range(n):
            assert got[i] == ora.key_schedule(hl, shared[i], hello[i], fin[i]), (hl, i)
        # the application secrets through the mirror's expand path agree with the chain's
        c, s = H.application_secrets(H.Hkdf.from_prk(ht, got[0][2]), fin[0])
        assert (c.pseudo_random_key, s.pseudo_random_key) == got[0][3:5]


def test_hash_batch_spans_near_uint64_max_are_refused():
    """A message or key span whose offset is close to 2^64 (off + len wraps) is refused with
    ILLEGAL_PARAMETER before anything reaches the device (the bounds check no longer
    wraps)."""
    import hashlib

    import numpy as np

    import anothertls_amd as atls
    from anothertls_amd import hash as H

    lib = atls.library()
    data = np.zeros(64, np.uint8)
    out = np.zeros(64, np.uint8)
    span = np.dtype([("off", "<u8"), ("len", "<u4"), ("reserved", "<u4")])
    good = np.array([(0, 16, 0)], span)
    for off, ln in [(2**64 - 8, 16), (2**64 - 1, 1), (65, 0), (60, 5)]:
        bad = np.array([(off, ln, 0)], span)
        for op, keys in [(0, None), (1, good)]:  # SHA (no keys), HMAC with a bad message span
            rc = lib.atls_hash_batch(H._engine()._e, op, 32, data.ctypes.data, len(data),
                                     None if keys is None else keys.ctypes.data, bad.ctypes.data, 1, 32,
                                     out.ctypes.data)
            assert rc == 47, (off, ln, op, rc)
        rc = lib.atls_hash_batch(H._engine()._e, 1, 32, data.ctypes.data, len(data), bad.ctypes.data,
                                 good.ctypes.data, 1, 32, out.ctypes.data)  # bad key span
        assert rc == 47, (off, ln, rc)
    ok = lib.atls_hash_batch(H._engine()._e, 0, 32, data.ctypes.data, len(data), None, good.ctypes.data, 1, 32,
                             out.ctypes.data)
    assert ok == 0 and bytes(out[:32]) == hashlib.sha256(bytes(16)).digest()
