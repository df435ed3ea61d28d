"""Oracle cross-checks beyond the reference's KATs: OpenSSL (GCM, ChaCha20-Poly1305 where
standard), Python hashlib/hmac (SHA-2, HMAC), RFC 8448 traffic keys, and the documented
quirks pinned explicitly."""
import hashlib
import hmac as pyhmac
import random

import pytest

import openssl_ref
import oracle as ora

H = bytes.fromhex
pytestmark = pytest.mark.skipif(not openssl_ref.available(), reason="libcrypto not found")


def rnd(rng, n):
    return bytes(rng.getrandbits(8) for _ in range(n))


@pytest.mark.parametrize("key_len", [16, 24, 32])
def test_gcm_vs_openssl(key_len):
    rng = random.Random(key_len)
    for n in [0, 1, 15, 16, 17, 63, 64, 100, 255, 1537]:
        for iv_len in [12, 8, 16, 60, 1]:
            key, iv, pt, aad = rnd(rng, key_len), rnd(rng, iv_len), rnd(rng, n), rnd(rng, rng.choice([0, 5, 13, 40]))
            rc, ct, tag = ora.gcm_encrypt(key, iv, pt, aad)
            ect, etag = openssl_ref.seal("gcm", key, iv, pt, aad)
            assert rc == 0 and ct == ect and tag == etag, (n, iv_len)


def test_chacha_poly_vs_openssl_and_f4_quirk():
    rng = random.Random(7)
    key, iv = rnd(rng, 32), rnd(rng, 12)
    for n in [0, 1, 63, 64, 65, 114, 127, 128, 1536, 1537, 16384, 16385]:
        pt, aad = rnd(rng, n), rnd(rng, 5)
        rc, ct, tag = ora.chacha_poly_encrypt(key, iv, pt, aad)
        ect, etag = openssl_ref.seal("chacha", key, iv, pt, aad)
        assert rc == 0
        if n % 64 != 0 or n == 0:
            assert (ct, tag) == (ect, etag), n
        else:
            # F4 (chacha20/cipher.rs:99-102): the last 64 bytes are left unencrypted.
            assert ct[:-64] == ect[:-64] and ct[-64:] == pt[-64:] and tag != etag, n
        rc2, back = ora.chacha_poly_decrypt(key, iv, ct, aad, tag)
        assert rc2 == 0 and back == pt


def test_sha_vs_hashlib():
    rng = random.Random(3)
    for n in list(range(0, 140)) + [255, 256, 1000]:
        m = rnd(rng, n)
        assert ora.sha(ora.SHA256, m) == hashlib.sha256(m).digest()
        assert ora.sha(ora.SHA384, m) == hashlib.sha384(m).digest()


def test_hmac_vs_stdlib_and_sha384_long_key_quirk():
    rng = random.Random(4)
    for kl in [0, 1, 32, 48, 64, 65, 100, 128, 129, 200]:
        key, msg = rnd(rng, kl), rnd(rng, 77)
        assert ora.hmac(ora.SHA256, key, msg) == pyhmac.new(key, msg, hashlib.sha256).digest()
        got = ora.hmac(ora.SHA384, key, msg)
        want = pyhmac.new(key, msg, hashlib.sha384).digest()
        if 64 < kl <= 128:
            # quirk 8 (hash/hmac.rs:41-49): keys of 65..128 bytes are hashed first for SHA-384
            assert got == pyhmac.new(hashlib.sha384(key).digest(), msg, hashlib.sha384).digest() and got != want
        else:
            assert got == want


def test_rfc8448_server_handshake_traffic_keys():
    # RFC 8448 §3 "Simple 1-RTT Handshake": server_handshake_traffic_secret -> write key/iv
    secret = H("b67b7d690cc16c4e75e54213cb2d37b4e9c912bcded9105d42befd59d391ad38")
    rc, key, iv = ora.key_from_secret(ora.SHA256, secret, 16, 12)
    assert rc == 0
    assert key.hex() == "3fce516009c21727d0f2e4e86ee403bc"
    assert iv.hex() == "5d313eb2671276ee13000b30"


def test_hkdf_expand_limit():
    assert ora.hkdf_expand(ora.SHA256, b"k" * 32, b"", 255 * 32) is not None
    assert ora.hkdf_expand(ora.SHA256, b"k" * 32, b"", 255 * 32 + 1) is None


def test_per_record_nonce():
    iv = bytes(range(12))
    assert ora.per_record_nonce(iv, 0) == iv
    n = ora.per_record_nonce(iv, 0x0102030405060708)
    assert n[:4] == iv[:4] and bytes(a ^ b for a, b in zip(n[4:], iv[4:])) == H("0102030405060708")


@pytest.mark.parametrize("suite,klen", [(0x1301, 16), (0x1302, 32), (0x1303, 32)])
def test_record_roundtrip_and_framing(suite, klen):
    rng = random.Random(suite)
    key, iv = rnd(rng, klen), rnd(rng, 12)
    for seq, L in [(0, 0), (1, 12), (2, 62), (3, 63), (4, 16384), (77, 1536)]:
        frag = rnd(rng, L)
        rc, wire = ora.record_seal(suite, key, iv, seq, 23, frag)
        assert rc == 0 and len(wire) == 5 + L + 1 + 16
        assert wire[:3] == b"\x17\x03\x03" and int.from_bytes(wire[3:5], "big") == (L + 17) & 0xFFFF
        # independent: OpenSSL over inner plaintext with header AAD (not for F4 lengths)
        nonce = ora.per_record_nonce(iv, seq)
        kind = "chacha" if suite == 0x1303 else "gcm"
        if kind == "gcm" or (L + 1) % 64:
            ect, etag = openssl_ref.seal(kind, key, nonce, frag + b"\x17", wire[:5])
            assert wire[5:] == ect + etag
        rc, content, ctype = ora.record_open(suite, key, iv, seq, wire)
        assert rc == 0 and content == frag and ctype == 23
        bad = bytearray(wire)
        bad[-1] ^= 1
        assert ora.record_open(suite, key, iv, seq, bytes(bad))[0] == 50  # DecryptError (record.rs:222)
        assert ora.record_open(suite, key, iv, seq + 1, wire)[0] == 50


def test_record_open_padding_scan_and_invalid():
    key, iv = b"\x11" * 16, b"\x22" * 12
    # inner plaintext all zero -> RecordType::Invalid with empty body (record.rs:229-239)
    rc, wire = ora.record_seal(0x1301, key, iv, 5, 0, b"\0" * 10)
    rc, content, ctype = ora.record_open(0x1301, key, iv, 5, wire)
    assert rc == 0 and content == b"" and ctype == 0
    # zero padding after the type byte is stripped
    rc, wire = ora.record_seal(0x1301, key, iv, 6, 0, b"hello" + b"\x16" + b"\0" * 7)
    rc, content, ctype = ora.record_open(0x1301, key, iv, 6, wire)
    assert rc == 0 and content == b"hello" and ctype == 22
    # a non-zero byte that is not a RecordType -> DecodeError
    rc, wire = ora.record_seal(0x1301, key, iv, 7, 0x99, b"abc")
    assert ora.record_open(0x1301, key, iv, 7, wire)[0] == 51
    # short fragment / truncated buffer -> DecodeError (reference panics; documented divergence)
    assert ora.record_open(0x1301, key, iv, 7, b"\x17\x03\x03\x00\x05abcde")[0] == 51
    assert ora.record_open(0x1301, key, iv, 7, b"\x17\x03")[0] == 51


def test_suite_and_parameter_errors():
    assert ora.cipher_encrypt(0x00FF, b"k" * 16, b"i" * 12, b"x")[0] == 71
    assert ora.cipher_encrypt(0x1301, b"k" * 15, b"i" * 12, b"x")[0] == 47
    assert ora.cipher_encrypt(0x1303, b"k" * 16, b"i" * 12, b"x")[0] == 47
    assert ora.cipher_encrypt(0x1303, b"k" * 32, b"i" * 8, b"x")[0] == 47
    # 0x1301 with a 32-byte key still runs AES-256 (gcm.rs:49 sizes AES from key.len())
    rc, ct, tag = ora.cipher_encrypt(0x1301, b"k" * 32, b"i" * 12, b"x" * 20)
    assert rc == 0 and (ct, tag) == openssl_ref.seal("gcm", b"k" * 32, b"i" * 12, b"x" * 20)
    # wrong-length tag is a mismatch
    assert ora.cipher_decrypt(0x1301, b"k" * 16, b"i" * 12, b"", b"", b"\0" * 15)[0] == 20
