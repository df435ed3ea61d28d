"""The oracle (literal restatement of the reference) against the reference's own KATs."""
import json
import os

import pytest

import oracle as ora

KATS = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_kats.json")))
H = bytes.fromhex


@pytest.mark.parametrize("v", KATS["aes_block"], ids=lambda v: v["name"])
def test_aes_block(v):
    rc, ct = ora.aes_encrypt_block(H(v["key"]), H(v["pt"]))
    assert rc == 0 and ct.hex() == v["ct"]
    rc, pt = ora.aes_decrypt_block(H(v["key"]), ct)  # cipher.rs:393-417 round trip
    assert rc == 0 and pt.hex() == v["pt"]


@pytest.mark.parametrize("v", KATS["gcm"], ids=lambda v: v["name"])
def test_gcm(v):
    rc, ct, tag = ora.gcm_encrypt(H(v["key"]), H(v["iv"]), H(v["pt"]), H(v["aad"]))
    assert rc == 0 and tag.hex() == v["tag"]
    if "ct" in v:
        assert ct.hex() == v["ct"]
    rc, pt = ora.gcm_decrypt(H(v["key"]), H(v["iv"]), ct, H(v["aad"]), tag)
    assert rc == 0 and pt.hex() == v["pt"]
    bad = bytes([tag[0] ^ 1]) + tag[1:]
    assert ora.gcm_decrypt(H(v["key"]), H(v["iv"]), ct, H(v["aad"]), bad)[0] == 20


@pytest.mark.parametrize("v", KATS["chacha20"], ids=lambda v: v["name"])
def test_chacha20(v):
    rc, ct = ora.chacha20_encrypt(H(v["key"]), H(v["iv"]), H(v["pt"]), v["counter"])
    assert rc == 0 and ct.hex() == v["ct"]
    assert ora.chacha20_encrypt(H(v["key"]), H(v["iv"]), ct, v["counter"])[1].hex() == v["pt"]


def test_poly1305_mac():
    for v in KATS["poly1305"]["mac"]:
        assert ora.poly1305_mac(H(v["key"]), H(v["msg"])).hex() == v["tag"]


def test_poly1305_key_gen():
    for v in KATS["poly1305"]["key_gen"]:
        rc, otk = ora.poly1305_key_gen(H(v["key"]), H(v["iv"]))
        assert rc == 0 and otk.hex() == v["otk"]


@pytest.mark.parametrize("v", KATS["poly1305"]["aead"], ids=lambda v: v["name"])
def test_chacha_poly_aead(v):
    rc, ct, tag = ora.chacha_poly_encrypt(H(v["key"]), H(v["iv"]), H(v["pt"]), H(v["aad"]))
    assert rc == 0 and ct.hex() == v["ct"] and tag.hex() == v["tag"]
    rc, pt = ora.chacha_poly_decrypt(H(v["key"]), H(v["iv"]), H(v["ct"]), H(v["aad"]), H(v["tag"]))
    assert rc == 0 and pt.hex() == v["pt"]


@pytest.mark.parametrize("v", KATS["sha"], ids=lambda v: v["hash"] + ":" + v["msg"][:8])
def test_sha(v):
    hl = ora.SHA384 if v["hash"] == "sha384" else ora.SHA256
    assert ora.sha(hl, H(v["msg"])).hex() == v["digest"]


@pytest.mark.parametrize("v", KATS["hmac"], ids=lambda v: v["hash"] + ":" + v["key"][:8])
def test_hmac(v):
    hl = ora.SHA384 if v["hash"] == "sha384" else ora.SHA256
    assert ora.hmac(hl, H(v["key"]), H(v["data"])).hex() == v["mac"]


@pytest.mark.parametrize("v", KATS["hkdf"], ids=lambda v: v["ikm"][:8] + ":" + v["salt"][:4])
def test_hkdf(v):
    prk = ora.hkdf_extract(ora.SHA256, H(v["salt"]), H(v["ikm"]))
    assert ora.hkdf_expand(ora.SHA256, prk, H(v["info"]), len(v["okm"]) // 2).hex() == v["okm"]
