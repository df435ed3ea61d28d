"""GPU parity: the HIP path (through the C ABI) against the oracle, the reference's KATs and
OpenSSL, on seeded inputs. Bit-exact for every byte and tag."""
import json
import os
import random

import numpy as np
import pytest

import anothertls_amd as atls
import openssl_ref
import oracle as ora
from anothertls_amd import workload

pytestmark = pytest.mark.gpu
KATS = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_kats.json")))
H = bytes.fromhex
NTHREADS = min(16, os.cpu_count() or 1)


@pytest.fixture(scope="module")
def eng():
    e = atls.Engine(int(os.environ.get("ATLS_DEVICE", "0")))
    yield e
    e.close()


def oracle_keys(keys):
    arr = (ora.OraKey * len(keys))()
    for i, k in enumerate(keys):
        arr[i].suite = int(k["suite"])
        arr[i].key_len = int(k["key_len"])
        arr[i].iv_len = int(k["iv_len"])
        for j in range(32):
            arr[i].key[j] = int(k["key"][j])
        for j in range(12):
            arr[i].static_iv[j] = int(k["static_iv"][j])
    return arr


def oracle_recs(recs):
    arr = (ora.OraRec * len(recs)).from_buffer_copy(recs.tobytes())
    return arr


# ---------------------------------------------------------------- Cipher-trait drop-in ----
@pytest.mark.parametrize("v", KATS["gcm"], ids=lambda v: v["name"])
def test_gcm_kats(v):
    c = atls.Gcm()
    ct, tag = c.encrypt(H(v["key"]), H(v["iv"]), H(v["pt"]), H(v["aad"]))
    assert tag.hex() == v["tag"]
    assert c.decrypt(H(v["key"]), H(v["iv"]), ct, H(v["aad"]), tag).hex() == v["pt"]


@pytest.mark.parametrize("v", KATS["poly1305"]["aead"], ids=lambda v: v["name"])
def test_chacha_poly_kats(v):
    c = atls.Poly1305()
    ct, tag = c.encrypt(H(v["key"]), H(v["iv"]), H(v["pt"]), H(v["aad"]))
    assert ct.hex() == v["ct"] and tag.hex() == v["tag"]
    assert c.decrypt(H(v["key"]), H(v["iv"]), H(v["ct"]), H(v["aad"]), H(v["tag"])).hex() == v["pt"]


SINGLE_LENS = [0, 1, 5, 15, 16, 17, 31, 32, 33, 63, 64, 65, 100, 127, 128, 129, 255, 256, 1023, 1024, 1025,
               1536, 1537, 4095, 4096, 4097, 16384, 16385]


@pytest.mark.parametrize("suite,klen", [(0x1301, 16), (0x1301, 24), (0x1302, 32), (0x1303, 32)])
def test_single_calls_vs_oracle(suite, klen):
    rng = random.Random(suite * 100 + klen)
    c = atls.CipherSuite(suite).get_cipher()
    for n in SINGLE_LENS:
        key = bytes(rng.getrandbits(8) for _ in range(klen))
        ivl = 12 if suite == 0x1303 else rng.choice([12, 12, 1, 8, 16, 60])
        iv = bytes(rng.getrandbits(8) for _ in range(ivl))
        aad = bytes(rng.getrandbits(8) for _ in range(rng.choice([0, 5, 13, 16, 40])))
        pt = bytes(rng.getrandbits(8) for _ in range(n))
        ct, tag = c.encrypt(key, iv, pt, aad)
        rc, ect, etag = ora.cipher_encrypt(suite, key, iv, pt, aad)
        assert rc == 0 and ct == ect and tag == etag, (n, ivl, len(aad))
        assert c.decrypt(key, iv, ct, aad, tag) == pt
        with pytest.raises(atls.TlsError) as e:
            c.decrypt(key, iv, ct, aad, bytes([tag[0] ^ 0x80]) + tag[1:])
        assert e.value.code == 20


# ---------------------------------------------------------------------------- batches ----
def fill_payload(batch, seed):
    rng = np.random.default_rng(seed)
    inbuf = rng.integers(0, 256, size=max(batch["in_bytes"], 16), dtype=np.uint8)
    return inbuf


def seal_both(eng, batch, inbuf, aux=None, nthreads=NTHREADS):
    keys, recs = batch["keys"], batch["recs"]
    aux = np.zeros(16, np.uint8) if aux is None else aux
    eng.set_keys(keys)
    out = np.zeros(max(batch["out_bytes"], 16), np.uint8)
    tags = np.zeros(16 * len(recs), np.uint8)
    eng.seal_batch(recs, inbuf, aux, out, tags)
    oout = np.zeros_like(out)
    otags = np.zeros_like(tags)
    assert ora.seal_batch(oracle_keys(keys), oracle_recs(recs), inbuf, aux, oout, otags, nthreads) == 0
    return out, tags, oout, otags


def assert_same(out, tags, oout, otags, recs):
    bad = [i for i in range(len(recs)) if tags[16 * i:16 * i + 16].tobytes() != otags[16 * i:16 * i + 16].tobytes()]
    assert not bad, f"{len(bad)} tag mismatches, first records {bad[:5]}"
    assert np.array_equal(out, oout)


EDGE_LENS = [0, 1, 2, 14, 15, 16, 17, 31, 47, 62, 63, 64, 65, 126, 127, 128, 1023, 1535, 1536, 1537, 2047,
             4095, 16383, 16384]


def mixed_suites(k):
    r = np.random.default_rng(11)
    return r.choice(np.array([0x1301, 0x1302, 0x1303], dtype=np.uint16), size=k)


def test_batch_tls_mixed_seal_open(eng):
    rng = np.random.default_rng(5)
    lens = np.array(EDGE_LENS * 6 + list(rng.integers(0, 20000, size=300)), dtype=np.uint64)
    batch = workload.tls_batch(len(lens), lens, mixed_suites, n_keys=37, content_type=23, seq_base=2**40 - 3)
    # one AES-192 connection (0x1301 with a 24-byte key: gcm.rs:49)
    batch["keys"][3]["suite"], batch["keys"][3]["key_len"] = 0x1301, 24
    inbuf = fill_payload(batch, 1)
    out, tags, oout, otags = seal_both(eng, batch, inbuf)
    assert_same(out, tags, oout, otags, batch["recs"])

    # open the sealed records (ciphertext = content||type) and check framing results
    recs = batch["recs"]
    orecs = recs.copy()
    orecs["in_off"] = recs["out_off"]
    orecs["len"] = recs["len"] + 1
    pt = np.zeros_like(out)
    res = np.zeros(len(recs), atls.OPEN_RESULT_DTYPE)
    tags_t = tags.copy()
    tampered = rng.choice(len(recs), size=20, replace=False)
    for i in tampered:
        tags_t[16 * i + 7] ^= 1
    eng.open_batch(orecs, out, np.zeros(16, np.uint8), tags_t, pt, res)
    for i in range(len(recs)):
        L, o, io = int(recs[i]["len"]), int(recs[i]["out_off"]), int(recs[i]["in_off"])
        if i in tampered:
            assert res[i]["status"] == 50, i  # DecryptError (record.rs:222)
            continue
        assert res[i]["status"] == 0, (i, res[i])
        assert res[i]["content_type"] == 23 and res[i]["content_len"] == L, (i, res[i])
        assert pt[o:o + L].tobytes() == inbuf[io:io + L].tobytes() and pt[o + L] == 23


def test_batch_padding_scan_and_bad_types(eng):
    # content types, zero padding inside the content, all-zero records (record.rs:229-239)
    contents = [b"", b"\0" * 40, b"hello\x16" + b"\0" * 9, b"x" * 63, b"abc\x99", b"\0" * 16384]
    types = [23, 0, 0, 22, 0, 21]
    n = len(contents)
    for suite in (0x1301, 0x1303):
        batch = workload.tls_batch(n, [len(c) for c in contents], suite, n_keys=2)
        inbuf = np.zeros(max(batch["in_bytes"], 16), np.uint8)
        for i, c in enumerate(contents):
            io = int(batch["recs"][i]["in_off"])
            inbuf[io:io + len(c)] = np.frombuffer(c, np.uint8)
        batch["recs"]["content_type"] = types
        out, tags, oout, otags = seal_both(eng, batch, inbuf)
        assert_same(out, tags, oout, otags, batch["recs"])
        recs = batch["recs"].copy()
        recs["in_off"] = batch["recs"]["out_off"]
        recs["len"] = batch["recs"]["len"] + 1
        pt = np.zeros_like(out)
        res = np.zeros(n, atls.OPEN_RESULT_DTYPE)
        eng.open_batch(recs, out, np.zeros(16, np.uint8), tags, pt, res)
        ores = (ora.OraOpenResult * n)()
        opt = np.zeros_like(out)
        ora.open_batch(oracle_keys(batch["keys"]), oracle_recs(recs), out, np.zeros(16, np.uint8), tags, opt, ores)
        for i in range(n):
            assert (res[i]["status"], res[i]["content_len"], res[i]["content_type"]) == \
                   (ores[i].status, ores[i].content_len, ores[i].content_type), (suite, i)
        assert [int(r) for r in res["status"]] == [0, 0, 0, 0, 51, 0]
        assert int(res[2]["content_len"]) == 5 and int(res[2]["content_type"]) == 22
        assert int(res[1]["content_len"]) == 0 and int(res[1]["content_type"]) == 0


def test_batch_raw_mode_vs_oracle(eng):
    rng = np.random.default_rng(9)
    n = 200
    suites = np.array([0x1301, 0x1302, 0x1303], dtype=np.uint16)
    keys = workload.make_keys(n, rng.choice(suites, size=n))
    recs = np.zeros(n, atls.REC_DTYPE)
    aux_parts, in_parts = [], []
    aoff = ioff = 0
    for i in range(n):
        L = int(rng.choice([0, 1, 16, 64, 100, 1000, 4096, 5000]))
        ivl = 12 if keys[i]["suite"] == 0x1303 else int(rng.choice([12, 12, 1, 8, 16, 60]))
        al = int(rng.choice([0, 1, 5, 16, 17, 100]))
        r = recs[i:i + 1]
        r["in_off"], r["out_off"], r["aux_off"], r["len"], r["key_slot"] = ioff, ioff, aoff, L, i
        r["aad_len"], r["mode"], r["iv_len"] = al, atls.MODE_RAW, ivl
        aux_parts.append(rng.integers(0, 256, ivl + al, dtype=np.uint8))
        aoff += ivl + al
        in_parts.append(rng.integers(0, 256, (L + 15) // 16 * 16, dtype=np.uint8))
        ioff += (L + 15) // 16 * 16
    aux = np.concatenate(aux_parts + [np.zeros(16, np.uint8)])
    inbuf = np.concatenate(in_parts + [np.zeros(16, np.uint8)])
    batch = dict(keys=keys, recs=recs, out_bytes=len(inbuf))
    out, tags, oout, otags = seal_both(eng, batch, inbuf, aux)
    assert_same(out, tags, oout, otags, recs)
    pt = np.zeros_like(out)
    res = np.zeros(n, atls.OPEN_RESULT_DTYPE)
    eng.open_batch(recs, out, aux, tags, pt, res)
    assert (res["status"] == 0).all()
    for i in range(n):
        o, L = int(recs[i]["out_off"]), int(recs[i]["len"])
        assert pt[o:o + L].tobytes() == inbuf[o:o + L].tobytes(), i


def test_unaligned_offsets(eng):
    rng = np.random.default_rng(13)
    n = 64
    lens = rng.integers(0, 3000, size=n).astype(np.uint64)
    batch = workload.tls_batch(n, lens, mixed_suites, n_keys=5)
    recs = batch["recs"]
    recs["in_off"] += np.arange(n, dtype=np.uint64) * 7 + 3
    recs["out_off"] += np.arange(n, dtype=np.uint64) * 5 + 1
    batch["in_bytes"] += 7 * n + 16
    batch["out_bytes"] += 5 * n + 16
    inbuf = fill_payload(batch, 3)
    out, tags, oout, otags = seal_both(eng, batch, inbuf)
    assert_same(out, tags, oout, otags, recs)


def test_device_pointers_inplace_and_device_recs(eng):
    torch = pytest.importorskip("torch")
    n = 512
    batch = workload.tls_batch(n, 4096, mixed_suites, n_keys=64)
    recs = batch["recs"].copy()
    # in-place: TLS open of the ciphertext, written back over itself
    inbuf = fill_payload(batch, 21)
    eng.set_keys(batch["keys"])
    ref_out = np.zeros(batch["out_bytes"], np.uint8)
    ref_tags = np.zeros(16 * n, np.uint8)
    eng.seal_batch(recs, inbuf, np.zeros(16, np.uint8), ref_out, ref_tags)
    dev = torch.device("cuda", eng.device)
    d_in = torch.from_numpy(inbuf).to(dev)
    d_out = torch.zeros(batch["out_bytes"], dtype=torch.uint8, device=dev)
    d_tags = torch.zeros(16 * n, dtype=torch.uint8, device=dev)
    d_aux = torch.zeros(16, dtype=torch.uint8, device=dev)
    d_recs = torch.from_numpy(recs.view(np.uint8)).to(dev)
    torch.cuda.synchronize()
    eng.seal_batch(d_recs.data_ptr(), d_in, d_aux, d_out, d_tags,
                   flags=atls.FLAG_DEVICE_PTRS | atls.FLAG_DEVICE_RECS, n=n)
    assert np.array_equal(d_out.cpu().numpy(), ref_out) and np.array_equal(d_tags.cpu().numpy(), ref_tags)
    orecs = recs.copy()
    orecs["in_off"] = recs["out_off"]
    orecs["len"] = recs["len"] + 1
    d_res = torch.zeros(8 * n, dtype=torch.uint8, device=dev)
    eng.open_batch(orecs, d_out, d_aux, d_tags, d_out, d_res, flags=atls.FLAG_DEVICE_PTRS)  # in place
    res = d_res.cpu().numpy().view(atls.OPEN_RESULT_DTYPE)
    assert (res["status"] == 0).all() and (res["content_len"] == 4096).all()
    o = d_out.cpu().numpy()
    for i in range(0, n, 37):
        a, b = int(recs[i]["out_off"]), int(recs[i]["in_off"])
        assert o[a:a + 4096].tobytes() == inbuf[b:b + 4096].tobytes()


def test_c2_sample_vs_oracle(eng):
    batch = workload.config_batch("c2_aes128gcm_64Ki_x_16KiB", n=2048)
    inbuf = fill_payload(batch, workload.SEEDS["payload"])
    out, tags, oout, otags = seal_both(eng, batch, inbuf)
    assert_same(out, tags, oout, otags, batch["recs"])


def test_c3_full_vs_openssl_and_sample_vs_oracle(eng):
    batch = workload.config_batch("c3_chacha20poly1305_64Ki_x_1.5KiB")
    inbuf = fill_payload(batch, workload.SEEDS["payload"])
    eng.set_keys(batch["keys"])
    recs, keys = batch["recs"], batch["keys"]
    out = np.zeros(batch["out_bytes"], np.uint8)
    tags = np.zeros(16 * len(recs), np.uint8)
    eng.seal_batch(recs, inbuf, np.zeros(16, np.uint8), out, tags)
    for i in range(0, len(recs), 1):
        r = recs[i]
        k = keys[r["key_slot"]]
        L, io, oo = int(r["len"]), int(r["in_off"]), int(r["out_off"])
        nonce = ora.per_record_nonce(bytes(k["static_iv"]), int(r["seq"]))
        hdr = bytes([23, 3, 3, (L + 17) >> 8, (L + 17) & 255])
        ect, etag = openssl_ref.seal("chacha", bytes(k["key"]), nonce, inbuf[io:io + L].tobytes() + b"\x17", hdr)
        assert out[oo:oo + L + 1].tobytes() == ect and tags[16 * i:16 * i + 16].tobytes() == etag, i
    sub = workload.config_batch("c3_chacha20poly1305_64Ki_x_1.5KiB", n=1024)
    o2, t2, oo2, ot2 = seal_both(eng, sub, inbuf)
    assert_same(o2, t2, oo2, ot2, sub["recs"])


def test_derive_keys_vs_oracle(eng):
    secret = H("b67b7d690cc16c4e75e54213cb2d37b4e9c912bcded9105d42befd59d391ad38")  # RFC 8448
    k = eng.derive_keys(0x1301, secret)
    assert bytes(k[0]["key"][:16]).hex() == "3fce516009c21727d0f2e4e86ee403bc"
    assert bytes(k[0]["static_iv"]).hex() == "5d313eb2671276ee13000b30"
    rng = np.random.default_rng(17)
    for suite, hl, kl in [(0x1301, 32, 16), (0x1302, 48, 32), (0x1303, 32, 32)]:
        secrets = rng.integers(0, 256, size=(50, hl), dtype=np.uint8)
        got = eng.derive_keys(suite, secrets.tobytes())
        for i in range(50):
            rc, key, iv = ora.key_from_secret(hl, secrets[i].tobytes(), kl, 12)
            assert rc == 0 and bytes(got[i]["key"][:kl]) == key and bytes(got[i]["static_iv"]) == iv
            assert int(got[i]["suite"]) == suite and int(got[i]["key_len"]) == kl
