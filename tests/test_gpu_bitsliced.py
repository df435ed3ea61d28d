"""GPU parity of the bitsliced AES-GCM kernels (anothertls_amd/csrc/gcm_bs.hip).

The batch split (gcm_common.h bs_class/bs_taken) sends records of >= 1023 full blocks with a
96-bit nonce to the bitsliced kernels and everything else to the T-table kernel. These tests
build batches around that boundary and compare every byte and tag against the oracle, and the
bitsliced engine (ATLS_GCM_BS=1; off by default while it is slower than the T-table kernel on
the headline config) against one with the bitsliced path switched off (ATLS_GCM_BS=0)."""
import os

import numpy as np
import pytest

import anothertls_amd as atls
import oracle as ora
from anothertls_amd import workload
from test_gpu_parity import NTHREADS, assert_same, oracle_keys, oracle_recs, seal_both

pytestmark = pytest.mark.gpu

# content lengths around the eligibility boundary (TLS seal: len // 16 + 1 >= 1024 and at most
# 64 blocks after the last full pass) and past it
BOUNDARY_LENS = [16351, 16352, 16367, 16368, 16369, 16383, 16384, 16385, 16400, 16401, 17000, 17391, 17392,
                 17393, 17407, 17408, 18000, 32751, 32752, 32767, 32768, 33279, 33280, 33281, 65535]


def _engine(bs):
    old = os.environ.get("ATLS_GCM_BS")
    os.environ["ATLS_GCM_BS"] = "1" if bs else "0"
    try:
        return atls.Engine(int(os.environ.get("ATLS_DEVICE", "0")))
    finally:
        if old is None:
            del os.environ["ATLS_GCM_BS"]
        else:
            os.environ["ATLS_GCM_BS"] = old


@pytest.fixture(scope="module")
def engines():
    a, b = _engine(True), _engine(False)
    yield a, b
    a.close()
    b.close()


def aes_suites(k):
    r = np.random.default_rng(3)
    return r.choice(np.array([0x1301, 0x1302], dtype=np.uint16), size=k)


def _seal(eng, batch, inbuf, aux):
    eng.set_keys(batch["keys"])
    out = np.zeros(max(batch["out_bytes"], 16), np.uint8)
    tags = np.zeros(16 * len(batch["recs"]), np.uint8)
    eng.seal_batch(batch["recs"], inbuf, aux, out, tags)
    return out, tags


def test_tls_boundary_lengths_vs_oracle_and_ttable(engines):
    bs, tt = engines
    rng = np.random.default_rng(41)
    lens = np.array(BOUNDARY_LENS * 3 + list(rng.integers(16000, 18000, size=60)), dtype=np.uint64)
    rng.shuffle(lens)
    batch = workload.tls_batch(len(lens), lens, aes_suites, n_keys=23, seq_base=2**32 - 5)
    batch["keys"][4]["key_len"] = 24  # an AES-192 connection
    batch["keys"][4]["suite"] = 0x1301
    inbuf = np.random.default_rng(1).integers(0, 256, size=batch["in_bytes"] + 16, dtype=np.uint8)
    out, tags, oout, otags = seal_both(bs, batch, inbuf)
    assert_same(out, tags, oout, otags, batch["recs"])
    out2, tags2 = _seal(tt, batch, inbuf, np.zeros(16, np.uint8))
    assert np.array_equal(out, out2) and np.array_equal(tags, tags2)


def test_tls_open_padding_and_tamper(engines):
    bs, _ = engines
    n = 64
    rng = np.random.default_rng(43)
    lens = np.array([16384, 16380, 16370, 16368] * 16, dtype=np.uint64)
    batch = workload.tls_batch(n, lens, aes_suites, n_keys=7)
    recs = batch["recs"]
    inbuf = rng.integers(0, 256, size=batch["in_bytes"] + 16, dtype=np.uint8)
    # trailing zero padding inside the content (record.rs:229-237 scans back over it), of a length
    # that ends the non-zero bytes inside a full pass, in the tail, or nowhere (all zero)
    types = np.zeros(n, np.uint8)
    for i in range(n):
        io, L = int(recs[i]["in_off"]), int(recs[i]["len"])
        z = [0, 1, 17, 40, 300, L][i % 6]
        inbuf[io + L - z:io + L] = 0
        if i % 6 in (1, 2, 3):
            types[i] = 0  # type byte 0: the scan continues into the content
            inbuf[io + L - z - 1] = [20, 21, 22, 23][i % 4]
        else:
            types[i] = 23
    recs["content_type"] = types
    out, tags, oout, otags = seal_both(bs, batch, inbuf)
    assert_same(out, tags, oout, otags, recs)
    orecs = recs.copy()
    orecs["in_off"] = recs["out_off"]
    orecs["len"] = recs["len"] + 1
    tags_t = tags.copy()
    for i in range(0, n, 9):
        tags_t[16 * i + 3] ^= 0x10
    pt = np.zeros_like(out)
    res = np.zeros(n, atls.OPEN_RESULT_DTYPE)
    bs.open_batch(orecs, out, np.zeros(16, np.uint8), tags_t, pt, res)
    ores = (ora.OraOpenResult * n)()
    opt = np.zeros_like(out)
    ora.open_batch(oracle_keys(batch["keys"]), oracle_recs(orecs), out, np.zeros(16, np.uint8), tags_t, opt, ores)
    for i in range(n):
        assert (int(res[i]["status"]), int(res[i]["content_len"]), int(res[i]["content_type"])) == \
               (ores[i].status, ores[i].content_len, ores[i].content_type), i
        if i % 9:
            o, L = int(recs[i]["out_off"]), int(recs[i]["len"])
            assert pt[o:o + L + 1].tobytes() == opt[o:o + L + 1].tobytes(), i


def _raw_batch(rng, lens, aads, n_keys=11):
    n = len(lens)
    keys = workload.make_keys(n_keys, aes_suites(n_keys))
    recs = np.zeros(n, atls.REC_DTYPE)
    aux_parts, in_parts = [], []
    aoff = ioff = 0
    for i in range(n):
        L, al = int(lens[i]), int(aads[i])
        r = recs[i:i + 1]
        r["in_off"], r["out_off"], r["aux_off"], r["len"], r["key_slot"] = ioff, ioff, aoff, L, i % n_keys
        r["aad_len"], r["mode"], r["iv_len"] = al, atls.MODE_RAW, 12
        aux_parts.append(rng.integers(0, 256, 12 + al, dtype=np.uint8))
        aoff += 12 + al
        in_parts.append(rng.integers(0, 256, (L + 15) // 16 * 16, dtype=np.uint8))
        ioff += (L + 15) // 16 * 16
    aux = np.concatenate(aux_parts + [np.zeros(16, np.uint8)])
    inbuf = np.concatenate(in_parts + [np.zeros(16, np.uint8)])
    return dict(keys=keys, recs=recs, out_bytes=len(inbuf)), inbuf, aux


def test_raw_mode_multi_pass_and_long_aad(engines):
    bs, tt = engines
    rng = np.random.default_rng(47)
    lens = [16368, 16384, 16400, 17392, 32752, 32768, 33280, 49136, 65520, 65536, 66000, 16384, 16384, 20000]
    aads = [0, 1, 13, 16, 17, 100, 255, 256, 511, 512, 513, 32, 496, 5]
    batch, inbuf, aux = _raw_batch(rng, lens, aads)
    out, tags, oout, otags = seal_both(bs, batch, inbuf, aux)
    assert_same(out, tags, oout, otags, batch["recs"])
    out2, tags2 = _seal(tt, batch, inbuf, aux)
    assert np.array_equal(out, out2) and np.array_equal(tags, tags2)
    pt = np.zeros_like(out)
    res = np.zeros(len(lens), atls.OPEN_RESULT_DTYPE)
    bs.open_batch(batch["recs"], out, aux, tags, pt, res)
    assert (res["status"] == 0).all()
    assert np.array_equal(pt[:len(inbuf) - 16], inbuf[:len(inbuf) - 16])
    bad = tags.copy()
    bad[16 * 4] ^= 1
    bs.open_batch(batch["recs"], out, aux, bad, pt, res)
    assert int(res[4]["status"]) == 20 and (np.delete(res["status"], 4) == 0).all()


def test_c4_shape_sample_vs_oracle(engines):
    bs, _ = engines
    batch = workload.config_batch("c4_aes256gcm_1Mi_x_16KiB", n=1024)
    inbuf = np.random.default_rng(workload.SEEDS["payload"]).integers(0, 256, size=batch["in_bytes"], dtype=np.uint8)
    out, tags, oout, otags = seal_both(bs, batch, inbuf)
    assert_same(out, tags, oout, otags, batch["recs"])
