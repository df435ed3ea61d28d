"""GPU: the three ChaCha20-Poly1305 lane widths (chacha.hip). In a direct batch each wave takes 32
consecutive records and runs them 2 lanes per record when all are tiny (<= ATLS_CHACHA_TINY = 2048
B), else 4 lanes per record in two rounds when all are short (<= ATLS_CHACHA_SHORT = 4096 B), else
16 lanes per record in eight rounds (the third case below puts one long record among short ones,
so two widths run in one launch); a batch of at most ATLS_CHACHA_LAT_MAX = 32 records (the single
call) runs one record per wave at 64 lanes (chacha_kernel_lat, the fourth case); each case runs on the
2-wave and on the 3-wave direct kernel (ATLS_CHACHA_W2); all are
checked against the oracle on the lengths that exercise the per-lane Poly1305 combine and the
reference's F4 quirk (ChaCha20::encrypt leaves the last block unencrypted when len % 64 == 0,
crypto/chacha20/cipher.rs:99-102), sealed and reopened, with tampered tags."""
import numpy as np
import pytest

import oracle as ora

pytestmark = pytest.mark.gpu

SHORT = [0, 1, 15, 16, 17, 62, 63, 64, 65, 127, 128, 191, 255, 256, 1000, 1023, 1024, 1535, 1536, 2047, 4095, 4096]
TINY = [n for n in SHORT if n < 2048]


@pytest.fixture(scope="module")
def atls():
    import anothertls_amd as a

    if not a.device_available():
        pytest.skip("no HIP device")
    return a


@pytest.mark.parametrize("w2", ["1", "0"], ids=["2-wave-kernel", "3-wave-kernel"])
@pytest.mark.parametrize("lens", [TINY * 20, SHORT * 20, SHORT * 20 + [16384], SHORT + [16383, 16384, 5000]],
                         ids=["all-tiny-2-lanes", "all-short-4-lanes", "one-long-16-lanes", "few-records-64-lanes"])
def test_chacha_widths_vs_oracle(atls, lens, w2, monkeypatch):
    """w2: direct batches take chacha_kernel_w2 (256 VGPRs, each slot's data loaded a step ahead);
    ATLS_CHACHA_W2=0 sends them to the 3-wave chacha_kernel, so both direct kernels see every width."""
    from anothertls_amd import workload

    monkeypatch.setenv("ATLS_CHACHA_W2", w2)
    lens = np.array(lens, np.uint64)
    n = len(lens)
    b = workload.tls_batch(n, lens, 0x1303, n_keys=7)
    recs = b["recs"]
    rng = np.random.default_rng(n)
    inbuf = rng.integers(0, 256, b["in_bytes"] + 16, dtype=np.uint8)
    eng = atls.Engine(0)
    eng.set_keys(b["keys"])
    out = np.zeros(b["out_bytes"] + 16, np.uint8)
    tags = np.zeros(16 * n, np.uint8)
    eng.seal_batch(recs, inbuf, np.zeros(16, np.uint8), out, tags)
    okeys = (ora.OraKey * len(b["keys"])).from_buffer_copy(b["keys"].tobytes())
    orecs = (ora.OraRec * n).from_buffer_copy(recs.tobytes())
    oout, otags = np.zeros_like(out), np.zeros_like(tags)
    assert ora.seal_batch(okeys, orecs, inbuf, np.zeros(16, np.uint8), oout, otags, 8) == 0
    assert np.array_equal(out, oout) and np.array_equal(tags, otags)
    r2 = recs.copy()
    r2["in_off"], r2["len"] = recs["out_off"], recs["len"] + 1
    bad = tags.copy()
    bad[16 * np.arange(0, n, 5) + 7] ^= 0x40
    pt = np.zeros_like(out)
    res = np.zeros(n, atls.OPEN_RESULT_DTYPE)
    eng.open_batch(r2, out, np.zeros(16, np.uint8), bad, pt, res)
    tampered = np.arange(n) % 5 == 0
    assert (res["status"][tampered] == 50).all() and (res["status"][~tampered] == 0).all()
    assert (res["content_len"][~tampered] == recs["len"][~tampered]).all()
    for i in np.flatnonzero(~tampered)[::7]:
        o, io, L = int(r2["out_off"][i]), int(recs["in_off"][i]), int(recs["len"][i])
        assert np.array_equal(pt[o:o + L], inbuf[io:io + L]), i
    eng.close()


@pytest.mark.parametrize("w2", ["1", "2"], ids=["past-2-waves-3-wave-kernel", "default-2-wave-kernel"])
def test_chacha_direct_batch_past_two_waves_per_simd(atls, w2, monkeypatch):
    """A direct batch one wave step larger than two waves per SIMD of work (8 x CUs x 32 records + 32)
    leaves chacha_kernel_w2 for the 3-wave chacha_kernel under ATLS_CHACHA_W2=1; the default (2) keeps the
    2-wave kernel at every size, its waves then taking several wave steps each. Both against the oracle."""
    import torch
    from anothertls_amd import workload

    monkeypatch.setenv("ATLS_CHACHA_W2", w2)
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    n = 8 * cus * 32 + 32
    lens = np.random.default_rng(n).integers(0, 200, n).astype(np.uint64)
    b = workload.tls_batch(n, lens, 0x1303, n_keys=97)
    recs = b["recs"]
    inbuf = np.random.default_rng(1).integers(0, 256, b["in_bytes"] + 16, dtype=np.uint8)
    eng = atls.Engine(0)
    eng.set_keys(b["keys"])
    out = np.zeros(b["out_bytes"] + 16, np.uint8)
    tags = np.zeros(16 * n, np.uint8)
    eng.seal_batch(recs, inbuf, np.zeros(16, np.uint8), out, tags)
    okeys = (ora.OraKey * len(b["keys"])).from_buffer_copy(b["keys"].tobytes())
    orecs = (ora.OraRec * n).from_buffer_copy(recs.tobytes())
    oout, otags = np.zeros_like(out), np.zeros_like(tags)
    assert ora.seal_batch(okeys, orecs, inbuf, np.zeros(16, np.uint8), oout, otags, 8) == 0
    assert np.array_equal(out, oout) and np.array_equal(tags, otags)
    r2 = recs.copy()
    r2["in_off"], r2["len"] = recs["out_off"], recs["len"] + 1
    pt = np.zeros_like(out)
    res = np.zeros(n, atls.OPEN_RESULT_DTYPE)
    eng.open_batch(r2, out, np.zeros(16, np.uint8), tags, pt, res)
    assert (res["status"] == 0).all() and (res["content_len"] == recs["len"]).all()
    eng.close()
