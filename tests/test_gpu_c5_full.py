"""BASELINE config C5 at its stated size on one MI355X: the whole mixed batch -- 262,144
TLS records, suite ~ Bernoulli(0.5) between AES-128-GCM and ChaCha20-Poly1305, content U{64..16384}
(2.16 GB in, 2.16 GB out, input and output offsets well past 2^31) -- sealed through the planned mixed
path (plan.hip, gcm_kernel beside chacha_kernel<..., true> on the side stream)

* by one engine, and
* by atls_multi with device 0 repeated 8 times in ATLS_MULTI_RCCL_SELF=1 mode: the root-resident layout
  of the 8-GPU config, every non-root part's byte-balanced range scattered and gathered over RCCL,

each compared against the oracle on EVERY record (the ChaCha last-block-quirk records included,
chacha20/cipher.rs:99-102), the non-quirk records also against OpenSSL, the records that
straddle the 2^31 and 2^32 input and output offsets named and checked explicitly, and opened back on the
device with tampered tags: DecryptError (50) exactly at the tampered records, every other record's
plaintext byte for byte.
Reference: net/record.rs:162-240, crypto/aes/gcm.rs:42-162, crypto/chacha20/poly1305.rs:69-104,
net/key_schedule.rs:51-64 (records are independent, so a sharded batch equals the whole batch)."""
import os

import numpy as np
import pytest

import anothertls_amd as atls
import openssl_ref
import oracle as ora
from anothertls_amd import workload

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
C5 = "c5_mixed_256Ki_x_64B-16KiB"
NTHREADS = 16
CHUNK = 1 << 30
BOUNDS = (1 << 31, 1 << 32)


@pytest.fixture(scope="module")
def c5():
    batch = workload.config_batch(C5)
    recs, keys = batch["recs"], batch["keys"]
    n = len(recs)
    chacha = keys["suite"][recs["key_slot"]] == int(atls.CipherSuite.TLS_CHACHA20_POLY1305_SHA256)
    assert n == 262144 and 0.45 < chacha.mean() < 0.55
    assert batch["in_bytes"] > (1 << 31) and batch["out_bytes"] > (1 << 31)
    dev = torch.device("cuda", int(os.environ.get("ATLS_DEVICE", "0")))
    g = torch.Generator(device=dev).manual_seed(workload.SEEDS["payload"])
    d_in = torch.randint(0, 256, (batch["in_bytes"] + 16,), dtype=torch.uint8, device=dev, generator=g)
    h_in = d_in.cpu().numpy()
    # the oracle (the reference's algorithm restated) seals every record: the expected bytes of both tests
    okeys = (ora.OraKey * len(keys)).from_buffer_copy(keys.tobytes())
    orecs = (ora.OraRec * n).from_buffer_copy(recs.tobytes())
    want_out = np.zeros(batch["out_bytes"] + 16, np.uint8)
    want_tags = np.zeros(16 * n, np.uint8)
    assert ora.seal_batch(okeys, orecs, h_in, np.zeros(16, np.uint8), want_out, want_tags, NTHREADS) == 0
    quirk = chacha & ((recs["len"].astype(np.int64) + 1) % 64 == 0)
    assert quirk.sum() > 0
    # OpenSSL independently, on every record where the reference is standard
    eout, etags, skipped = openssl_ref.seal_tls_batch(keys, recs, h_in, batch["out_bytes"] + 16, NTHREADS)
    assert np.array_equal(skipped.astype(bool), quirk), "OpenSSL skips exactly the F4-quirk records"
    lo_out = recs["out_off"].astype(np.int64)
    for i in np.flatnonzero(quirk):  # OpenSSL left these zero: take the oracle's bytes there
        a, b = lo_out[i], lo_out[i] + int(recs["len"][i]) + 1
        eout[a:b] = want_out[a:b]
    bad_tags = np.flatnonzero((etags.reshape(-1, 16) != want_tags.reshape(-1, 16)).any(axis=1) & ~quirk)
    assert not len(bad_tags), f"oracle != OpenSSL tags on {bad_tags[:5]}"
    assert np.array_equal(eout, want_out), "oracle != OpenSSL ciphertext on a non-quirk record"
    del eout, etags
    yield dict(batch=batch, dev=dev, d_in=d_in, h_in=h_in, want_out=want_out, want_tags=want_tags,
               chacha=chacha, quirk=quirk)


def _straddlers(recs):
    """Records whose input or output range crosses (or starts at) 2^31 or 2^32, and their neighbours."""
    lo_in, lo_out = recs["in_off"].astype(np.int64), recs["out_off"].astype(np.int64)
    hi_in, hi_out = lo_in + recs["len"].astype(np.int64), lo_out + recs["len"].astype(np.int64) + 1
    pick = set()
    for b in BOUNDS:
        for lo, hi in ((lo_in, hi_in), (lo_out, hi_out)):
            for i in np.flatnonzero((lo <= b) & (hi > b - 1)).tolist():
                pick.update(j for j in (i - 1, i, i + 1) if 0 <= j < len(recs))
    pick.add(len(recs) - 1)
    return sorted(pick)


def _check_sealed(c5, d_out, d_tags):
    """Every record's ciphertext and tag against the oracle; the straddlers one by one first."""
    recs, want_out, want_tags = c5["batch"]["recs"], c5["want_out"], c5["want_tags"]
    h_tags = d_tags.cpu().numpy()
    which = _straddlers(recs)
    assert max(int(recs["in_off"][i]) for i in which) > (1 << 31)
    for i in which:
        o, L = int(recs["out_off"][i]), int(recs["len"][i]) + 1
        assert d_out[o:o + L].cpu().numpy().tobytes() == want_out[o:o + L].tobytes(), f"straddler {i}"
        assert h_tags[16 * i:16 * i + 16].tobytes() == want_tags[16 * i:16 * i + 16].tobytes(), f"straddler {i} tag"
    bad_tags = np.flatnonzero((h_tags.reshape(-1, 16) != want_tags.reshape(-1, 16)).any(axis=1))
    assert not len(bad_tags), f"{len(bad_tags)} tags differ from the oracle, first {bad_tags[:5]}"
    # outputs: the gaps between records are zero on both sides, so whole 1 GiB pieces compare
    for off in range(0, want_out.size, CHUNK):
        a = d_out[off:off + CHUNK].cpu().numpy()
        if not np.array_equal(a, want_out[off:off + CHUNK]):
            first = off + int(np.flatnonzero(a != want_out[off:off + CHUNK])[0])
            rec = int(np.searchsorted(recs["out_off"].astype(np.int64), first, side="right") - 1)
            raise AssertionError(f"ciphertext differs from the oracle at byte {first} (record {rec})")


def _open_back(c5, opener, d_out, d_tags):
    """Open every sealed record on the device with some tags tampered: DecryptError exactly there, every
    other record's status, length, type and plaintext."""
    batch, d_in, chacha, quirk = c5["batch"], c5["d_in"], c5["chacha"], c5["quirk"]
    recs = batch["recs"]
    n = len(recs)
    dev = d_in.device
    rng = np.random.default_rng(0xC5)
    straddle = _straddlers(recs)
    tamper = sorted(set(rng.integers(0, n, 256).tolist()) | {int(np.flatnonzero(chacha)[-1]),
                                                             int(np.flatnonzero(~chacha)[-1]),
                                                             int(np.flatnonzero(quirk)[-1]), straddle[len(straddle) // 2]})
    d_tags = d_tags.clone()
    d_tags[torch.as_tensor(np.asarray(tamper, np.int64) * 16, device=dev)] ^= 0x80
    orecs = recs.copy()
    orecs["in_off"], orecs["len"] = recs["out_off"], recs["len"] + 1
    d_pt = torch.zeros_like(d_out)
    d_res = torch.zeros(8 * n, dtype=torch.uint8, device=dev)
    opener(orecs, d_out, d_tags, d_pt, d_res)
    res = d_res.cpu().numpy().view(atls.OPEN_RESULT_DTYPE)
    bad = np.zeros(n, bool)
    bad[tamper] = True
    assert (res["status"][bad] == atls.TlsError.DECRYPT_ERROR).all()
    assert (res["status"][~bad] == 0).all(), np.flatnonzero((res["status"] != 0) & ~bad)[:5]
    assert (res["content_len"][~bad] == recs["len"][~bad]).all() and (res["content_type"][~bad] == 23).all()
    # plaintext: records are packed by offset, so walk 1 GiB windows of both buffers
    io, oo, L = (recs[k].astype(np.int64) for k in ("in_off", "out_off", "len"))
    h_in = c5["h_in"]
    a = 0
    while a < n:
        base = oo[a]
        b = int(np.searchsorted(oo, base + CHUNK, side="left"))
        b = max(b, a + 1)
        win = d_pt[base:oo[b - 1] + L[b - 1]].cpu().numpy()
        for i in range(a, b):
            if bad[i]:
                continue
            got = win[oo[i] - base:oo[i] - base + L[i]]
            assert got.tobytes() == h_in[io[i]:io[i] + L[i]].tobytes(), f"plaintext of record {i}"
        a = b
    del d_pt


def test_c5_whole_batch_one_engine(c5):
    batch, dev = c5["batch"], c5["dev"]
    recs = batch["recs"]
    n = len(recs)
    eng = atls.Engine(dev.index)
    try:
        eng.set_keys(batch["keys"])
        d_out = torch.zeros(batch["out_bytes"] + 16, dtype=torch.uint8, device=dev)
        d_tags = torch.zeros(16 * n, dtype=torch.uint8, device=dev)
        d_recs = torch.from_numpy(recs.view(np.uint8).copy()).to(dev)
        d_aux = torch.zeros(16, dtype=torch.uint8, device=dev)
        torch.cuda.synchronize()
        eng.seal_batch(d_recs.data_ptr(), c5["d_in"], d_aux, d_out, d_tags,
                       flags=atls.FLAG_DEVICE_PTRS | atls.FLAG_DEVICE_RECS, n=n)
        eng.sync()
        _check_sealed(c5, d_out, d_tags)

        def opener(orecs, ct, tags, pt, res):
            eng.open_batch(orecs, ct, d_aux, tags, pt, res, flags=atls.FLAG_DEVICE_PTRS)

        _open_back(c5, opener, d_out, d_tags)
    finally:
        eng.close()
        torch.cuda.empty_cache()


def test_c5_whole_batch_root_resident_multi_rccl_self_x8(c5):
    """The 8-GPU config's layout on one GPU: the whole mixed batch on the root, eight byte-balanced ranges
    (atls_partition: unequal record counts), seven scattered and gathered by RCCL send / recv (rank 0 to
    itself), each sealed by its own engine through the planned path; then opened the same way."""
    batch, dev = c5["batch"], c5["dev"]
    recs = batch["recs"]
    n = len(recs)
    first = atls.partition(recs, 8)
    cnt = np.diff(first)
    assert cnt.sum() == n and len(set(cnt.tolist())) > 1  # byte-balanced, not count-balanced
    os.environ["ATLS_MULTI_RCCL_SELF"] = "1"
    try:
        m = atls.MultiEngine([dev.index] * 8)
    finally:
        del os.environ["ATLS_MULTI_RCCL_SELF"]
    try:
        assert m.uses_rccl
        m.set_keys(batch["keys"])
        d_out = torch.zeros(batch["out_bytes"] + 16, dtype=torch.uint8, device=dev)
        d_tags = torch.zeros(16 * n, dtype=torch.uint8, device=dev)
        d_aux = torch.zeros(16, dtype=torch.uint8, device=dev)
        m.seal_batch(recs, c5["d_in"], d_aux, d_out, d_tags, flags=atls.FLAG_DEVICE_PTRS)
        torch.cuda.synchronize()
        _check_sealed(c5, d_out, d_tags)

        def opener(orecs, ct, tags, pt, res):
            m.open_batch(orecs, ct, d_aux, tags, pt, res, flags=atls.FLAG_DEVICE_PTRS)

        _open_back(c5, opener, d_out, d_tags)
    finally:
        m.close()
        torch.cuda.empty_cache()
