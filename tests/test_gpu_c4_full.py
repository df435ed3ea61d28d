"""BASELINE config C4 at its stated size on one MI355X: AES-256-GCM over the whole
1 Mi x 16 KiB batch -- 17.2 GB in, 17.2 GB out, one device-resident launch, every buffer past the 2^32,
2^33 and 2^34-byte offsets -- sealed

* by one engine, and
* by atls_multi with device 0 repeated 8 times in ATLS_MULTI_RCCL_SELF=1 mode: the root-resident layout
  of the 8-GPU config, with every part's range scattered and gathered over RCCL (rank 0 to itself),

each compared against OpenSSL on EVERY record (ciphertext and tag; valid for 96-bit-IV GCM),
against the oracle on the records that straddle the 2^32 / 2^33 / 2^34 input and output offsets, and
opened back on the device with every plaintext byte compared.
Reference: crypto/aes/gcm.rs:42-162, net/record.rs:162-240, net/key_schedule.rs:51-64 (records are
independent, so a sharded batch must equal the whole batch byte for byte)."""
import os

import numpy as np
import pytest

import anothertls_amd as atls
import openssl_ref
import oracle as ora
from anothertls_amd import workload

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
C4 = "c4_aes256gcm_1Mi_x_16KiB"
NTHREADS = 16
CHUNK = 1 << 30


@pytest.fixture(scope="module")
def c4():
    batch = workload.config_batch(C4)
    recs = batch["recs"]
    assert len(recs) == 1048576 and (batch["keys"]["key_len"] == 32).all()
    assert batch["in_bytes"] == 1 << 34 and batch["out_bytes"] > 1 << 34
    dev = torch.device("cuda", int(os.environ.get("ATLS_DEVICE", "0")))
    g = torch.Generator(device=dev).manual_seed(workload.SEEDS["payload"])
    d_in = torch.randint(0, 256, (batch["in_bytes"] + 16,), dtype=torch.uint8, device=dev, generator=g)
    h_in = d_in.cpu().numpy()
    eout, etags, skipped = openssl_ref.seal_tls_batch(batch["keys"], recs, h_in, batch["out_bytes"] + 16, NTHREADS)
    assert not skipped.any()
    yield dict(batch=batch, dev=dev, d_in=d_in, h_in=h_in, eout=eout, etags=etags)


def _first_diff(d_buf, h_buf):
    """First byte offset where the device tensor and the host array differ (1 GiB chunks), or None."""
    assert d_buf.numel() == h_buf.size
    for off in range(0, h_buf.size, CHUNK):
        a = d_buf[off:off + CHUNK].cpu().numpy()
        b = h_buf[off:off + CHUNK]
        if not np.array_equal(a, b):
            return off + int(np.flatnonzero(a != b)[0])
    return None


def _straddlers(recs):
    """Records whose input or output range crosses (or starts at) 2^32, 2^33 or 2^34, and their neighbours."""
    lo_in, lo_out = recs["in_off"].astype(np.int64), recs["out_off"].astype(np.int64)
    hi_in, hi_out = lo_in + recs["len"].astype(np.int64), lo_out + recs["len"].astype(np.int64) + 1
    pick = set()
    for b in (1 << 32, 1 << 33, 1 << 34):
        for lo, hi in ((lo_in, hi_in), (lo_out, hi_out)):
            for i in np.flatnonzero((lo <= b) & (hi > b - 1)).tolist():
                pick.update(j for j in (i - 1, i, i + 1) if 0 <= j < len(recs))
    pick.add(len(recs) - 1)
    return sorted(pick)


def _vs_oracle(c4, d_out, d_tags, which):
    """The oracle (the reference's algorithm restated) on records `which`, rebased into small buffers."""
    batch, h_in = c4["batch"], c4["h_in"]
    sub = batch["recs"][which].copy()
    L = int(sub["len"][0])
    inb = np.concatenate([h_in[int(o):int(o) + L] for o in sub["in_off"]])
    sub["in_off"] = np.arange(len(sub), dtype=np.uint64) * np.uint64(L)
    want_out = np.zeros(len(sub) * (L + 16), np.uint8)
    sub["out_off"] = np.arange(len(sub), dtype=np.uint64) * np.uint64(L + 16)
    want_tags = np.zeros(16 * len(sub), np.uint8)
    okeys = (ora.OraKey * len(batch["keys"])).from_buffer_copy(batch["keys"].tobytes())
    orecs = (ora.OraRec * len(sub)).from_buffer_copy(sub.tobytes())
    assert ora.seal_batch(okeys, orecs, inb, np.zeros(16, np.uint8), want_out, want_tags, 4) == 0
    for k, i in enumerate(which):
        o = int(batch["recs"]["out_off"][i])
        got = d_out[o:o + L + 1].cpu().numpy()
        assert got.tobytes() == want_out[k * (L + 16):k * (L + 16) + L + 1].tobytes(), i
        assert d_tags[16 * i:16 * i + 16].cpu().numpy().tobytes() == want_tags[16 * k:16 * k + 16].tobytes(), i


def _open_back(c4, opener, d_out, d_tags):
    """Open every sealed record on the device; every status, length, type and plaintext byte checked."""
    batch, d_in = c4["batch"], c4["d_in"]
    recs = batch["recs"]
    n = len(recs)
    orecs = recs.copy()
    orecs["in_off"], orecs["len"] = recs["out_off"], recs["len"] + 1
    d_pt = torch.zeros_like(d_out)
    d_res = torch.zeros(8 * n, dtype=torch.uint8, device=c4["dev"])
    opener(orecs, d_out, d_tags, d_pt, d_res)
    res = d_res.cpu().numpy().view(atls.OPEN_RESULT_DTYPE)
    assert (res["status"] == 0).all() and (res["content_len"] == recs["len"]).all() and (res["content_type"] == 23).all()
    L, so = int(recs["len"][0]), int(recs["out_off"][1] - recs["out_off"][0])
    per = CHUNK // so
    for a in range(0, n, per):
        b = min(n, a + per)
        got = d_pt[a * so:b * so].view(b - a, so)[:, :L]
        want = d_in[a * L:b * L].view(b - a, L)
        assert torch.equal(got, want), a
    del d_pt


def test_c4_whole_batch_one_engine(c4):
    batch, dev = c4["batch"], c4["dev"]
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
        eng.seal_batch(d_recs.data_ptr(), c4["d_in"], d_aux, d_out, d_tags,
                       flags=atls.FLAG_DEVICE_PTRS | atls.FLAG_DEVICE_RECS, n=n)
        eng.sync()
        assert np.array_equal(d_tags.cpu().numpy(), c4["etags"]), "tags differ from OpenSSL"
        assert _first_diff(d_out, c4["eout"]) is None
        which = _straddlers(recs)
        assert len(which) >= 6
        _vs_oracle(c4, d_out, d_tags, which)

        def opener(orecs, ct, tags, pt, res):
            eng.open_batch(orecs, ct, d_aux, tags, pt, res, flags=atls.FLAG_DEVICE_PTRS)

        _open_back(c4, opener, d_out, d_tags)
    finally:
        eng.close()
        torch.cuda.empty_cache()


def test_c4_whole_batch_root_resident_multi_rccl_self_x8(c4):
    """The 8-GPU config's layout on one GPU: the whole batch on the root, eight 131,072-record ranges,
    seven of them scattered and gathered by RCCL send / recv (rank 0 to itself), each sealed by its own
    engine; then opened the same way."""
    batch, dev = c4["batch"], c4["dev"]
    recs = batch["recs"]
    n = len(recs)
    first = atls.partition(recs, 8)
    assert np.array_equal(np.diff(first), [n // 8] * 8)
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
        m.seal_batch(recs, c4["d_in"], d_aux, d_out, d_tags, flags=atls.FLAG_DEVICE_PTRS)
        torch.cuda.synchronize()
        assert np.array_equal(d_tags.cpu().numpy(), c4["etags"]), "tags differ from OpenSSL"
        assert _first_diff(d_out, c4["eout"]) is None

        def opener(orecs, ct, tags, pt, res):
            m.open_batch(orecs, ct, d_aux, tags, pt, res, flags=atls.FLAG_DEVICE_PTRS)

        _open_back(c4, opener, d_out, d_tags)
    finally:
        m.close()
        torch.cuda.empty_cache()
