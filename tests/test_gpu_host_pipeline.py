"""GPU: host-memory batches through the engine's chunked pipeline (engine.cpp run_host_pipelined:
uploads, kernels and downloads on three streams): several chunks, the fixed-pitch layout (record bytes
copied back with hipMemcpy2DAsync, bytes between records untouched) and a variable-length layout (each
chunk's output range staged in and out); and the same batches in page-locked host buffers with
ATLS_ZERO_COPY=1, where the kernels read and write the host buffers in place (engine.cpp host_alias),
and =2, where the inputs go up in chunks and the kernels write their output in place.
Results are checked against the oracle record by record, and the bytes of `out` between records must
come back as the caller left them."""
import numpy as np
import pytest

import oracle as ora

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def atls():
    import anothertls_amd as a

    if not a.device_available():
        pytest.skip("no HIP device")
    return a


def _host(nbytes, pinned):
    if not pinned:
        return np.zeros(nbytes, np.uint8)
    import torch

    return torch.zeros(nbytes, dtype=torch.uint8, pin_memory=True).numpy()


def _check(atls, b, seed, pinned=False):
    eng = atls.Engine(0)
    eng.set_keys(b["keys"])
    rng = np.random.default_rng(seed)
    n = len(b["recs"])
    inbuf = _host(b["in_bytes"] + 16, pinned)
    inbuf[:] = rng.integers(0, 256, b["in_bytes"] + 16, dtype=np.uint8)
    out = _host(b["out_bytes"] + 16, pinned)
    out[:] = 0xA5  # gap bytes must survive
    tags = _host(16 * n, pinned)
    eng.seal_batch(b["recs"], inbuf, np.zeros(16, np.uint8), out, tags)
    okeys = (ora.OraKey * len(b["keys"])).from_buffer_copy(b["keys"].tobytes())
    orecs = (ora.OraRec * n).from_buffer_copy(b["recs"].tobytes())
    oout = np.full_like(out, 0xA5)
    otags = np.zeros_like(tags)
    assert ora.seal_batch(okeys, orecs, inbuf, np.zeros(16, np.uint8), oout, otags, 16) == 0
    assert np.array_equal(tags, otags)
    assert np.array_equal(out, oout)  # record bytes and the untouched gaps
    # and back: open in host memory through the same pipeline
    r2 = b["recs"].copy()
    r2["in_off"], r2["len"] = b["recs"]["out_off"], b["recs"]["len"] + 1
    pt = _host(out.nbytes, pinned)
    res = _host(n * atls.OPEN_RESULT_DTYPE.itemsize, pinned).view(atls.OPEN_RESULT_DTYPE)
    eng.open_batch(r2, out, np.zeros(16, np.uint8), tags, pt, res)
    assert (res["status"] == 0).all() and (res["content_len"] == b["recs"]["len"]).all()
    for i in range(0, n, max(1, n // 64)):
        o, L = int(r2["in_off"][i]), int(b["recs"]["len"][i])
        io = int(b["recs"]["in_off"][i])
        assert np.array_equal(pt[o:o + L], inbuf[io:io + L]), i
    eng.close()


@pytest.mark.parametrize("zero_copy", [0, 1, 2], ids=["staged", "zero-copy", "zero-copy-out"])
def test_pitched_layout_multi_chunk(atls, zero_copy, monkeypatch):
    from anothertls_amd import workload

    monkeypatch.setenv("ATLS_ZERO_COPY", str(zero_copy))
    b = workload.tls_batch(6000, 16000, 0x1301, n_keys=64)  # ~96 MiB: 6 chunks, fixed pitch
    _check(atls, b, 5, pinned=bool(zero_copy))


@pytest.mark.parametrize("zero_copy", [0, 1, 2], ids=["staged", "zero-copy", "zero-copy-out"])
def test_variable_layout_multi_chunk(atls, zero_copy, monkeypatch):
    from anothertls_amd import workload

    monkeypatch.setenv("ATLS_ZERO_COPY", str(zero_copy))
    lens = np.random.default_rng(9).integers(0, 16385, 9000).astype(np.uint64)
    b = workload.tls_batch(len(lens), lens, 0x1303, n_keys=32)  # ~72 MiB, staged chunks
    _check(atls, b, 6, pinned=bool(zero_copy))


def test_zero_copy_mixed_suites_planned(atls, monkeypatch):
    """A planned (AES-GCM + ChaCha20-Poly1305) batch in page-locked buffers, read and written in place."""
    from anothertls_amd import workload

    monkeypatch.setenv("ATLS_ZERO_COPY", "1")
    b = workload.shard_batch("c5_mixed_256Ki_x_64B-16KiB", 0, n=3000)
    _check(atls, b, 7, pinned=True)
