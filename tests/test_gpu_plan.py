"""GPU: the batch plan (anothertls_amd/csrc/plan.hip). A key table with several record kernels
(AES-128, AES-256, ChaCha20-Poly1305) plans every batch: each record lands in its kernel's work
list, lists ordered by length class longest first; rejected records get their status. Results
are checked against the oracle in both planned and direct (single-kernel key table) batches."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def atls():
    import anothertls_amd as a

    if not a.device_available():
        pytest.skip("no HIP device")
    return a


def _plan(atls, eng, n):
    lib = atls.library()
    lib.atls_debug_plan.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32), ctypes.c_uint32]
    hdr_words = 5 + 4 + 64 + 64
    buf = (ctypes.c_uint32 * (hdr_words + n))()
    assert lib.atls_debug_plan(eng._e, buf, n) == 0
    w = np.frombuffer(buf, np.uint32)
    return w[:5].copy(), w[hdr_words:].copy()


def test_plan_lists_and_order(atls):
    import oracle as ora
    from anothertls_amd import workload

    rng = np.random.default_rng(7)
    n = 600
    suites = np.array([0x1301, 0x1302, 0x1303], np.uint16)
    lens = rng.integers(0, 16385, n).astype(np.uint64)
    b = workload.tls_batch(n, lens, lambda k: suites[np.arange(k) % 3], n_keys=3)
    recs = b["recs"].copy()
    eng = atls.Engine(0)
    eng.set_keys(b["keys"])
    inbuf = rng.integers(0, 256, b["in_bytes"], dtype=np.uint8)
    out = np.zeros(b["out_bytes"], np.uint8)
    tags = np.zeros(16 * n, np.uint8)
    eng.seal_batch(recs, inbuf, np.zeros(16, np.uint8), out, tags)
    off, idx = _plan(atls, eng, n)
    slot = recs["key_slot"]
    want = {0: np.flatnonzero(slot == 0), 2: np.flatnonzero(slot == 1), 3: np.flatnonzero(slot == 2)}  # AES-256: 14 rounds
    assert off[4] == n
    for lst, members in want.items():
        got = idx[off[lst]:off[lst + 1]]
        assert sorted(got.tolist()) == sorted(members.tolist()), lst
        cls = np.minimum(recs["len"][got] >> 10, 15)
        assert (np.diff(cls.astype(np.int64)) <= 0).all(), "longest class first"
    assert off[1] == off[2]  # no 12-round keys
    # every accepted record sealed exactly as the oracle does
    okeys = (ora.OraKey * 3).from_buffer_copy(b["keys"].tobytes())
    orecs = (ora.OraRec * n).from_buffer_copy(recs.tobytes())
    oout, otags = np.zeros_like(out), np.zeros_like(tags)
    ora.seal_batch(okeys, orecs, inbuf, np.zeros(16, np.uint8), oout, otags, 8)
    assert np.array_equal(out, oout) and np.array_equal(tags, otags)
    eng.close()


@pytest.mark.parametrize("planned", [False, True])
def test_rejected_records_device_descriptors(atls, planned):
    """Device-resident descriptors skip the host-side check: the plan (or, for a direct batch,
    the kernel) rejects a bad key slot / mode / suite and opens report the status per record."""
    torch = pytest.importorskip("torch")
    from anothertls_amd import workload

    n = 64
    suite_of = (lambda k: np.where(np.arange(k) % 2 == 0, 0x1301, 0x1303).astype(np.uint16)) if planned else 0x1301
    b = workload.tls_batch(n, 1000, suite_of, n_keys=4)
    recs = b["recs"].copy()
    recs["key_slot"][3] = 77  # out of range
    recs["mode"][9] = 5       # unknown mode
    dev = torch.device("cuda", 0)
    eng = atls.Engine(0)
    eng.set_keys(b["keys"])
    d_in = torch.randint(0, 256, (b["out_bytes"] + 64,), dtype=torch.uint8, device=dev)
    d_out = torch.zeros(b["out_bytes"] + 64, dtype=torch.uint8, device=dev)
    d_tags = torch.zeros(16 * n, dtype=torch.uint8, device=dev)
    d_aux = torch.zeros(16, dtype=torch.uint8, device=dev)
    d_res = torch.zeros(8 * n, dtype=torch.uint8, device=dev)
    d_recs = torch.from_numpy(recs.view(np.uint8).copy()).to(dev)
    with pytest.raises(atls.TlsError) as ei:
        eng.open_batch(d_recs.data_ptr(), d_in, d_aux, d_tags, d_out, d_res,
                       flags=atls.FLAG_DEVICE_PTRS | atls.FLAG_DEVICE_RECS, n=n)
    assert ei.value.code == atls.TlsError.ILLEGAL_PARAMETER
    res = d_res.cpu().numpy().view(atls.OPEN_RESULT_DTYPE)
    assert res["status"][3] == atls.TlsError.ILLEGAL_PARAMETER and res["status"][9] == atls.TlsError.ILLEGAL_PARAMETER
    # the other records were opened (random tags: DecryptError in TLS mode)
    others = np.setdiff1d(np.arange(n), [3, 9])
    assert (res["status"][others] == atls.TlsError.DECRYPT_ERROR).all()
    eng.close()


def test_plan_large_batch_many_workgroups(atls):
    """A mixed batch large enough that every plan workgroup strides over several chunks of
    records (300 Ki records, 512 workgroups): every record lands in its list exactly once,
    longest class first, and sampled records seal as the oracle does."""
    import oracle as ora
    from anothertls_amd import workload

    rng = np.random.default_rng(17)
    n = 300 * 1024
    lens = rng.integers(0, 2048, n).astype(np.uint64)
    b = workload.tls_batch(n, lens, lambda k: np.where(np.arange(k) % 2 == 0, 0x1301, 0x1303).astype(np.uint16),
                           n_keys=64)
    recs = b["recs"]
    eng = atls.Engine(0)
    eng.set_keys(b["keys"])
    inbuf = rng.integers(0, 256, b["in_bytes"] + 16, dtype=np.uint8)
    out = np.zeros(b["out_bytes"] + 16, np.uint8)
    tags = np.zeros(16 * n, np.uint8)
    eng.seal_batch(recs, inbuf, np.zeros(16, np.uint8), out, tags)
    off, idx = _plan(atls, eng, n)
    assert off[4] == n
    aes = np.flatnonzero(recs["key_slot"] % 2 == 0)
    for lst, members in ((0, aes), (3, np.setdiff1d(np.arange(n), aes))):
        got = idx[off[lst]:off[lst + 1]]
        assert np.array_equal(np.sort(got), members), lst
        cls = np.minimum(recs["len"][got] >> 10, 15)
        assert (np.diff(cls.astype(np.int64)) <= 0).all()
    sample = np.sort(rng.choice(n, 512, replace=False))
    okeys = (ora.OraKey * len(b["keys"])).from_buffer_copy(b["keys"].tobytes())
    srecs = recs[sample].copy()
    orecs = (ora.OraRec * len(srecs)).from_buffer_copy(srecs.tobytes())
    oout, otags = np.zeros_like(out), np.zeros(16 * len(srecs), np.uint8)
    assert ora.seal_batch(okeys, orecs, inbuf, np.zeros(16, np.uint8), oout, otags, 8) == 0
    for j, i in enumerate(sample):
        o, L = int(recs["out_off"][i]), int(recs["len"][i]) + 1
        assert np.array_equal(out[o:o + L], oout[o:o + L]), i
        assert np.array_equal(tags[16 * i:16 * i + 16], otags[16 * j:16 * j + 16]), i
    eng.close()


def test_sticky_error_reported_at_sync_and_cleared(atls):
    """A descriptor the kernel refuses (device-resident, key slot out of range) sets the engine's
    sticky error word: a NO_SYNC batch returns 0 and the next atls_engine_sync reports
    IllegalParameter (47) once; later batches are clean again (engine.cpp take_err)."""
    torch = pytest.importorskip("torch")
    from anothertls_amd import workload

    for suite in (0x1301, 0x1303):  # the GCM and ChaCha kernels both refuse it
        b = workload.tls_batch(64, 1000, suite, n_keys=4)
        eng = atls.Engine(0)
        eng.set_keys(b["keys"])
        dev = torch.device("cuda", 0)
        recs = b["recs"].copy()
        recs["key_slot"][7] = 99
        d_in = torch.zeros(b["in_bytes"] + 16, dtype=torch.uint8, device=dev)
        d_out = torch.zeros(b["out_bytes"] + 16, dtype=torch.uint8, device=dev)
        d_tags = torch.zeros(16 * 64, dtype=torch.uint8, device=dev)
        d_aux = torch.zeros(16, dtype=torch.uint8, device=dev)
        d_bad = torch.from_numpy(recs.view(np.uint8).copy()).to(dev)
        d_good = torch.from_numpy(b["recs"].view(np.uint8).copy()).to(dev)
        flags = atls.FLAG_DEVICE_PTRS | atls.FLAG_DEVICE_RECS
        eng.seal_batch(d_bad.data_ptr(), d_in, d_aux, d_out, d_tags, flags=flags | atls.FLAG_NO_SYNC, n=64)
        with pytest.raises(atls.TlsError) as e:
            eng.sync()
        assert e.value.code == 47
        eng.sync()  # cleared
        eng.seal_batch(d_good.data_ptr(), d_in, d_aux, d_out, d_tags, flags=flags, n=64)
        with pytest.raises(atls.TlsError) as e:
            eng.seal_batch(d_bad.data_ptr(), d_in, d_aux, d_out, d_tags, flags=flags, n=64)
        assert e.value.code == 47
        eng.seal_batch(d_good.data_ptr(), d_in, d_aux, d_out, d_tags, flags=flags, n=64)
        eng.close()


def test_lazy_join_batches_equal_joined_batches(atls):
    """ATLS_FLAG_LAZY_JOIN (mixed-suite batches leave their ChaCha20-Poly1305 kernel un-joined, the
    two plan sets alternate): many back-to-back planned batches into different output buffers, with
    a key-table update and an open in between, give exactly the joined batches' results; the
    engine stream covers everything after atls_engine_join."""
    import torch

    from anothertls_amd import workload

    b = workload.config_batch("c5_mixed_256Ki_x_64B-16KiB", n=3000)
    n = len(b["recs"])
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(5)
    d_in = torch.randint(0, 256, (b["in_bytes"] + 16,), dtype=torch.uint8, device=dev, generator=g)
    d_aux = torch.zeros(16, dtype=torch.uint8, device=dev)
    d_recs = torch.from_numpy(b["recs"].view(np.uint8).copy()).to(dev)
    ref = atls.Engine(0)
    ref.set_keys(b["keys"])
    r_out = torch.zeros(b["out_bytes"] + 16, dtype=torch.uint8, device=dev)
    r_tags = torch.zeros(16 * n, dtype=torch.uint8, device=dev)
    ref.seal_batch(d_recs.data_ptr(), d_in, d_aux, r_out, r_tags, flags=atls.FLAG_DEVICE_PTRS | atls.FLAG_DEVICE_RECS, n=n)
    eng = atls.Engine(0)
    eng.set_keys(b["keys"])
    torch.cuda.synchronize()
    lazy = atls.FLAG_DEVICE_PTRS | atls.FLAG_DEVICE_RECS | atls.FLAG_NO_SYNC | atls.FLAG_LAZY_JOIN
    outs = [torch.zeros_like(r_out) for _ in range(5)]
    tags = [torch.zeros_like(r_tags) for _ in range(5)]
    for _ in range(3):  # the same buffers again: the sets and the side stream are reused
        for o, t in zip(outs, tags):
            eng.seal_batch(d_recs.data_ptr(), d_in.data_ptr(), d_aux.data_ptr(), o.data_ptr(), t.data_ptr(), flags=lazy, n=n)
    eng.join()
    done = torch.cuda.Event()
    done.record(torch.cuda.ExternalStream(eng.stream, device=dev))
    done.synchronize()  # the engine stream alone now covers every kernel of those batches
    for o, t in zip(outs, tags):
        assert torch.equal(o, r_out) and torch.equal(t, r_tags)
    # a key-table update after lazy batches waits for their side kernels (same keys: same results)
    eng.seal_batch(d_recs.data_ptr(), d_in.data_ptr(), d_aux.data_ptr(), outs[0].data_ptr(), tags[0].data_ptr(),
                   flags=lazy, n=n)
    eng.update_keys(0, b["keys"][:5])
    # open the lazily sealed records, lazily too, then a synchronous batch joins everything
    orecs = b["recs"].copy()
    orecs["in_off"], orecs["len"] = b["recs"]["out_off"], b["recs"]["len"] + 1
    d_orecs = torch.from_numpy(orecs.view(np.uint8).copy()).to(dev)
    d_pt = torch.zeros_like(r_out)
    d_res = torch.zeros(8 * n, dtype=torch.uint8, device=dev)
    eng.open_batch(d_orecs.data_ptr(), outs[0].data_ptr(), d_aux.data_ptr(), tags[0].data_ptr(), d_pt.data_ptr(),
                   d_res.data_ptr(), flags=lazy, n=n)
    eng.seal_batch(d_recs.data_ptr(), d_in, d_aux, outs[1], tags[1], flags=atls.FLAG_DEVICE_PTRS | atls.FLAG_DEVICE_RECS, n=n)
    res = d_res.cpu().numpy().view(atls.OPEN_RESULT_DTYPE)
    assert (res["status"] == 0).all() and (res["content_len"] == b["recs"]["len"]).all()
    assert torch.equal(outs[0], r_out) and torch.equal(outs[1], r_out) and torch.equal(tags[1], r_tags)
    h_in, h_pt = d_in.cpu().numpy(), d_pt.cpu().numpy()
    for i in range(n):
        o, s, L = int(b["recs"]["out_off"][i]), int(b["recs"]["in_off"][i]), int(b["recs"]["len"][i])
        assert h_pt[o:o + L].tobytes() == h_in[s:s + L].tobytes(), i
    eng.close()
    ref.close()


def test_lazy_flag_with_engine_staged_descriptors_and_scratch_tags(atls):
    """LAZY_JOIN with host descriptors (staged into the engine's one descriptor buffer) or
    without a tags array (WIRE records, the engine's scratch tags) must not leave a side kernel reading
    a buffer the next batch rewrites: such batches join like unflagged ones. Batches of different sizes
    back to back, alternating the two records sets, each equal to a synchronous seal."""
    import torch

    from anothertls_amd import workload

    dev = torch.device("cuda", 0)
    full = workload.config_batch("c5_mixed_256Ki_x_64B-16KiB", n=2500)
    eng = atls.Engine(0)
    eng.set_keys(full["keys"])
    g = torch.Generator(device=dev).manual_seed(11)
    d_in = torch.randint(0, 256, (full["in_bytes"] + 16,), dtype=torch.uint8, device=dev, generator=g)
    d_aux = torch.zeros(16, dtype=torch.uint8, device=dev)
    wire = workload.wire_batch(full)
    lazy = atls.FLAG_DEVICE_PTRS | atls.FLAG_NO_SYNC | atls.FLAG_LAZY_JOIN
    cases = []
    for n in (2500, 700, 2500, 1200, 300):
        for kind in ("tls", "wire"):
            recs = (full if kind == "tls" else wire)["recs"][:n].copy()
            out_bytes = (full if kind == "tls" else wire)["out_bytes"] + 64
            out = torch.zeros(out_bytes, dtype=torch.uint8, device=dev)
            tags = torch.zeros(16 * n, dtype=torch.uint8, device=dev) if kind == "tls" else None
            cases.append((recs, out, tags))
    torch.cuda.synchronize()
    for recs, out, tags in cases:  # host descriptors; WIRE batches without a tags array
        eng.seal_batch(recs, d_in.data_ptr(), d_aux.data_ptr(), out.data_ptr(), None if tags is None else tags.data_ptr(),
                       flags=lazy, n=len(recs))
    eng.sync()
    ref = atls.Engine(0)
    ref.set_keys(full["keys"])
    for recs, out, tags in cases:
        r_out = torch.zeros_like(out)
        r_tags = None if tags is None else torch.zeros_like(tags)
        ref.seal_batch(recs, d_in, d_aux, r_out, r_tags, flags=atls.FLAG_DEVICE_PTRS)
        assert torch.equal(out, r_out)
        if tags is not None:
            assert torch.equal(tags, r_tags)
    ref.close()
    eng.close()
