"""ATLS_MODE_WIRE: record framing fused into the record kernels.

Seal writes RecordPayloadProtection::encrypt's whole output, header || ciphertext || tag
(net/record.rs:162-198); open reads a received wire record, uses its header bytes as the AAD
(record.rs:219, the header Record::from_raw kept, :81-102) and its inline tag. The CPU tests pin
the oracle's batch WIRE mode to its per-record restatement of encrypt/decrypt (ora_record_seal /
ora_record_open); the GPU tests compare the device kernels with the oracle on the same
descriptors, including headers the reference rejects."""
import numpy as np
import pytest

import oracle as ora

SUITES = (0x1301, 0x1302, 0x1303)
LENS = np.array([0, 1, 15, 16, 17, 62, 63, 64, 65, 127, 1000, 1536, 4095, 16383, 16384], np.uint64)


def _batch(suite, lens=LENS, n_keys=3):
    from anothertls_amd import workload

    b = workload.tls_batch(len(lens), lens, suite, n_keys=n_keys)
    return workload.wire_batch(b)


def _mixed(lens):
    from anothertls_amd import workload

    b = workload.tls_batch(len(lens), lens, lambda k: np.array([SUITES[i % 3] for i in range(k)], np.uint16),
                           n_keys=6)
    return workload.wire_batch(b)


def _okeys(keys):
    return (ora.OraKey * len(keys)).from_buffer_copy(keys.tobytes())


def _orecs(recs):
    return (ora.OraRec * len(recs)).from_buffer_copy(recs.tobytes())


def _oracle_seal(b, inbuf):
    out = np.zeros(b["out_bytes"] + 16, np.uint8)
    tags = np.zeros(16 * len(b["recs"]), np.uint8)
    assert ora.seal_batch(_okeys(b["keys"]), _orecs(b["recs"]), inbuf, np.zeros(16, np.uint8), out, tags, 4) == 0
    return out, tags


def _oracle_open(keys, recs, wire, out_bytes):
    out = np.zeros(out_bytes + 16, np.uint8)
    res = (ora.OraOpenResult * len(recs))()
    tags = np.zeros(16 * len(recs), np.uint8)  # not read in WIRE mode
    assert ora.open_batch(_okeys(keys), _orecs(recs), wire, np.zeros(16, np.uint8), tags, out, res, 4) == 0
    return out, np.frombuffer(bytes(res), dtype=np.dtype([("content_len", "<u4"), ("status", "u1"),
                                                           ("content_type", "u1"), ("reserved", "u1", 2)]))


def _tamper(wire, recs):
    """Damaged copies of a wire stream, with the status the reference gives each record."""
    w = wire.copy()
    want = np.zeros(len(recs), np.uint8)
    offs = recs["in_off"].astype(np.int64)
    for i in range(len(recs)):
        o = int(offs[i])
        kind = i % 5
        if kind == 1:  # not a RecordType: from_raw -> DecodeError (record.rs:84)
            w[o] = 24
            want[i] = 51
        elif kind == 2:  # version byte: still a record, but the AAD differs -> DecryptError
            w[o + 1] ^= 1
            want[i] = 50
        elif kind == 3:  # tag byte -> DecryptError (record.rs:222)
            w[o + 5 + int(recs["len"][i]) + 3] ^= 0x80
            want[i] = 50
        elif kind == 4:  # length field does not frame this record
            w[o + 4] ^= 1
            want[i] = 51
    return w, want


def test_oracle_wire_mode_matches_record_functions():
    for suite in SUITES:
        b = _batch(suite)
        inbuf = np.random.default_rng(suite).integers(0, 256, b["in_bytes"] + 16, dtype=np.uint8)
        out, tags = _oracle_seal(b, inbuf)
        want = b""
        for i, r in enumerate(b["recs"]):
            k = b["keys"][int(r["key_slot"])]
            frag = inbuf[int(r["in_off"]):int(r["in_off"]) + int(r["len"])].tobytes()
            rc, w = ora.record_seal(suite, bytes(k["key"][:int(k["key_len"])]), bytes(k["static_iv"]), int(r["seq"]),
                                    23, frag)
            assert rc == 0
            assert tags[16 * i:16 * i + 16].tobytes() == w[-16:]
            want += w
        assert out[:b["out_bytes"]].tobytes() == want
        from anothertls_amd import workload

        orecs, ob = workload.wire_open_descs(b["recs"])
        pt, res = _oracle_open(b["keys"], orecs, out, ob)
        assert (res["status"] == 0).all() and (res["content_len"] == b["recs"]["len"]).all()
        assert (res["content_type"] == 23).all()
        for i, r in enumerate(b["recs"]):
            o, L = int(orecs["out_off"][i]), int(r["len"])
            assert np.array_equal(pt[o:o + L], inbuf[int(r["in_off"]):int(r["in_off"]) + L])
        bad, want_st = _tamper(out, orecs)
        _, res = _oracle_open(b["keys"], orecs, bad, ob)
        assert np.array_equal(res["status"], want_st)
        for i in range(len(orecs)):  # the per-record restatement agrees record by record
            if i % 5 == 4:  # header length vs descriptor: the batch API's own framing check
                continue
            k = b["keys"][int(orecs["key_slot"][i])]
            o = int(orecs["in_off"][i])
            rc = ora.record_open(suite, bytes(k["key"][:int(k["key_len"])]), bytes(k["static_iv"]),
                                 int(orecs["seq"][i]), bad[o:o + 21 + int(orecs["len"][i])].tobytes())[0]
            assert rc == want_st[i], i


# ---------------------------------------------------------------------------- GPU parity ----
@pytest.fixture(scope="module")
def atls():
    import anothertls_amd as a

    if not a.device_available():
        pytest.skip("no HIP device")
    return a


def _gpu_roundtrip(atls, b, seed, device):
    import torch

    from anothertls_amd import workload

    rng = np.random.default_rng(seed)
    n = len(b["recs"])
    inbuf = rng.integers(0, 256, b["in_bytes"] + 16, dtype=np.uint8)
    want, _ = _oracle_seal(b, inbuf)
    eng = atls.Engine(0)
    eng.set_keys(b["keys"])
    orecs, ob = workload.wire_open_descs(b["recs"])
    if device:
        dev = torch.device("cuda", 0)
        d_in = torch.from_numpy(inbuf).to(dev)
        d_out = torch.zeros(b["out_bytes"] + 16, dtype=torch.uint8, device=dev)
        eng.seal_batch(b["recs"], d_in, torch.zeros(16, dtype=torch.uint8, device=dev), d_out, None,
                       flags=atls.FLAG_DEVICE_PTRS)
        out = d_out.cpu().numpy()
    else:
        out = np.zeros(b["out_bytes"] + 16, np.uint8)
        eng.seal_batch(b["recs"], inbuf, np.zeros(16, np.uint8), out, None)
    assert np.array_equal(out, want)
    bad, want_st = _tamper(out, orecs)
    for wire, st in ((out, np.zeros(n, np.uint8)), (bad, want_st)):
        ref_pt, ref_res = _oracle_open(b["keys"], orecs, wire, ob)
        res = np.zeros(n, atls.OPEN_RESULT_DTYPE)
        if device:
            d_w = torch.from_numpy(wire.copy()).to(dev)
            d_pt = torch.zeros(ob + 16, dtype=torch.uint8, device=dev)
            d_res = torch.zeros(8 * n, dtype=torch.uint8, device=dev)
            eng.open_batch(orecs, d_w, torch.zeros(16, dtype=torch.uint8, device=dev), None, d_pt, d_res,
                           flags=atls.FLAG_DEVICE_PTRS)
            pt = d_pt.cpu().numpy()
            res = d_res.cpu().numpy().view(atls.OPEN_RESULT_DTYPE)
        else:
            pt = np.zeros(ob + 16, np.uint8)
            eng.open_batch(orecs, wire, np.zeros(16, np.uint8), None, pt, res)
        assert np.array_equal(res["status"], st)
        assert np.array_equal(res["status"], ref_res["status"])
        ok = res["status"] == 0
        assert np.array_equal(res["content_len"][ok], ref_res["content_len"][ok])
        assert np.array_equal(res["content_type"][ok], ref_res["content_type"][ok])
        for i in np.nonzero(ok)[0]:
            o, L = int(orecs["out_off"][i]), int(res["content_len"][i])
            assert np.array_equal(pt[o:o + L], ref_pt[o:o + L]), i
    eng.close()


@pytest.mark.gpu
@pytest.mark.parametrize("suite", SUITES)
@pytest.mark.parametrize("device", [True, False], ids=["device", "host"])
def test_gpu_wire_single_suite(atls, suite, device):
    _gpu_roundtrip(atls, _batch(suite), suite, device)


@pytest.mark.gpu
@pytest.mark.parametrize("device", [True, False], ids=["device", "host"])
def test_gpu_wire_mixed_planned(atls, device):
    lens = np.random.default_rng(11).integers(0, 16385, 300).astype(np.uint64)
    _gpu_roundtrip(atls, _mixed(lens), 12, device)


@pytest.mark.gpu
def test_gpu_wire_large_host_pipeline(atls):
    # ~64 MiB wire stream: several 32 MiB chunks of the host pipeline, unaligned records
    lens = np.random.default_rng(13).integers(8000, 16385, 5000).astype(np.uint64)
    _gpu_roundtrip(atls, _batch(0x1301, lens, n_keys=64), 14, False)


@pytest.mark.gpu
def test_wire_requires_tags_for_other_modes():
    """Without a tags array every record must be WIRE (checked on the host before any launch)."""
    import anothertls_amd as a
    from anothertls_amd import workload

    if not a.device_available():
        pytest.skip("no HIP device")  # the engine needs a device; covered by the GPU run
    b = workload.tls_batch(2, 100, 0x1301, n_keys=1)
    eng = a.Engine(0)
    eng.set_keys(b["keys"])
    with pytest.raises(a.TlsError):
        eng.seal_batch(b["recs"], np.zeros(256, np.uint8), np.zeros(16, np.uint8), np.zeros(256, np.uint8), None)
    eng.close()
