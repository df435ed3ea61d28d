"""Host record framing (anothertls_amd/record.py) against net/record.rs behaviour and the oracle's
wire records, and the C1 loopback plumbing (tools/c1_loopback.py) on the CPU reference path."""
import os
import sys

import numpy as np
import pytest

import oracle as ora

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _record():
    from anothertls_amd import record

    return record


def test_record_roundtrip_and_quirks():
    record = _record()
    from anothertls_amd import TlsError

    r = record.Record.new(record.RecordType.ApplicationData, b"hello")
    wire = r.as_bytes()
    assert wire == bytes([23, 3, 3, 0, 5]) + b"hello"  # record.rs:103-114
    consumed, back = record.Record.from_raw(wire + b"trailing")
    assert consumed == 10 and back.fragment == b"hello" and back.header == wire[:5] and back.version == 0x0303
    with pytest.raises(TlsError) as e:  # unknown content type: RecordType::new -> DecodeError
        record.Record.from_raw(bytes([24, 3, 3, 0, 0]))
    assert e.value.code == TlsError.DECODE_ERROR
    with pytest.raises(TlsError):  # shorter than a header
        record.Record.from_raw(b"\x17\x03\x03")
    # the reference's bounds check is 2 + len (record.rs:88): 5 + len - 3 bytes pass it and then
    # the reference panics on the slice; the mirror reports DecodeError
    with pytest.raises(TlsError):
        record.Record.from_raw(bytes([23, 3, 3, 0, 8]) + b"12345")


def test_frame_sealed_matches_oracle_wire_records():
    record = _record()
    from anothertls_amd import workload

    rng = np.random.default_rng(3)
    lens = np.array([0, 1, 15, 16, 100, 4096, 16384], np.uint64)
    b = workload.tls_batch(len(lens), lens, 0x1301, n_keys=1)
    inbuf = rng.integers(0, 256, b["in_bytes"] + 16, dtype=np.uint8)
    out = np.zeros(b["out_bytes"] + 16, np.uint8)
    tags = np.zeros(16 * len(lens), np.uint8)
    okeys = (ora.OraKey * 1).from_buffer_copy(b["keys"].tobytes())
    orecs = (ora.OraRec * len(lens)).from_buffer_copy(b["recs"].tobytes())
    assert ora.seal_batch(okeys, orecs, inbuf, np.zeros(16, np.uint8), out, tags, 1) == 0
    wire = record.frame_sealed(b["recs"], out, tags)
    k = b["keys"][0]
    want = b""
    for i, r in enumerate(b["recs"]):
        frag = inbuf[int(r["in_off"]):int(r["in_off"]) + int(r["len"])].tobytes()
        rc, w = ora.record_seal(0x1301, bytes(k["key"][:16]), bytes(k["static_iv"]), int(r["seq"]), 23, frag)
        assert rc == 0
        want += w
    assert wire.tobytes() == want
    offs, flens = record.parse_stream(wire)
    assert list(flens) == [int(x) + 17 for x in lens]
    assert offs[0] == 0 and all(offs[i + 1] == offs[i] + 5 + flens[i] for i in range(len(offs) - 1))


@pytest.mark.timeout(300)
def test_c1_cpu_reference_loop():
    """bench.py's C1 CPU baseline (the oracle per record through the socket loop) round-trips."""
    sys.path.insert(0, ROOT)
    import bench

    body = np.random.default_rng(2).integers(0, 256, 64 * 16384, dtype=np.uint8).tobytes()
    assert bench.c1_cpu_reference(body, 1) > 0


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_c1_loopback_gpu():
    import anothertls_amd as atls

    if not atls.device_available():
        pytest.skip("no HIP device")
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import c1_loopback

    body = np.random.default_rng(1).integers(0, 256, c1_loopback.N_REC * c1_loopback.CONTENT,
                                            dtype=np.uint8).tobytes()
    dt, pt = c1_loopback.run_gpu(body, 2)
    assert pt == body and dt > 0
    dt, pt = c1_loopback.run_gpu(body, 1, conns=4)  # four connections sharing each batch
    assert pt == body and dt > 0
