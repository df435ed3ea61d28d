"""Multi-GPU paths of the product on the GPU box (one GPU there, so several ranges share device 0):

* atls_multi_* (MultiEngine): a batch split by cumulative bytes over several engines, scattered,
  sealed / opened and gathered, equals one engine's result byte for byte (bytes between records
  included), for device-resident and host buffers, TLS and WIRE records, and tampered-tag opens.
  With a repeated device the transport is device-to-device copies; distinct GPUs use RCCL. The
  RCCL branch itself runs here too: ATLS_MULTI_RCCL_SELF=1 with device 0 repeated makes a one-rank
  communicator through the product's rccl() loader, and every part's scatter / gather is a grouped
  send / recv of rank 0 to itself (the same run_device code as between distinct GPUs).
  Descriptors the engines would refuse are refused before anything is queued, and leave no
  sticky error behind.
* dist.seal_sharded with the real engine in two ranks (gloo, both on device 0): the batch at
  rank 0 is scattered, each rank's engine seals its range, and the gathered result equals the
  unsharded batch.
Reference: records are independent because nonce = static_iv ^ seq (net/key_schedule.rs:51-64)."""
import os
import socket
import sys

import numpy as np
import pytest

import anothertls_amd as atls
from anothertls_amd import workload

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _batch(n=3000):
    b = workload.config_batch("c5_mixed_256Ki_x_64B-16KiB", n=n)
    inbuf = np.random.default_rng(3).integers(0, 256, b["in_bytes"] + 16, dtype=np.uint8)
    return b, inbuf


def _single_seal(b, inbuf, recs=None, out_bytes=None):
    recs = b["recs"] if recs is None else recs
    e = atls.Engine(0)
    e.set_keys(b["keys"])
    out = np.full((out_bytes or b["out_bytes"]) + 16, 0x5A, np.uint8)
    tags = np.zeros(16 * len(recs), np.uint8)
    e.seal_batch(recs, inbuf, np.zeros(16, np.uint8), out, tags)
    e.close()
    return out, tags


@pytest.mark.parametrize("devices,rccl_self,chunk_mb", [([0], False, None), ([0, 0], False, None), ([0, 0, 0], False, None),
                                                        ([0, 0], True, None), ([0, 0, 0, 0], True, None),
                                                        ([0, 0, 0], True, "1")],
                         ids=["1-copy", "2-copy", "3-copy", "2-rccl-self", "4-rccl-self", "3-rccl-self-1MiB-pieces"])
def test_multi_engine_device_buffers_equal_single_engine(devices, rccl_self, chunk_mb, monkeypatch):
    """...; with ATLS_MULTI_CHUNK_MB=1 every range travels in several RCCL messages (the 1 GiB cap of
    csrc/multi.cpp scaled down), matched in order on both sides."""
    b, inbuf = _batch()
    ref_out, ref_tags = _single_seal(b, inbuf)
    if rccl_self:
        monkeypatch.setenv("ATLS_MULTI_RCCL_SELF", "1")
    if chunk_mb:
        monkeypatch.setenv("ATLS_MULTI_CHUNK_MB", chunk_mb)
    m = atls.MultiEngine(devices)
    assert m.uses_rccl == rccl_self  # repeated device: copies, or RCCL rank 0 to itself
    m.set_keys(b["keys"])
    dev = torch.device("cuda", 0)
    d_in = torch.from_numpy(inbuf).to(dev)
    d_out = torch.full((b["out_bytes"] + 16,), 0x5A, dtype=torch.uint8, device=dev)
    d_tags = torch.zeros(16 * len(b["recs"]), dtype=torch.uint8, device=dev)
    d_aux = torch.zeros(16, dtype=torch.uint8, device=dev)
    m.seal_batch(b["recs"], d_in, d_aux, d_out, d_tags, flags=atls.FLAG_DEVICE_PTRS)
    assert np.array_equal(d_tags.cpu().numpy(), ref_tags)
    assert np.array_equal(d_out.cpu().numpy(), ref_out)
    # open through the multi engine, with a few tampered tags
    recs = b["recs"]
    orecs = recs.copy()
    orecs["in_off"] = recs["out_off"]
    orecs["len"] = recs["len"] + 1
    bad = [5, 1500, 2999]
    d_tags[torch.tensor(bad) * 16] ^= 1
    d_back = torch.zeros_like(d_out)
    d_res = torch.zeros(8 * len(recs), dtype=torch.uint8, device=dev)
    m.open_batch(orecs, d_out, d_aux, d_tags, d_back, d_res, flags=atls.FLAG_DEVICE_PTRS)
    res = d_res.cpu().numpy().view(atls.OPEN_RESULT_DTYPE)
    mask = np.zeros(len(recs), bool)
    mask[bad] = True
    assert (res["status"][mask] == 50).all() and (res["status"][~mask] == 0).all()
    assert (res["content_len"][~mask] == recs["len"][~mask]).all()
    back = d_back.cpu().numpy()
    for i in np.flatnonzero(~mask)[::97]:
        o, s, L = int(recs[i]["out_off"]), int(recs[i]["in_off"]), int(recs[i]["len"])
        assert back[o:o + L].tobytes() == inbuf[s:s + L].tobytes()
    m.close()


def test_multi_engine_host_buffers_and_wire_records():
    b, inbuf = _batch(1200)
    wb = workload.wire_batch(b)
    ref_out, ref_tags = _single_seal(b, inbuf, wb["recs"], wb["out_bytes"])
    m = atls.MultiEngine([0, 0, 0, 0])
    m.set_keys(b["keys"])
    out = np.full(wb["out_bytes"] + 16, 0x5A, np.uint8)
    tags = np.zeros(16 * len(b["recs"]), np.uint8)
    m.seal_batch(wb["recs"], inbuf, np.zeros(16, np.uint8), out, tags)  # host memory: each part stages its range
    assert np.array_equal(tags, ref_tags) and np.array_equal(out, ref_out)
    # interleaved ranges are refused (the split needs offsets increasing with the index)
    r2 = b["recs"][::-1].copy()
    with pytest.raises(atls.TlsError) as e:
        m.seal_batch(r2, inbuf, np.zeros(16, np.uint8), out, tags)
    assert e.value.code == 47
    m.close()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, world, port, q):
    sys.path.insert(0, ROOT)
    os.environ.update(RANK=str(rank), LOCAL_RANK="0", WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    import torch as t

    import anothertls_amd as a
    from anothertls_amd import dist

    assert dist.init("gloo")
    b, inbuf = _batch(2000)
    eng = a.Engine(0)
    eng.set_keys(b["keys"])

    def seal(recs, inp, out, tags):  # host tensors (gloo): the engine stages them over PCIe
        eng.seal_batch(recs, inp.numpy(), np.zeros(16, np.uint8), out.numpy(), tags.numpy())

    inp = out = tags = None
    if rank == 0:
        inp = t.from_numpy(inbuf)
        out = t.full((b["out_bytes"] + 16,), 0x5A, dtype=t.uint8)
        tags = t.zeros(16 * len(b["recs"]), dtype=t.uint8)
    rng = dist.seal_sharded(seal, b["recs"], inp, out, tags)
    q.put((rank, rng, (out.numpy().tobytes(), tags.numpy().tobytes()) if rank == 0 else None))
    eng.close()
    dist.close()


@pytest.mark.timeout(300)
def test_two_rank_seal_sharded_with_engine():
    import torch.multiprocessing as mp

    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in procs], key=lambda r: r[0])
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert res[0][1][0] == 0 and res[0][1][1] == res[1][1][0] and res[1][1][1] == 2000
    b, inbuf = _batch(2000)
    ref_out, ref_tags = _single_seal(b, inbuf)
    got_out, got_tags = res[0][2]
    assert got_tags == ref_tags.tobytes()
    assert got_out == ref_out.tobytes()


def test_multi_engine_edge_cases_raw_records_and_wire_open():
    rng = np.random.default_rng(12)
    # RAW records (explicit nonce || AAD in aux) of mixed suites and random lengths
    n = 40
    lens = rng.integers(0, 5000, n).astype(np.uint64)
    b = workload.tls_batch(n, lens, lambda k: np.array([0x1301, 0x1303, 0x1302] * k, np.uint16)[:k], n_keys=3)
    recs = b["recs"].copy()
    recs["mode"] = atls.MODE_RAW
    recs["iv_len"] = 12
    recs["aad_len"] = rng.integers(0, 30, n)
    recs["aux_off"] = np.arange(n, dtype=np.uint64) * 64
    aux = rng.integers(0, 256, 64 * n + 16, dtype=np.uint8)
    inbuf = rng.integers(0, 256, b["in_bytes"] + 16, dtype=np.uint8)
    e = atls.Engine(0)
    e.set_keys(b["keys"])
    ref_out = np.zeros(b["out_bytes"] + 16, np.uint8)
    ref_tags = np.zeros(16 * n, np.uint8)
    e.seal_batch(recs, inbuf, aux, ref_out, ref_tags)
    m = atls.MultiEngine([0, 0, 0])
    m.set_keys(b["keys"])
    dev = torch.device("cuda", 0)
    d_in, d_aux = torch.from_numpy(inbuf).to(dev), torch.from_numpy(aux).to(dev)
    d_out = torch.zeros(b["out_bytes"] + 16, dtype=torch.uint8, device=dev)
    d_tags = torch.zeros(16 * n, dtype=torch.uint8, device=dev)
    m.seal_batch(recs, d_in, d_aux, d_out, d_tags, flags=atls.FLAG_DEVICE_PTRS)
    assert np.array_equal(d_tags.cpu().numpy(), ref_tags) and np.array_equal(d_out.cpu().numpy(), ref_out)
    m.close()
    # more parts than records: empty parts are skipped
    m = atls.MultiEngine([0] * 5)
    m.set_keys(b["keys"])
    few = b["recs"][:3]
    out = np.zeros(b["out_bytes"] + 16, np.uint8)
    tags = np.zeros(48, np.uint8)
    m.seal_batch(few, inbuf, np.zeros(16, np.uint8), out, tags)
    o2, t2 = np.zeros_like(out), np.zeros_like(tags)
    e.seal_batch(few, inbuf, np.zeros(16, np.uint8), o2, t2)
    assert np.array_equal(out, o2) and np.array_equal(tags, t2)
    # WIRE records: seal through one engine, open through the multi engine (device buffers)
    wb = workload.wire_batch(b)
    wire = np.zeros(wb["out_bytes"] + 16, np.uint8)
    e.seal_batch(wb["recs"], inbuf, np.zeros(16, np.uint8), wire, np.zeros(16 * n, np.uint8))
    orecs, pt_bytes = workload.wire_open_descs(wb["recs"])
    d_wire = torch.from_numpy(wire).to(dev)
    d_pt = torch.zeros(pt_bytes + 16, dtype=torch.uint8, device=dev)
    d_res = torch.zeros(8 * n, dtype=torch.uint8, device=dev)
    m.open_batch(orecs, d_wire, torch.zeros(16, dtype=torch.uint8, device=dev), None, d_pt, d_res,
                 flags=atls.FLAG_DEVICE_PTRS)
    res = d_res.cpu().numpy().view(atls.OPEN_RESULT_DTYPE)
    assert (res["status"] == 0).all() and (res["content_len"] == lens).all()
    pt = d_pt.cpu().numpy()
    for i in range(n):
        o, s, L = int(orecs[i]["out_off"]), int(b["recs"][i]["in_off"]), int(lens[i])
        assert pt[o:o + L].tobytes() == inbuf[s:s + L].tobytes(), i
    m.close()
    e.close()


@pytest.mark.parametrize("rccl_self", [False, True])
def test_multi_engine_refuses_before_queueing(rccl_self, monkeypatch):
    """A descriptor the engines would refuse (key slot past the table, unknown mode, no tag array
    for a non-WIRE record) fails the whole batch with ILLEGAL_PARAMETER before anything is queued:
    the caller's output is untouched, and the next good batch reports no stale error."""
    if rccl_self:
        monkeypatch.setenv("ATLS_MULTI_RCCL_SELF", "1")
    b, inbuf = _batch(600)
    m = atls.MultiEngine([0, 0, 0])
    m.set_keys(b["keys"])
    dev = torch.device("cuda", 0)
    d_in = torch.from_numpy(inbuf).to(dev)
    d_aux = torch.zeros(16, dtype=torch.uint8, device=dev)
    d_tags = torch.zeros(16 * len(b["recs"]), dtype=torch.uint8, device=dev)
    for field, value in (("key_slot", len(b["keys"])), ("mode", 7)):
        bad = b["recs"].copy()
        bad[550][field] = value  # in the last part's range
        d_out = torch.full((b["out_bytes"] + 16,), 0x5A, dtype=torch.uint8, device=dev)
        with pytest.raises(atls.TlsError) as e:
            m.seal_batch(bad, d_in, d_aux, d_out, d_tags, flags=atls.FLAG_DEVICE_PTRS)
        assert e.value.code == 47
        assert bool((d_out == 0x5A).all())  # nothing ran
    with pytest.raises(atls.TlsError) as e:  # TLS records need a tag array
        m.seal_batch(b["recs"], d_in, d_aux, d_out, None, flags=atls.FLAG_DEVICE_PTRS)
    assert e.value.code == 47
    ref_out, ref_tags = _single_seal(b, inbuf)
    d_out = torch.full((b["out_bytes"] + 16,), 0x5A, dtype=torch.uint8, device=dev)
    m.seal_batch(b["recs"], d_in, d_aux, d_out, d_tags, flags=atls.FLAG_DEVICE_PTRS)  # no stale error
    assert np.array_equal(d_out.cpu().numpy(), ref_out) and np.array_equal(d_tags.cpu().numpy(), ref_tags)
    m.close()


@pytest.mark.parametrize("per_part", [65535, 65536, 65537], ids=["under", "at", "over"])
def test_rccl_message_cap_boundary(per_part, monkeypatch):
    """The RCCL message cap at its real size: two parts in RCCL-self mode, part 1's range of
    `per_part` 16 KiB records -- 2^30 - 16 KiB, exactly 2^30 and 2^30 + 16 KiB of input (one, one and two
    messages), and 16,400-B output slots (just over 2^30 each time: two messages) -- sealed and opened,
    equal to one engine byte for byte; the loaded RCCL's version and the 1 GiB cap are reported."""
    monkeypatch.setenv("ATLS_MULTI_RCCL_SELF", "1")
    monkeypatch.delenv("ATLS_MULTI_CHUNK_MB", raising=False)
    n = 2 * per_part
    b = workload.config_batch("c2_aes128gcm_64Ki_x_16KiB", n=n, n_keys=64)
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(7)
    d_in = torch.randint(0, 256, (b["in_bytes"] + 16,), dtype=torch.uint8, device=dev, generator=g)
    d_aux = torch.zeros(16, dtype=torch.uint8, device=dev)
    first = atls.partition(b["recs"], 2)
    assert int(first[1]) == per_part
    e = atls.Engine(0)
    e.set_keys(b["keys"])
    ref_out = torch.zeros(b["out_bytes"] + 16, dtype=torch.uint8, device=dev)
    ref_tags = torch.zeros(16 * n, dtype=torch.uint8, device=dev)
    e.seal_batch(b["recs"], d_in, d_aux, ref_out, ref_tags, flags=atls.FLAG_DEVICE_PTRS)
    e.close()
    m = atls.MultiEngine([0, 0])
    try:
        assert m.uses_rccl and m.rccl_version >= 22600 and m.max_message == 1 << 30
        m.set_keys(b["keys"])
        out = torch.zeros_like(ref_out)
        tags = torch.zeros_like(ref_tags)
        m.seal_batch(b["recs"], d_in, d_aux, out, tags, flags=atls.FLAG_DEVICE_PTRS)
        torch.cuda.synchronize()
        assert torch.equal(tags, ref_tags) and torch.equal(out, ref_out)
        orecs = b["recs"].copy()
        orecs["in_off"], orecs["len"] = b["recs"]["out_off"], b["recs"]["len"] + 1
        pt = torch.zeros_like(out)
        res = torch.zeros(8 * n, dtype=torch.uint8, device=dev)
        m.open_batch(orecs, out, d_aux, tags, pt, res, flags=atls.FLAG_DEVICE_PTRS)
        torch.cuda.synchronize()
        r = res.cpu().numpy().view(atls.OPEN_RESULT_DTYPE)
        assert (r["status"] == 0).all() and (r["content_len"] == 16384).all()
        assert torch.equal(pt[: n * 16400].view(n, 16400)[:, :16384], d_in[: n * 16384].view(n, 16384))
    finally:
        m.close()
        del d_in, ref_out
        torch.cuda.empty_cache()
