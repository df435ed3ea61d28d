"""GPU: hybrid direct AES batches (engine.cpp). The first records of the batch
get their AES-CTR keystream from the bitsliced kernel (ks_bs.hip, VALU) while the T-table kernel
seals the rest; a KS launch of the record kernel then seals the first records from the
keystream. Forced on small batches with ATLS_HYBRID / ATLS_HYBRID_MIN (read when an engine is
created) and checked against the oracle: TLS records of every length class, RAW records with
96-bit IVs (keystream) and other IV lengths (T-table fallback inside the KS launch), AES-128 and
AES-256, seal and open (with tampered tags), device and host buffers."""
import os

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


def _engine(atls, f, staged=False):
    """An engine with the hybrid split forced on; staged: host batches go through the one-piece
    staging path (which splits) rather than the chunk pipeline (which does not)."""
    old = {k: os.environ.get(k) for k in ("ATLS_HYBRID", "ATLS_HYBRID_MIN", "ATLS_NO_PIPELINE")}
    os.environ["ATLS_HYBRID"], os.environ["ATLS_HYBRID_MIN"] = str(f), "1"
    os.environ["ATLS_NO_PIPELINE"] = "1" if staged else "0"
    try:
        return atls.Engine(0)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _batch(atls, suite, klen, n, seed):
    from anothertls_amd import workload

    rng = np.random.default_rng(seed)
    keys = workload.make_keys(n, np.full(n, suite, np.uint16), key_lens=np.full(n, klen))
    recs = np.zeros(n, atls.REC_DTYPE)
    aux_parts, aoff, ioff = [], 0, 0
    for i in range(n):
        L = int(rng.choice([0, 1, 15, 16, 17, 1000, 4095, 16383, 16384, int(rng.integers(0, 16385))]))
        r = recs[i:i + 1]
        r["in_off"], r["out_off"], r["len"], r["key_slot"], r["seq"] = ioff, ioff, L, i % 7, i
        r["content_type"] = 23
        kind = i % 5
        if kind < 3:
            r["mode"] = atls.MODE_TLS
        else:  # RAW: 96-bit IV (keystream) or another IV length (T-table fallback)
            ivl = 12 if kind == 3 else int(rng.choice([1, 8, 16, 60]))
            al = int(rng.choice([0, 5, 17]))
            r["mode"], r["iv_len"], r["aad_len"], r["aux_off"] = atls.MODE_RAW, ivl, al, aoff
            aux_parts.append(rng.integers(0, 256, ivl + al, dtype=np.uint8))
            aoff += ivl + al
        ioff += (L + 1 + 15) // 16 * 16
    aux = np.concatenate(aux_parts + [np.zeros(16, np.uint8)])
    inbuf = rng.integers(0, 256, ioff + 16, dtype=np.uint8)
    return keys[:7], recs, aux, inbuf


def _oracle(keys, recs, inbuf, aux):
    okeys = (ora.OraKey * len(keys)).from_buffer_copy(keys.tobytes())
    orecs = (ora.OraRec * len(recs)).from_buffer_copy(recs.tobytes())
    out = np.zeros_like(inbuf)
    tags = np.zeros(16 * len(recs), np.uint8)
    assert ora.seal_batch(okeys, orecs, inbuf, aux, out, tags, 16) == 0
    return out, tags


@pytest.mark.parametrize("suite,klen", [(0x1301, 16), (0x1302, 32)])
@pytest.mark.parametrize("device", [True, False], ids=["device", "host"])
def test_hybrid_seal_open_vs_oracle(atls, suite, klen, device):
    import torch

    keys, recs, aux, inbuf = _batch(atls, suite, klen, 600, klen)
    want_out, want_tags = _oracle(keys, recs, inbuf, aux)
    eng = _engine(atls, 0.5, staged=not device)
    eng.set_keys(keys)
    dev = torch.device("cuda", 0)
    n = len(recs)
    if device:
        t = lambda a: torch.from_numpy(a.copy()).to(dev)  # noqa: E731
        d_in, d_aux, d_out, d_tags = t(inbuf), t(aux), t(np.zeros_like(inbuf)), t(np.zeros(16 * n, np.uint8))
        eng.seal_batch(recs, d_in, d_aux, d_out, d_tags, flags=atls.FLAG_DEVICE_PTRS)
        out, tags = d_out.cpu().numpy(), d_tags.cpu().numpy()
    else:
        out, tags = np.zeros_like(inbuf), np.zeros(16 * n, np.uint8)
        eng.seal_batch(recs, inbuf, aux, out, tags)
    for i in range(n):
        o, L = int(recs[i]["out_off"]), int(recs[i]["len"]) + (1 if recs[i]["mode"] == atls.MODE_TLS else 0)
        assert np.array_equal(out[o:o + L], want_out[o:o + L]), i
        assert np.array_equal(tags[16 * i:16 * i + 16], want_tags[16 * i:16 * i + 16]), i
    # open: TLS records read len + 1 bytes of ciphertext; flip a tag byte on every 9th record
    orecs = recs.copy()
    tls = orecs["mode"] == atls.MODE_TLS
    orecs["len"][tls] += 1
    bad = tags.copy()
    bad[16 * np.arange(0, n, 9)] ^= 1
    res = np.zeros(n, atls.OPEN_RESULT_DTYPE)
    pt = np.zeros_like(inbuf)
    if device:
        d_ct, d_pt = t(out), t(np.zeros_like(inbuf))
        d_res = torch.zeros(8 * n, dtype=torch.uint8, device=dev)
        eng.open_batch(orecs, d_ct, d_aux, t(bad), d_pt, d_res, flags=atls.FLAG_DEVICE_PTRS)
        pt, res = d_pt.cpu().numpy(), d_res.cpu().numpy().view(atls.OPEN_RESULT_DTYPE)
    else:
        eng.open_batch(orecs, out, aux, bad, pt, res)
    for i in range(n):
        tampered = i % 9 == 0
        raw = recs[i]["mode"] == atls.MODE_RAW
        want_st = (20 if raw else 50) if tampered else 0
        assert res[i]["status"] == want_st, i
        if not tampered:
            o, L = int(recs[i]["out_off"]), int(recs[i]["len"])
            assert np.array_equal(pt[o:o + L], inbuf[o:o + L]), i
    eng.close()


def test_hybrid_c2_shape_vs_plain(atls):
    """A C2-shaped batch (16 KiB TLS records, 4096 connections) gives identical bytes with and
    without the hybrid split."""
    import torch

    from anothertls_amd import workload

    b = workload.config_batch("c2_aes128gcm_64Ki_x_16KiB", n=8192)
    dev = torch.device("cuda", 0)
    d_in = torch.randint(0, 256, (b["in_bytes"],), dtype=torch.uint8, device=dev)
    outs = []
    for f in (0.0, 0.4):
        eng = _engine(atls, f)
        eng.set_keys(b["keys"])
        d_out = torch.zeros(b["out_bytes"], dtype=torch.uint8, device=dev)
        d_tags = torch.zeros(16 * len(b["recs"]), dtype=torch.uint8, device=dev)
        eng.seal_batch(b["recs"], d_in, torch.zeros(16, dtype=torch.uint8, device=dev), d_out, d_tags,
                       flags=atls.FLAG_DEVICE_PTRS)
        outs.append((d_out.cpu(), d_tags.cpu()))
        eng.close()
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
