"""GPU parity at the BASELINE configs' full per-GPU sizes (SURVEY §8d "Parity" row), through the
C ABI with device-resident buffers, as the benchmark runs them:

* C3 (ChaCha20-Poly1305, 65,536 x 1.5 KiB) in the bench's one device-resident launch: every record
  against OpenSSL, a 4,096-record sample against the oracle.
* C2 (AES-128-GCM, 65,536 x 16 KiB) and C4 (AES-256-GCM, the 131,072 x 16 KiB shard one GPU holds
  of 1 Mi records): EVERY record's ciphertext and tag against OpenSSL (valid for all 96-bit-IV GCM,
  SURVEY F5), a 4,096-record sample against the oracle, and open(seal(x)) == x on the device.
* C5 (mixed 50/50 AES-128-GCM / ChaCha20-Poly1305, content U{64..16384}, the 32,768-record shard):
  the whole batch against the oracle (including the ChaCha last-block-quirk records,
  chacha20/cipher.rs:99-102), the non-quirk records also against OpenSSL, and open_batch with
  tampered tags (DecryptError exactly there, record.rs:222).
Reference: crypto/aes/gcm.rs:42-128, crypto/chacha20/poly1305.rs:69-104, net/record.rs:162-240."""
import os

import numpy as np
import pytest

import anothertls_amd as atls
import openssl_ref
import oracle as ora
from anothertls_amd import workload

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
NTHREADS = min(16, os.cpu_count() or 1)


@pytest.fixture(scope="module")
def eng():
    e = atls.Engine(int(os.environ.get("ATLS_DEVICE", "0")))
    yield e
    e.close()


def _device_seal(eng, batch, seed):
    """Seal the batch on the device from a seeded device-generated payload; returns the device
    tensors (in, out, tags) and their host copies."""
    dev = torch.device("cuda", eng.device)
    n = len(batch["recs"])
    g = torch.Generator(device=dev).manual_seed(seed)
    d_in = torch.randint(0, 256, (batch["in_bytes"] + 16,), dtype=torch.uint8, device=dev, generator=g)
    d_out = torch.zeros(batch["out_bytes"] + 16, dtype=torch.uint8, device=dev)
    d_tags = torch.zeros(16 * n, dtype=torch.uint8, device=dev)
    d_aux = torch.zeros(16, dtype=torch.uint8, device=dev)
    d_recs = torch.from_numpy(batch["recs"].view(np.uint8).copy()).to(dev)
    eng.set_keys(batch["keys"])
    torch.cuda.synchronize()
    eng.seal_batch(d_recs.data_ptr(), d_in, d_aux, d_out, d_tags,
                   flags=atls.FLAG_DEVICE_PTRS | atls.FLAG_DEVICE_RECS, n=n)
    eng.sync()
    return (d_in, d_out, d_tags, d_aux), (d_in.cpu().numpy(), d_out.cpu().numpy(), d_tags.cpu().numpy())


def _mismatches(recs, out, tags, eout, etags, which=None):
    """Indices of records whose ciphertext (len + 1 B) or tag differ."""
    idx = range(len(recs)) if which is None else which
    bad = []
    for i in idx:
        o, L = int(recs[i]["out_off"]), int(recs[i]["len"]) + 1
        if out[o:o + L].tobytes() != eout[o:o + L].tobytes() or tags[16 * i:16 * i + 16].tobytes() != \
                etags[16 * i:16 * i + 16].tobytes():
            bad.append(i)
    return bad


def _vs_openssl(batch, h_in, h_out, h_tags):
    recs = batch["recs"]
    eout, etags, skipped = openssl_ref.seal_tls_batch(batch["keys"], recs, h_in, batch["out_bytes"] + 16, NTHREADS)
    # whole-buffer compare first (fast), then per record where they differ
    ok_tags = np.array_equal(h_tags.reshape(-1, 16)[~skipped.astype(bool)], etags.reshape(-1, 16)[~skipped.astype(bool)])
    if not skipped.any() and ok_tags and np.array_equal(h_out, eout):
        return 0
    bad = _mismatches(recs, h_out, h_tags, eout, etags, np.flatnonzero(skipped == 0))
    assert not bad, f"{len(bad)} records differ from OpenSSL, first {bad[:5]}"
    return int(skipped.sum())


def _vs_oracle(batch, h_in, h_out, h_tags, sample=None):
    """Oracle seal of records [0, sample) (all if None) compared byte for byte."""
    keys, recs = batch["keys"], batch["recs"]
    sub = recs if sample is None else recs[:sample]
    okeys = (ora.OraKey * len(keys)).from_buffer_copy(keys.tobytes())
    orecs = (ora.OraRec * len(sub)).from_buffer_copy(sub.tobytes())
    oout, otags = np.zeros_like(h_out), np.zeros(16 * len(sub), np.uint8)
    assert ora.seal_batch(okeys, orecs, h_in, np.zeros(16, np.uint8), oout, otags, NTHREADS) == 0
    bad = _mismatches(sub, h_out, h_tags[:16 * len(sub)], oout, otags)
    assert not bad, f"{len(bad)} records differ from the oracle, first {bad[:5]}"


def _open_roundtrip(eng, batch, dev_bufs, tamper=()):
    """Open the sealed records on the device (TLS mode); tampered tags must give DecryptError
    (50) exactly at `tamper`, every other record its content back."""
    d_in, d_out, d_tags, d_aux = dev_bufs
    recs = batch["recs"]
    n = len(recs)
    dev = d_in.device
    orecs = recs.copy()
    orecs["in_off"] = recs["out_off"]
    orecs["len"] = recs["len"] + 1
    if len(tamper):
        t = torch.as_tensor(np.asarray(tamper, np.int64) * 16, device=dev)
        d_tags[t] ^= 0x01
    d_back = torch.zeros_like(d_out)
    d_res = torch.zeros(8 * n, dtype=torch.uint8, device=dev)
    eng.open_batch(orecs, d_out, d_aux, d_tags, d_back, d_res, flags=atls.FLAG_DEVICE_PTRS)
    res = d_res.cpu().numpy().view(atls.OPEN_RESULT_DTYPE)
    bad = np.zeros(n, bool)
    bad[list(tamper)] = True
    assert (res["status"][bad] == atls.TlsError.DECRYPT_ERROR).all()
    assert (res["status"][~bad] == 0).all() and (res["content_len"][~bad] == recs["len"][~bad]).all()
    assert (res["content_type"][~bad] == 23).all()
    # every record's plaintext (the tampered ones are zeroed: no unauthenticated plaintext)
    L0, io, oo = recs["len"], recs["in_off"].astype(np.int64), recs["out_off"].astype(np.int64)
    if (L0 == L0[0]).all() and (np.diff(io) == io[1] - io[0]).all() and (np.diff(oo) == oo[1] - oo[0]).all():
        L, si, so = int(L0[0]), int(io[1] - io[0]), int(oo[1] - oo[0])
        got = d_back[: n * so].view(n, so)[:, :L]
        want = d_in[: n * si].view(n, si)[:, :L]
        same = (got == want).all(dim=1).cpu().numpy()
        assert same[~bad].all(), np.flatnonzero(~same & ~bad)[:5]
    else:
        h_back, h_in = d_back.cpu().numpy(), d_in.cpu().numpy()
        for i in np.flatnonzero(~bad):
            o, s, L = int(oo[i]), int(io[i]), int(L0[i])
            assert h_back[o:o + L].tobytes() == h_in[s:s + L].tobytes(), i
    return res


def _full_config(eng, name, n):
    batch = workload.config_batch(name, n=n)
    dev_bufs, (h_in, h_out, h_tags) = _device_seal(eng, batch, workload.SEEDS["payload"])
    return batch, dev_bufs, h_in, h_out, h_tags


def test_c2_key_per_record_full_batch_vs_openssl_and_oracle(eng):
    """VERDICT r5 parity softness (ii): C2's layout with a key per record (65,536 connections, the bench's
    "a key per record" config and SURVEY §8(d)'s worst case: no lane group forms, every record takes the
    one-record-per-wave path with its own key schedule) -- every record against OpenSSL at full size, a sample
    against the oracle, open(seal(x)) == x with tampered tags (net/record.rs:162-240, crypto/aes/gcm.rs:42-128)."""
    name = "c2_aes128gcm_64Ki_x_16KiB"
    batch = workload.config_batch(name, n_keys=workload.CONFIGS[name][1])
    assert len(batch["recs"]) == 65536 and len(batch["keys"]) == 65536
    dev_bufs, (h_in, h_out, h_tags) = _device_seal(eng, batch, workload.SEEDS["payload"] + 17)
    assert _vs_openssl(batch, h_in, h_out, h_tags) == 0
    _vs_oracle(batch, h_in, h_out, h_tags, sample=2048)
    _open_roundtrip(eng, batch, dev_bufs, tamper=[1, 30000, 65534])


def test_c2_full_batch_vs_openssl_and_oracle(eng):
    batch, dev_bufs, h_in, h_out, h_tags = _full_config(eng, "c2_aes128gcm_64Ki_x_16KiB", None)
    assert len(batch["recs"]) == 65536
    assert _vs_openssl(batch, h_in, h_out, h_tags) == 0
    _vs_oracle(batch, h_in, h_out, h_tags, sample=4096)
    _open_roundtrip(eng, batch, dev_bufs, tamper=[0, 4097, 65535])


def test_c3_full_batch_device_resident_vs_openssl_and_oracle(eng):
    """C3 exactly as the bench runs it: device-resident buffers and descriptors, one launch over
    all 65,536 records (the 2-lane path), every record against OpenSSL (no C3 record hits the F4
    quirk: 1,537 % 64 != 0), a 4,096-record sample against the oracle, open with tampered tags."""
    batch, dev_bufs, h_in, h_out, h_tags = _full_config(eng, "c3_chacha20poly1305_64Ki_x_1.5KiB", None)
    assert len(batch["recs"]) == 65536
    assert _vs_openssl(batch, h_in, h_out, h_tags) == 0
    _vs_oracle(batch, h_in, h_out, h_tags, sample=4096)
    _open_roundtrip(eng, batch, dev_bufs, tamper=[3, 40000, 65535])


def test_c4_shard_full_vs_openssl_and_oracle(eng):
    n = workload.records_per_rank("c4_aes256gcm_1Mi_x_16KiB")
    batch, dev_bufs, h_in, h_out, h_tags = _full_config(eng, "c4_aes256gcm_1Mi_x_16KiB", n)
    assert n == 131072 and (batch["keys"]["key_len"] == 32).all()
    assert _vs_openssl(batch, h_in, h_out, h_tags) == 0
    _vs_oracle(batch, h_in, h_out, h_tags, sample=4096)
    _open_roundtrip(eng, batch, dev_bufs, tamper=[1, 77777, n - 1])


def test_c5_shard_full_vs_oracle_and_openssl(eng):
    n = workload.records_per_rank("c5_mixed_256Ki_x_64B-16KiB")
    batch, dev_bufs, h_in, h_out, h_tags = _full_config(eng, "c5_mixed_256Ki_x_64B-16KiB", n)
    recs, keys = batch["recs"], batch["keys"]
    chacha = keys["suite"][recs["key_slot"]] == 0x1303
    assert n == 32768 and 0.45 < chacha.mean() < 0.55
    quirk_records = _vs_openssl(batch, h_in, h_out, h_tags)
    assert quirk_records == int((chacha & ((recs["len"] + 1) % 64 == 0)).sum()) > 0
    _vs_oracle(batch, h_in, h_out, h_tags)  # every record, quirk records included
    rng = np.random.default_rng(9)
    tamper = sorted(set(rng.integers(0, n, 64).tolist()) | {int(np.flatnonzero(chacha)[0]),
                                                            int(np.flatnonzero(~chacha)[0])})
    _open_roundtrip(eng, batch, dev_bufs, tamper=tamper)
