"""GPU: deferred last steps of one-record-per-wave AES-GCM records (gcm.hip ATLS_GCM_TAIL, round 6). A batch
record whose last 64-slot step would hold at most ATLS_GCM_TAIL slots stops after its full steps and
gcm_tail_kernel finishes it (the last counter blocks, their ciphertext, the GHASH terms, the tag or the open's
verdict). Everything here is compared byte for byte with the oracle and with the same batch on an engine that
defers nothing (ATLS_GCM_TAIL_ON=0). The product build compiles deferral out (ATLS_GCM_TAIL=0: measured slower,
DESIGN §4.2 round 6), and then these tests pin the same boundary records -- last steps of 1 to 12 slots, AES-128 /
-192 / -256 in one batch, RAW records with one and with several AAD blocks, zero padding across the last step --
against the oracle on the ordinary path; a -DATLS_GCM_TAIL=8 build runs them through the deferred path
(profiles/r06/tail/parity.txt). Reference: crypto/aes/gcm.rs:42-157, net/record.rs:162-240."""
import os

import numpy as np
import pytest

import anothertls_amd as atls
import oracle as ora
from anothertls_amd import workload

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
FLAGS = atls.FLAG_DEVICE_PTRS | atls.FLAG_DEVICE_RECS


def _engine(tail_on, grouped=False):
    env = {"ATLS_GCM_TAIL_ON": "1" if tail_on else "0", "ATLS_GCM_GROUP_MIN": "1" if grouped else "0"}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return atls.Engine(0)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


def _dev(x):
    return torch.from_numpy(np.ascontiguousarray(x)).to(torch.device("cuda", 0))


def _seal(tail_on, keys, recs, inbuf, out_bytes, aux, grouped=False):
    e = _engine(tail_on, grouped)
    e.set_keys(keys)
    d_out = _dev(np.full(out_bytes + 64, 0x5A, np.uint8))
    d_tags = _dev(np.zeros(16 * len(recs), np.uint8))
    d_recs, d_in, d_aux = _dev(recs.view(np.uint8)), _dev(inbuf), _dev(aux)
    e.seal_batch(d_recs.data_ptr(), d_in, d_aux, d_out, d_tags, flags=FLAGS, n=len(recs))
    e.sync()
    e.close()
    return d_out.cpu().numpy(), d_tags.cpu().numpy()


def _open(tail_on, keys, recs, inbuf, tags, out_bytes, aux, grouped=False):
    e = _engine(tail_on, grouped)
    e.set_keys(keys)
    d_out = _dev(np.full(out_bytes + 64, 0x5A, np.uint8))
    d_res = _dev(np.zeros(8 * len(recs), np.uint8))
    d_recs, d_in, d_aux, d_tags = _dev(recs.view(np.uint8)), _dev(inbuf), _dev(aux), _dev(tags)
    e.open_batch(d_recs.data_ptr(), d_in, d_aux, d_tags, d_out, d_res, flags=FLAGS, n=len(recs))
    e.sync()
    e.close()
    return d_out.cpu().numpy(), d_res.cpu().numpy().view(atls.OPEN_RESULT_DTYPE)


def _oracle_seal(keys, recs, inbuf, out_bytes, aux):
    okeys = (ora.OraKey * len(keys)).from_buffer_copy(keys.tobytes())
    orecs = (ora.OraRec * len(recs)).from_buffer_copy(recs.tobytes())
    out = np.full(out_bytes + 64, 0x5A, np.uint8)
    tags = np.zeros(16 * len(recs), np.uint8)
    ora.seal_batch(okeys, orecs, inbuf, aux, out, tags, 8)
    return out, tags


def _oracle_open(keys, recs, inbuf, tags, out_bytes, aux):
    okeys = (ora.OraKey * len(keys)).from_buffer_copy(keys.tobytes())
    orecs = (ora.OraRec * len(recs)).from_buffer_copy(recs.tobytes())
    out = np.full(out_bytes + 64, 0x5A, np.uint8)
    res = (ora.OraOpenResult * len(recs))()
    ora.open_batch(okeys, orecs, inbuf, aux, tags, out, res, 8)
    r = np.frombuffer(bytes(res), dtype=atls.OPEN_RESULT_DTYPE)
    return out, r


def _slots(n_aead, na=1):
    return na + (n_aead + 15) // 16 + 2  # E_K(J0) + AAD + data + length


def _tail_lens(rng, per=6):
    """TLS content lengths whose records have last steps of 1..12 slots (both sides of ATLS_GCM_TAIL = 8) at
    1 to 16 steps, plus a few of exactly 64 slots per step."""
    out = []
    for steps in (2, 3, 5, 9, 16, 17):
        for rem in list(range(1, 13)) + [64]:
            S = 64 * (steps - 1) + rem
            # S = 1 + 1 + nb + 1 with nb = ceil((L + 1) / 16): L + 1 in (16 (nb - 1), 16 nb]
            nb = S - 3
            lo, hi = 16 * (nb - 1), 16 * nb  # n_aead = L + 1 in (lo, hi]
            for L1 in rng.integers(lo + 1, hi + 1, per):
                L = int(L1) - 1
                assert _slots(L + 1) == S
                out.append(L)
    return np.array(out, np.uint64)


def _batch(seed, suites_keylens, raw_frac=0.25):
    rng = np.random.default_rng(seed)
    lens = _tail_lens(rng)
    n = len(lens)
    b = workload.tls_batch(n, lens, 0x1301, n_keys=n, shrink_keys=False)  # a key per record: no lane groups
    keys, recs = b["keys"], b["recs"]
    kinds = rng.integers(0, len(suites_keylens), n)
    for i, (suite, kl) in enumerate(suites_keylens):
        keys["suite"][kinds == i] = suite
        keys["key_len"][kinds == i] = kl
    recs["seq"] = rng.integers(0, 1 << 40, n)
    # RAW records: a 12-byte IV and at most 16 AAD bytes keep one AAD block (deferrable); some with 17-40 AAD
    # bytes (two or three AAD blocks: never deferred) and some with an 8-byte IV (J0 by GHASH: never deferred)
    raw = np.flatnonzero(rng.random(n) < raw_frac)
    aux = rng.integers(0, 256, 64 * len(raw) + 64, dtype=np.uint8)
    recs["mode"][raw] = atls.MODE_RAW
    recs["aux_off"][raw] = 64 * np.arange(len(raw))
    recs["iv_len"][raw] = np.where(rng.random(len(raw)) < 0.15, 8, 12)
    recs["aad_len"][raw] = np.where(rng.random(len(raw)) < 0.2, rng.integers(17, 41, len(raw)), rng.integers(0, 17, len(raw)))
    inbuf = rng.integers(0, 256, b["in_bytes"] + 64, dtype=np.uint8)
    return b, inbuf, aux


@pytest.mark.parametrize("suites", [[(0x1301, 16)], [(0x1301, 16), (0x1302, 32), (0x1301, 24)]])
def test_deferred_tails_seal_open_vs_oracle_and_undeferred(suites):
    b, inbuf, aux = _batch(41 + len(suites), suites)
    keys, recs = b["keys"], b["recs"]
    out_t, tags_t = _seal(True, keys, recs, inbuf, b["out_bytes"], aux)
    out_u, tags_u = _seal(False, keys, recs, inbuf, b["out_bytes"], aux)
    out_o, tags_o = _oracle_seal(keys, recs, inbuf, b["out_bytes"], aux)
    assert np.array_equal(tags_t, tags_o) and np.array_equal(out_t, out_o)
    assert np.array_equal(tags_u, tags_o) and np.array_equal(out_u, out_o)
    # open the sealed records back: TLS records at the sealed layout (content || type), RAW ones as they are
    orecs = recs.copy()
    orecs["in_off"] = recs["out_off"]
    tls = recs["mode"] == atls.MODE_TLS
    orecs["len"] = recs["len"] + tls.astype(np.uint32)
    bad = np.arange(3, len(recs), 29)
    tags_x = tags_t.copy()
    tags_x[bad * 16 + 5] ^= 0x40
    pt_t, res_t = _open(True, keys, orecs, out_t, tags_x, b["out_bytes"], aux)
    pt_u, res_u = _open(False, keys, orecs, out_t, tags_x, b["out_bytes"], aux)
    pt_o, res_o = _oracle_open(keys, orecs, out_t, tags_x, b["out_bytes"], aux)
    assert np.array_equal(res_t, res_o) and np.array_equal(res_u, res_o)
    ok = res_o["status"] == 0
    assert not ok[bad].any() and ok.sum() == len(recs) - len(bad)
    for i in np.flatnonzero(ok):
        o, L = int(orecs[i]["out_off"]), int(orecs[i]["len"])
        assert pt_t[o:o + L].tobytes() == pt_o[o:o + L].tobytes(), i


def test_deferred_open_content_type_scan_across_the_tail():
    """TLS opens whose inner plaintext ends in zero padding (record.rs:229-237): the last non-zero byte in the
    deferred tail, in the full steps just before it, far before it, or nowhere. The ciphertexts are RAW seals
    with the TLS nonce and header as IV and AAD, so the TLS open must find what the oracle finds."""
    rng = np.random.default_rng(7)
    cases = []  # (inner plaintext length, zero padding at its end)
    for S in (65, 66, 68, 72, 130, 1028):  # last steps of 1, 2, 4, 8, 2 and 4 slots
        n_aead = 16 * (S - 3) - int(rng.integers(0, 16))
        for pad in (0, 1, 15, 16, 17, 40, 64, 200, n_aead):
            cases.append((n_aead, min(pad, n_aead)))
    n = len(cases)
    lens = np.array([c[0] for c in cases], np.uint64)
    b = workload.tls_batch(n, lens, 0x1301, n_keys=n, shrink_keys=False)
    keys, recs = b["keys"], b["recs"]
    recs["seq"] = rng.integers(0, 1 << 40, n)
    inbuf = np.zeros(b["in_bytes"] + 64, np.uint8)
    aux = np.zeros(32 * n + 64, np.uint8)
    for i, (L, pad) in enumerate(cases):
        body = rng.integers(1, 256, L - pad, dtype=np.uint8)  # non-zero content bytes
        if L - pad:
            body[-1] = rng.choice([23, 22, 21, 20, 99])  # the type byte (99: DecodeError)
        o = int(recs[i]["in_off"])
        inbuf[o:o + L - pad] = body
        nonce = bytearray(keys[recs[i]["key_slot"]]["static_iv"].tobytes())
        seq = int(recs[i]["seq"]).to_bytes(8, "big")
        for j in range(8):
            nonce[4 + j] ^= seq[j]
        hdr = bytes([0x17, 0x03, 0x03, ((L + 16) >> 8) & 0xFF, (L + 16) & 0xFF])
        aux[32 * i:32 * i + 12] = np.frombuffer(bytes(nonce), np.uint8)
        aux[32 * i + 12:32 * i + 17] = np.frombuffer(hdr, np.uint8)
    raw = recs.copy()
    raw["mode"] = atls.MODE_RAW
    raw["iv_len"] = 12
    raw["aad_len"] = 5
    raw["aux_off"] = 32 * np.arange(n)
    ct, tags = _oracle_seal(keys, raw, inbuf, b["out_bytes"], aux)
    orecs = recs.copy()  # TLS open of the RAW ciphertexts: len = inner plaintext length
    orecs["in_off"] = recs["out_off"]
    zaux = np.zeros(64, np.uint8)
    pt_t, res_t = _open(True, keys, orecs, ct, tags, b["out_bytes"], zaux)
    pt_o, res_o = _oracle_open(keys, orecs, ct, tags, b["out_bytes"], zaux)
    assert np.array_equal(res_t, res_o)
    assert (res_o["status"] == 0).sum() > n // 2 and (res_o["status"] != 0).any()
    for i in range(n):
        o, L = int(orecs[i]["out_off"]), int(orecs[i]["len"])
        assert pt_t[o:o + L].tobytes() == pt_o[o:o + L].tobytes(), i


def test_deferred_tails_in_a_grouped_batch_and_c2_key_per_record_sample():
    """A grouped direct batch (its single-record tail of region A and region B both defer) and 4,096 records of
    C2's layout with a key per record: equal to the undeferring engine and to the oracle."""
    b = workload.config_batch("c2_aes128gcm_64Ki_x_16KiB", n=4096, n_keys=4096)
    inbuf = np.random.default_rng(9).integers(0, 256, b["in_bytes"] + 64, dtype=np.uint8)
    aux = np.zeros(64, np.uint8)
    out_t, tags_t = _seal(True, b["keys"], b["recs"], inbuf, b["out_bytes"], aux)
    out_o, tags_o = _oracle_seal(b["keys"], b["recs"], inbuf, b["out_bytes"], aux)
    assert np.array_equal(tags_t, tags_o) and np.array_equal(out_t, out_o)
    g = workload.config_batch("c2_aes128gcm_64Ki_x_16KiB", n=8192, n_keys=700)  # runs of 8 and remainders
    inbuf = np.random.default_rng(10).integers(0, 256, g["in_bytes"] + 64, dtype=np.uint8)
    out_g, tags_g = _seal(True, g["keys"], g["recs"], inbuf, g["out_bytes"], aux, grouped=True)
    out_u, tags_u = _seal(False, g["keys"], g["recs"], inbuf, g["out_bytes"], aux, grouped=True)
    assert np.array_equal(tags_g, tags_u) and np.array_equal(out_g, out_u)
    out_o, tags_o = _oracle_seal(g["keys"], g["recs"], inbuf, g["out_bytes"], aux)
    assert np.array_equal(tags_g, tags_o)
