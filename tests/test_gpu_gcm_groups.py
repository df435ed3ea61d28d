"""GPU: key-grouped direct AES-GCM batches. A direct batch's records are counting-sorted by key
slot (plan.hip atls_launch_group): whole runs of 8 records of one key first, the rest after. Runs
whose records share a step count are sealed / opened by one wavefront in lane groups (gcm.hip
gcm_group); everything else (a key's remainder, unequal lengths, RAW records, refused
descriptors, records past the counter cache) takes the one-record-per-wave path. The results must not depend on the grouping: every case is
compared byte for byte with the same batch run ungrouped (ATLS_GCM_GROUP_MIN=0) and with the
oracle. Reference: crypto/aes/gcm.rs:42-128, net/record.rs:162-240."""
import os

import numpy as np
import pytest

import anothertls_amd as atls
import oracle as ora
from anothertls_amd import workload

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
FLAGS = atls.FLAG_DEVICE_PTRS | atls.FLAG_DEVICE_RECS


def _engine(grouped):
    os.environ["ATLS_GCM_GROUP_MIN"] = "1" if grouped else "0"
    try:
        return atls.Engine(0)
    finally:
        del os.environ["ATLS_GCM_GROUP_MIN"]


def _dev(x):
    return torch.from_numpy(np.ascontiguousarray(x)).to(torch.device("cuda", 0))


def _seal(grouped, keys, recs, inbuf, out_bytes, aux=None):
    e = _engine(grouped)
    e.set_keys(keys)
    d_out = _dev(np.full(out_bytes + 64, 0x5A, np.uint8))
    d_tags = _dev(np.zeros(16 * len(recs), np.uint8))
    d_aux = _dev(np.zeros(16, np.uint8) if aux is None else aux)
    d_recs, d_in = _dev(recs.view(np.uint8)), _dev(inbuf)
    err = 0
    try:
        e.seal_batch(d_recs.data_ptr(), d_in, d_aux, d_out, d_tags, flags=FLAGS, n=len(recs))
    except atls.TlsError as exc:
        err = exc.code
    e.sync()
    e.close()
    return d_out.cpu().numpy(), d_tags.cpu().numpy(), err


def _open(grouped, keys, recs, inbuf, tags, out_bytes):
    e = _engine(grouped)
    e.set_keys(keys)
    d_out = _dev(np.full(out_bytes + 64, 0x5A, np.uint8))
    d_res = _dev(np.zeros(8 * len(recs), np.uint8))
    # every device buffer stays referenced until the batch is done (a temporary's memory would go
    # back to torch's allocator and could hold the next tensor while the kernel reads it)
    d_recs, d_in, d_aux = _dev(recs.view(np.uint8)), _dev(inbuf), _dev(np.zeros(16, np.uint8))
    d_tags = None if tags is None else _dev(tags)
    err = 0
    try:
        e.open_batch(d_recs.data_ptr(), d_in, d_aux, d_tags, d_out, d_res, flags=FLAGS, n=len(recs))
    except atls.TlsError as exc:
        err = exc.code
    e.sync()
    e.close()
    return d_out.cpu().numpy(), d_res.cpu().numpy().view(atls.OPEN_RESULT_DTYPE), err


def _oracle_seal(keys, recs, inbuf, out_bytes, aux=None):
    okeys = (ora.OraKey * len(keys)).from_buffer_copy(keys.tobytes())
    orecs = (ora.OraRec * len(recs)).from_buffer_copy(recs.tobytes())
    out = np.full(out_bytes + 64, 0x5A, np.uint8)
    tags = np.zeros(16 * len(recs), np.uint8)
    ora.seal_batch(okeys, orecs, inbuf, np.zeros(16, np.uint8) if aux is None else aux, out, tags, 8)
    return out, tags


def _batch(seed, n, n_keys, suite=0x1301, key_len=None, lens=None):
    """n TLS records over n_keys slots with uneven multiplicities (1..~12 records per key), each
    key's records sharing one content length from a list that covers the lane-group step
    boundaries, plus 10 % of records at a random length (groups that fall back)."""
    rng = np.random.default_rng(seed)
    slot = rng.integers(0, n_keys, n).astype(np.uint32)
    if lens is None:
        choices = np.array([0, 1, 14, 15, 16, 17, 30, 31, 200, 238, 239, 240, 975, 976, 977, 1000, 4095, 4096,
                            8191, 16383, 16384], np.uint64)
        lens = choices[rng.integers(0, len(choices), n_keys)][slot]
        odd = rng.random(n) < 0.10
        lens[odd] = rng.integers(0, 16385, int(odd.sum()))
    b = workload.tls_batch(n, lens, suite, n_keys=n_keys, shrink_keys=False)
    b["recs"]["key_slot"] = slot
    b["recs"]["seq"] = rng.integers(0, 1 << 40, n)
    if key_len is not None:
        b["keys"]["key_len"] = key_len
    inbuf = rng.integers(0, 256, b["in_bytes"] + 64, dtype=np.uint8)
    return b, inbuf


@pytest.mark.parametrize("suite,key_len", [(0x1301, 16), (0x1301, 24), (0x1302, 32)])
def test_grouped_seal_open_equal_ungrouped_and_oracle(suite, key_len):
    b, inbuf = _batch(5 + key_len, 3000, 400, suite, key_len)
    keys, recs = b["keys"], b["recs"]
    out_g, tags_g, err_g = _seal(True, keys, recs, inbuf, b["out_bytes"])
    out_u, tags_u, err_u = _seal(False, keys, recs, inbuf, b["out_bytes"])
    assert err_g == err_u == 0
    assert np.array_equal(tags_g, tags_u) and np.array_equal(out_g, out_u)
    out_o, tags_o = _oracle_seal(keys, recs, inbuf, b["out_bytes"])
    assert np.array_equal(tags_g, tags_o) and np.array_equal(out_g, out_o)
    # open the sealed records (TLS mode), a few tags tampered
    orecs = recs.copy()
    orecs["in_off"] = recs["out_off"]
    orecs["len"] = recs["len"] + 1  # plaintext = content || type byte, at the sealed layout's offsets
    bad = [0, 7, 1234, 2999]
    tags_t = tags_g.copy()
    tags_t[np.array(bad) * 16 + 3] ^= 0x80
    pt_g, res_g, _ = _open(True, keys, orecs, out_g, tags_t, b["out_bytes"])
    pt_u, res_u, _ = _open(False, keys, orecs, out_g, tags_t, b["out_bytes"])
    assert np.array_equal(res_g, res_u) and np.array_equal(pt_g, pt_u)
    mask = np.zeros(len(recs), bool)
    mask[bad] = True
    assert (res_g["status"][mask] == atls.TlsError.DECRYPT_ERROR).all()
    assert (res_g["status"][~mask] == 0).all() and (res_g["content_len"][~mask] == recs["len"][~mask]).all()
    for i in np.flatnonzero(~mask)[::37]:
        o, s, L = int(recs[i]["out_off"]), int(recs[i]["in_off"]), int(recs[i]["len"])
        assert pt_g[o:o + L].tobytes() == inbuf[s:s + L].tobytes(), i


def test_grouped_wire_records_and_bad_headers():
    b, inbuf = _batch(11, 1500, 100)
    wb = workload.wire_batch(b)
    keys = b["keys"]
    wire_g, _, err = _seal(True, keys, wb["recs"], inbuf, wb["out_bytes"])
    wire_u, _, _ = _seal(False, keys, wb["recs"], inbuf, wb["out_bytes"])
    assert err == 0 and np.array_equal(wire_g, wire_u)
    wire_o, _ = _oracle_seal(keys, wb["recs"], inbuf, wb["out_bytes"])
    assert np.array_equal(wire_g, wire_o)
    orecs, pt_bytes = workload.wire_open_descs(wb["recs"])
    wire = wire_g.copy()
    bad_hdr = [3, 700]
    for i in bad_hdr:  # a length byte that does not frame the record: DecodeError (record.rs:81-102)
        wire[int(orecs[i]["in_off"]) + 4] ^= 1
    pt_g, res_g, _ = _open(True, keys, orecs, wire, None, pt_bytes)
    pt_u, res_u, _ = _open(False, keys, orecs, wire, None, pt_bytes)
    assert np.array_equal(res_g, res_u) and np.array_equal(pt_g, pt_u)
    assert (res_g["status"][bad_hdr] == atls.TlsError.DECODE_ERROR).all()
    ok = np.setdiff1d(np.arange(len(orecs)), bad_hdr)
    assert (res_g["status"][ok] == 0).all() and (res_g["content_len"][ok] == b["recs"]["len"][ok]).all()


def test_grouped_batch_with_refused_raw_and_oversized_records():
    """Refused descriptors (key slot out of range, unknown mode), RAW records and records too long
    for a lane group's counter cache sit among groupable ones: the batch reports
    IllegalParameter, and every accepted record equals the ungrouped run and the oracle."""
    n = 800
    lens = np.full(n, 1000, np.uint64)
    lens[100:108] = 66000  # 8 records of one key past the 16-lane counter cache (S > 4096 slots)
    b, inbuf = _batch(21, n, 50, lens=lens)
    recs = b["recs"]
    recs["key_slot"][100:108] = 7
    raw = np.arange(200, 260)
    recs["mode"][raw] = atls.MODE_RAW
    recs["iv_len"][raw] = 12
    recs["aad_len"][raw] = 13
    recs["aux_off"][raw] = np.arange(len(raw)) * 32
    aux = np.random.default_rng(3).integers(0, 256, 32 * len(raw) + 64, dtype=np.uint8)
    refused = [5, 333, 799]
    recs_bad = recs.copy()
    recs_bad["key_slot"][refused[:2]] = 1000
    recs_bad["mode"][refused[2]] = 9
    out_g, tags_g, err_g = _seal(True, b["keys"], recs_bad, inbuf, b["out_bytes"], aux)
    out_u, tags_u, err_u = _seal(False, b["keys"], recs_bad, inbuf, b["out_bytes"], aux)
    assert err_g == err_u == atls.TlsError.ILLEGAL_PARAMETER
    assert np.array_equal(tags_g, tags_u) and np.array_equal(out_g, out_u)
    # the accepted records against the oracle (sealed without the refused ones)
    keep = np.setdiff1d(np.arange(n), refused)
    out_o, tags_o = _oracle_seal(b["keys"], recs[keep], inbuf, b["out_bytes"], aux)
    assert np.array_equal(tags_g.reshape(-1, 16)[keep], tags_o.reshape(-1, 16))
    for i in keep:
        o = int(recs[i]["out_off"])
        L = int(recs[i]["len"]) + (0 if recs[i]["mode"] == atls.MODE_RAW else 1)
        assert out_g[o:o + L].tobytes() == out_o[o:o + L].tobytes(), i


def test_c2_layout_grouped_equals_ungrouped():
    """The C2 key layout (round-robin over 4,096 connections, 16 records per key, all 16 KiB): every
    record goes through a lane group; 8,192 records sealed both ways compare equal."""
    b = workload.config_batch("c2_aes128gcm_64Ki_x_16KiB", n=8192, n_keys=512)
    inbuf = np.random.default_rng(4).integers(0, 256, b["in_bytes"] + 64, dtype=np.uint8)
    out_g, tags_g, _ = _seal(True, b["keys"], b["recs"], inbuf, b["out_bytes"])
    out_u, tags_u, _ = _seal(False, b["keys"], b["recs"], inbuf, b["out_bytes"])
    assert np.array_equal(tags_g, tags_u) and np.array_equal(out_g, out_u)


def test_many_key_slots_both_regions():
    """30,000 key slots (several scan tiles in group_scan), slot k holding k % 11 records of a
    length set per slot: runs of 8 and remainders in both regions; equal to the ungrouped run
    and to the oracle on a sample."""
    n_keys = 30000
    per_key = np.arange(n_keys) % 11
    slot = np.repeat(np.arange(n_keys, dtype=np.uint32), per_key)
    rng = np.random.default_rng(8)
    slot = slot[rng.permutation(len(slot))]
    n = len(slot)
    lens = np.array([64, 100, 1000, 3000], np.uint64)[slot % 4]
    b = workload.tls_batch(n, lens, 0x1301, n_keys=n_keys, shrink_keys=False)
    b["recs"]["key_slot"] = slot
    inbuf = rng.integers(0, 256, b["in_bytes"] + 64, dtype=np.uint8)
    out_g, tags_g, _ = _seal(True, b["keys"], b["recs"], inbuf, b["out_bytes"])
    out_u, tags_u, _ = _seal(False, b["keys"], b["recs"], inbuf, b["out_bytes"])
    assert np.array_equal(tags_g, tags_u) and np.array_equal(out_g, out_u)
    sample = rng.choice(n, 2000, replace=False)
    out_o, tags_o = _oracle_seal(b["keys"], b["recs"][sample], inbuf, b["out_bytes"])
    assert np.array_equal(tags_g.reshape(-1, 16)[sample], tags_o.reshape(-1, 16))
