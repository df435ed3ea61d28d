"""Batched host socket path (anothertls_amd/stream.py): many connections' writes
sealed in one WIRE-mode batch, received byte streams split into records (partial records kept)
and opened in one batch, per-connection sequence numbers, errors per connection.

The CPU tests drive StreamBatch with a test-only engine stub that runs the oracle's batch
functions (same seal_batch/open_batch interface); the GPU test runs the same scenario on the
device engine. Wire bytes are checked against the oracle's per-record restatement of
RecordPayloadProtection::encrypt (net/record.rs:162-198)."""
import socket

import numpy as np
import pytest

import oracle as ora


class OracleEngine:
    """Test stub: the Engine batch interface over the oracle (CPU, test infrastructure only)."""

    def set_keys(self, keys):
        self.keys = keys.copy()
        self._ok = (ora.OraKey * len(keys)).from_buffer_copy(keys.tobytes())

    def seal_batch(self, recs, inp, aux, out, tags, flags=0, n=None):
        t = tags if tags is not None else np.zeros(16 * len(recs), np.uint8)
        orecs = (ora.OraRec * len(recs)).from_buffer_copy(recs.tobytes())
        assert ora.seal_batch(self._ok, orecs, inp, aux, out, t, 2) == 0

    def open_batch(self, recs, inp, aux, tags, out, results, flags=0, n=None):
        t = tags if tags is not None else np.zeros(16 * len(recs), np.uint8)
        orecs = (ora.OraRec * len(recs)).from_buffer_copy(recs.tobytes())
        res = (ora.OraOpenResult * len(recs))()
        assert ora.open_batch(self._ok, orecs, inp, aux, t, out, res, 2) == 0
        results[:] = np.frombuffer(bytes(res), results.dtype)


SUITES = [(0x1301, 16), (0x1302, 32), (0x1303, 32)]


def _keys(i):
    suite, kl = SUITES[i % 3]
    rng = np.random.default_rng(100 + i)
    srv = (suite, rng.integers(0, 256, kl, dtype=np.uint8).tobytes(), rng.integers(0, 256, 12, dtype=np.uint8).tobytes())
    cli = (suite, rng.integers(0, 256, kl, dtype=np.uint8).tobytes(), rng.integers(0, 256, 12, dtype=np.uint8).tobytes())
    return srv, cli


def _pairs(n):
    return [socket.socketpair() for _ in range(n)]


def _scenario(make_engine):
    from anothertls_amd import TlsError, stream
    from anothertls_amd.record import RecordType

    n = 6
    socks = _pairs(n)
    server, client = stream.StreamBatch(make_engine()), stream.StreamBatch(make_engine())
    sc, cc, keys = [], [], []
    for i, (a, b) in enumerate(socks):
        srv, cli = _keys(i)
        keys.append((srv, cli))
        sc.append(server.add_connection(a, srv, cli))
        cc.append(client.add_connection(b, cli, srv))
    rng = np.random.default_rng(7)
    sizes = [0, 1, 15, 16, 4096, 16384, 20000, 100]
    sent = [[] for _ in range(n)]
    for i in range(n):
        for s in sizes[i % 3:]:
            d = rng.integers(0, 256, s, dtype=np.uint8).tobytes()
            server.tls_write(sc[i], d)
            sent[i].append(d)
    assert server.flush() == sum(max(1, -(-len(d) // 16384)) for i in range(n) for d in sent[i])
    # connection 0: the raw wire bytes are the reference's records (one per write <= 2^14)
    raw = b""
    want_len = sum(len(d) + 22 for d in sent[0]) + 22  # the 20000-byte write is two records
    while len(raw) < want_len:
        raw += socks[0][1].recv(1 << 16)
    (suite, key, iv) = keys[0][0]
    pos, seq = 0, 0
    for d in sent[0]:
        frags = [d[j:j + 16384] for j in range(0, len(d), 16384)] or [b""]
        for f in frags:
            rc, w = ora.record_seal(suite, key, iv, seq, 23, f)
            assert rc == 0 and raw[pos:pos + len(w)] == w, (seq, len(f))
            pos += len(w)
            seq += 1
    assert pos == len(raw)
    # feed connection 0 in ragged pieces: partial records stay buffered
    cut = 0
    while cut < len(raw):
        k = int(rng.integers(1, 3000))
        client.feed(cc[0], raw[cut:cut + k])
        cut += k
    for i in range(n):
        got = b""
        want = b"".join(sent[i])
        while len(got) < len(want):
            got += client.tls_read(cc[i])
        assert got == want, i
    # the reverse direction, with a tampered record on connection 1 and a handshake record on 2
    for i in range(n):
        client.tls_write(cc[i], b"ping %d" % i)
    client.write_record(cc[2], RecordType.Handshake, b"\x14\x00\x00\x00")
    client.flush()
    bad = bytearray(socks[1][0].recv(1 << 16))
    bad[10] ^= 1
    server.feed(sc[1], bytes(bad))
    for i in (0, 3, 4, 5):
        assert server.tls_read(sc[i]) == b"ping %d" % i
    with pytest.raises(TlsError) as e:
        server.tls_read(sc[1])
    assert e.value.code == 50  # DecryptError (record.rs:222)
    assert server.tls_read(sc[2]) == b"ping 2"
    with pytest.raises(TlsError) as e:
        server.tls_read(sc[2])
    assert e.value.code == 10  # UnexpectedMessage (stream.rs:112-116)
    for a, b in socks:
        a.close()
        b.close()


def test_stream_batch_oracle_engine():
    _scenario(OracleEngine)


@pytest.mark.gpu
def test_stream_batch_device_engine():
    import anothertls_amd as atls

    if not atls.device_available():
        pytest.skip("no HIP device")
    _scenario(lambda: atls.Engine(0))
