"""GPU: the native batched record streams (anothertls_amd/csrc/stream.cpp, atls_sb_* in
include/atls.h; TlsStream::tls_write / tls_read of net/stream.rs batched over connections),
driven through the C ABI with ctypes over socket pairs. The wire bytes are the reference's
records (oracle restatement of RecordPayloadProtection::encrypt, record.rs:162-198) for writes
up to 2^14 bytes; longer writes are fragmented; partial records are kept across reads; a
tampered record ends only its connection (DecryptError); a non-application-data record gives
UnexpectedMessage (stream.rs:112-116). Also runs the C1 native loopback tool."""
import ctypes as C
import json
import os
import socket
import subprocess

import numpy as np
import pytest

import oracle as ora

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def atls():
    import anothertls_amd as a

    if not a.device_available():
        pytest.skip("no HIP device")
    lib = a.library()
    P = C.c_void_p
    lib.atls_sb_create.restype = P
    lib.atls_sb_create.argtypes = [P]
    lib.atls_sb_destroy.argtypes = [P]
    lib.atls_sb_add_connection.argtypes = [P, C.c_int, P, P]
    lib.atls_sb_write.argtypes = [P, C.c_int, C.c_uint8, P, C.c_size_t]
    lib.atls_sb_flush.restype = C.c_long
    lib.atls_sb_flush.argtypes = [P]
    lib.atls_sb_feed.argtypes = [P, C.c_int, P, C.c_size_t]
    lib.atls_sb_read.argtypes = [P, C.c_int, P, C.c_size_t, C.POINTER(C.c_size_t)]
    lib.atls_sb_read_ready.argtypes = [P, C.c_int, P, C.c_size_t, C.POINTER(C.c_size_t)]
    lib.atls_sb_set_threads.argtypes = [P, C.c_int]
    lib.atls_sb_recv_all.restype = C.c_long
    lib.atls_sb_recv_all.argtypes = [P, C.c_int]
    lib.atls_sb_open_pending.restype = C.c_long
    lib.atls_sb_open_pending.argtypes = [P]
    return a


def _keys(a, i):
    suite, kl = [(0x1301, 16), (0x1302, 32), (0x1303, 32)][i % 3]
    rng = np.random.default_rng(200 + i)
    k = lambda: (suite, rng.integers(0, 256, kl, dtype=np.uint8).tobytes(),  # noqa: E731
                 rng.integers(0, 256, 12, dtype=np.uint8).tobytes())
    return a.make_keys([k()]), a.make_keys([k()])


def _read(lib, sb, conn, cap=1 << 15):
    buf = (C.c_uint8 * cap)()
    n = C.c_size_t(0)
    rc = lib.atls_sb_read(sb, conn, buf, cap, C.byref(n))
    return rc, bytes(buf[:n.value])


def test_native_stream_batch(atls):
    lib = atls.library()
    e_s, e_c = atls.Engine(0), atls.Engine(0)
    s_sb, c_sb = lib.atls_sb_create(e_s._e), lib.atls_sb_create(e_c._e)
    n = 5
    pairs = [socket.socketpair() for _ in range(n)]
    keys = [_keys(atls, i) for i in range(n)]
    sconn = [lib.atls_sb_add_connection(s_sb, a.fileno(), w.ctypes.data, r.ctypes.data)
             for (a, _), (w, r) in zip(pairs, keys)]
    cconn = [lib.atls_sb_add_connection(c_sb, b.fileno(), r.ctypes.data, w.ctypes.data)
             for (_, b), (w, r) in zip(pairs, keys)]
    rng = np.random.default_rng(3)
    sizes = [0, 1, 16, 4096, 16384, 20000, 77]
    sent = []
    for i in range(n):
        ds = [rng.integers(0, 256, s, dtype=np.uint8).tobytes() for s in sizes[i % 2:]]
        for d in ds:
            assert lib.atls_sb_write(s_sb, sconn[i], 23, d, len(d)) == 0
        sent.append(ds)
    assert lib.atls_sb_flush(s_sb) == sum(max(1, -(-len(d) // 16384)) for ds in sent for d in ds)
    # connection 0 by hand: raw wire bytes against the oracle, then fed back in ragged pieces
    want = b""
    w = keys[0][0][0]
    seq = 0
    for d in sent[0]:
        for f in [d[j:j + 16384] for j in range(0, len(d), 16384)] or [b""]:
            rc, rec = ora.record_seal(int(w["suite"]), bytes(w["key"][:int(w["key_len"])]), bytes(w["static_iv"]),
                                      seq, 23, f)
            assert rc == 0
            want += rec
            seq += 1
    raw = b""
    while len(raw) < len(want):
        raw += pairs[0][1].recv(1 << 16)
    assert raw == want
    cut = 0
    while cut < len(raw):
        k = int(rng.integers(1, 5000))
        assert lib.atls_sb_feed(c_sb, cconn[0], raw[cut:cut + k], len(raw[cut:cut + k])) == 0
        cut += k
    for i in range(n):
        got = b""
        while len(got) < sum(map(len, sent[i])):
            rc, d = _read(lib, c_sb, cconn[i])
            assert rc == 0, (i, rc)
            got += d
        assert got == b"".join(sent[i]), i
    # reverse direction: a tampered record on connection 1, a handshake record on connection 2
    for i in range(n):
        msg = b"pong %d" % i
        assert lib.atls_sb_write(c_sb, cconn[i], 23, msg, len(msg)) == 0
    assert lib.atls_sb_write(c_sb, cconn[2], 22, b"\x14\x00\x00\x00", 4) == 0
    assert lib.atls_sb_flush(c_sb) == n + 1
    bad = bytearray(pairs[1][0].recv(1 << 16))
    bad[9] ^= 1
    assert lib.atls_sb_feed(s_sb, sconn[1], bytes(bad), len(bad)) == 0
    for i in (0, 3, 4):
        assert _read(lib, s_sb, sconn[i]) == (0, b"pong %d" % i)
    assert _read(lib, s_sb, sconn[1])[0] == 50  # DecryptError (record.rs:222)
    assert _read(lib, s_sb, sconn[2]) == (0, b"pong 2")
    assert _read(lib, s_sb, sconn[2])[0] == 10  # UnexpectedMessage (stream.rs:112-116)
    lib.atls_sb_destroy(s_sb)
    lib.atls_sb_destroy(c_sb)
    for a, b in pairs:
        a.close()
        b.close()
    e_s.close()
    e_c.close()


def test_native_stream_batch_threads(atls):
    """The multi-threaded socket path: 4 worker threads per batch. Flush sends every
    connection's slice from the workers; connection 0's wire bytes are taken off its socket and compared with
    the oracle's records, then fed back; the other connections arrive through atls_sb_recv_all (straight into
    their receive buffers), atls_sb_open_pending (gather and hand-over on the workers) and atls_sb_read_ready
    from several reader threads at once."""
    import threading

    lib = atls.library()
    e_s, e_c = atls.Engine(0), atls.Engine(0)
    s_sb, c_sb = lib.atls_sb_create(e_s._e), lib.atls_sb_create(e_c._e)
    assert lib.atls_sb_set_threads(s_sb, 4) == 0 and lib.atls_sb_set_threads(c_sb, 4) == 0
    assert lib.atls_sb_set_threads(c_sb, 0) == 47 and lib.atls_sb_set_threads(c_sb, 65) == 47
    n = 12
    pairs = [socket.socketpair() for _ in range(n)]
    keys = [_keys(atls, i) for i in range(n)]
    sconn = [lib.atls_sb_add_connection(s_sb, a.fileno(), w.ctypes.data, r.ctypes.data)
             for (a, _), (w, r) in zip(pairs, keys)]
    cconn = [lib.atls_sb_add_connection(c_sb, b.fileno(), r.ctypes.data, w.ctypes.data)
             for (_, b), (w, r) in zip(pairs, keys)]
    rng = np.random.default_rng(11)
    sent = [[rng.integers(0, 256, int(s), dtype=np.uint8).tobytes() for s in rng.integers(0, 40000, 5)]
            for _ in range(n)]
    for rnd in range(2):  # two flushes: sequence numbers continue across them
        for i in range(n):
            for d in sent[i][rnd::2]:
                assert lib.atls_sb_write(s_sb, sconn[i], 23, d, len(d)) == 0
        assert lib.atls_sb_flush(s_sb) > 0
    want, seq = b"", 0
    w = keys[0][0][0]
    for d in sent[0][0::2] + sent[0][1::2]:
        for f in [d[j:j + 16384] for j in range(0, len(d), 16384)] or [b""]:
            rc, rec = ora.record_seal(int(w["suite"]), bytes(w["key"][:int(w["key_len"])]), bytes(w["static_iv"]), seq, 23, f)
            assert rc == 0
            want += rec
            seq += 1
    raw = b""
    while len(raw) < len(want):
        raw += pairs[0][1].recv(1 << 20)
    assert raw == want
    assert lib.atls_sb_feed(c_sb, cconn[0], raw, len(raw)) == 0
    expect = [b"".join(sent[i][0::2] + sent[i][1::2]) for i in range(n)]
    got = [b""] * n
    lock = threading.Lock()
    for _ in range(200):
        if all(len(got[i]) == len(expect[i]) for i in range(n)):
            break
        assert lib.atls_sb_recv_all(c_sb, 200) >= 0
        assert lib.atls_sb_open_pending(c_sb) >= 0

        def reader(t):
            buf = (C.c_uint8 * 16384)()
            ln = C.c_size_t(0)
            for i in range(t, n, 3):
                while (rc := lib.atls_sb_read_ready(c_sb, cconn[i], buf, 16384, C.byref(ln))) == 0:
                    with lock:
                        got[i] += bytes(buf[:ln.value])
                assert rc == 0x100, rc  # ATLS_WOULD_BLOCK (outside the u8 TlsError range)

        ths = [threading.Thread(target=reader, args=(t,)) for t in range(3)]
        for th in ths:
            th.start()
        for th in ths:
            th.join()
    assert got == expect
    for sb in (s_sb, c_sb):
        lib.atls_sb_destroy(sb)
    for a, b in pairs:
        a.close()
        b.close()
    e_s.close()
    e_c.close()


@pytest.mark.timeout(120)
# (80, 8): 80 connections x 2 bodies is 168 MB of wire per flush and per receive round at most, so both go
# to the engine in several batches of whole connections (stream.cpp kBatchBytes, 64 MiB), sealed while the
# previous batch is sent
@pytest.mark.parametrize("conns,threads", [(4, 1), (16, 4), (80, 8)])
def test_c1_native_loopback_tool(atls, conns, threads):
    exe = os.path.join(ROOT, "tools", "c1_loopback_native")
    if not os.path.exists(exe):
        pytest.skip("tools/c1_loopback_native not built (tools/build_native.sh)")
    out = subprocess.run([exe, "2", str(conns), str(threads)], capture_output=True, text=True, timeout=100)
    assert out.returncode == 0, out.stderr[-2000:]
    line = json.loads(out.stdout.strip().splitlines()[-1])
    assert line["verified"] is True and line["gpu_MBps"] > 0 and line["threads"] == threads


def test_native_interleaved_writes_and_peer_close(atls):
    """(1) a server that writes round robin across its connections leaves the flush's inputs out of
    record order; the flush gathers such a batch's inputs into record order, so the engine's host pipeline still
    takes it (it would otherwise stage the whole arena prefix in one piece, once per batch) -- wire bytes against
    the oracle's records (record.rs:162-198), every byte read back. (2) A peer that closes ends its connection's
    stream with BrokenPipe (TlsStream::tcp_read at a zero-byte read, net/stream.rs:68-73) for an event loop that
    only uses recv_all / open_pending / read_ready: after the whole records that arrived before the close, with a
    partial record left behind, and with nothing; recv_all returns at once once every peer has closed."""
    import time

    lib = atls.library()
    lib.atls_debug_sb_gathered.restype = C.c_ulonglong
    lib.atls_debug_sb_gathered.argtypes = [C.c_void_p]
    lib.atls_debug_host_unpipelined.restype = C.c_ulonglong
    e_s, e_c = atls.Engine(0), atls.Engine(0)
    s_sb, c_sb = lib.atls_sb_create(e_s._e), lib.atls_sb_create(e_c._e)
    assert lib.atls_sb_set_threads(s_sb, 4) == 0 and lib.atls_sb_set_threads(c_sb, 4) == 0
    n = 6
    pairs = [socket.socketpair() for _ in range(n)]
    keys = [_keys(atls, i) for i in range(n)]
    sconn = [lib.atls_sb_add_connection(s_sb, a.fileno(), w.ctypes.data, r.ctypes.data)
             for (a, _), (w, r) in zip(pairs, keys)]
    cconn = [lib.atls_sb_add_connection(c_sb, b.fileno(), r.ctypes.data, w.ctypes.data)
             for (_, b), (w, r) in zip(pairs, keys)]
    rng = np.random.default_rng(29)
    sent = [[] for _ in range(n)]
    for k in range(8):  # round robin: connection i's k-th write lands after every connection's (k-1)-th
        for i in range(n):
            d = rng.integers(0, 256, int(rng.integers(0, 20000)), dtype=np.uint8).tobytes()
            assert lib.atls_sb_write(s_sb, sconn[i], 23, d, len(d)) == 0
            sent[i].append(d)
    unpipelined0 = lib.atls_debug_host_unpipelined()
    assert lib.atls_sb_flush(s_sb) == sum(max(1, -(-len(d) // 16384)) for ds in sent for d in ds)
    assert lib.atls_debug_sb_gathered(s_sb) >= 1
    assert lib.atls_debug_host_unpipelined() == unpipelined0  # the gathered batch went through the pipeline
    want, seq = b"", 0
    w = keys[0][0][0]
    for d in sent[0]:
        for f in [d[j:j + 16384] for j in range(0, len(d), 16384)] or [b""]:
            rc, rec = ora.record_seal(int(w["suite"]), bytes(w["key"][:int(w["key_len"])]), bytes(w["static_iv"]), seq, 23, f)
            assert rc == 0
            want += rec
            seq += 1
    raw = b""
    while len(raw) < len(want):
        raw += pairs[0][1].recv(1 << 20)
    assert raw == want
    assert lib.atls_sb_feed(c_sb, cconn[0], raw, len(raw)) == 0
    expect = [b"".join(ds) for ds in sent]
    got = [b""] * n
    buf = (C.c_uint8 * 16384)()
    ln = C.c_size_t(0)
    for _ in range(200):
        if got == expect:
            break
        assert lib.atls_sb_recv_all(c_sb, 200) >= 0
        assert lib.atls_sb_open_pending(c_sb) >= 0
        for i in range(n):
            while (rc := lib.atls_sb_read_ready(c_sb, cconn[i], buf, 16384, C.byref(ln))) == 0:
                got[i] += bytes(buf[:ln.value])
            assert rc == 0x100, (i, rc)
    assert got == expect
    # the peers close: connection 1 with nothing in flight, 2 after half a record, 3 after a whole record
    msg = b"last words"
    assert lib.atls_sb_write(s_sb, sconn[3], 23, msg, len(msg)) == 0
    assert lib.atls_sb_write(s_sb, sconn[2], 23, msg, len(msg)) == 0
    assert lib.atls_sb_flush(s_sb) == 2
    rec2 = b""
    while len(rec2) < 5 + len(msg) + 17:
        rec2 += pairs[2][1].recv(1 << 16)
    pairs[2][0].close()  # conn 2: the client gets only half of its record, fed by hand, then the socket's EOF
    assert lib.atls_sb_feed(c_sb, cconn[2], rec2[:10], 10) == 0
    for i in (1, 3):
        pairs[i][0].close()
    for _ in range(20):
        assert lib.atls_sb_recv_all(c_sb, 100) >= 0
        assert lib.atls_sb_open_pending(c_sb) >= 0
        if lib.atls_sb_read_ready(c_sb, cconn[1], buf, 16384, C.byref(ln)) != 0x100:
            break
    assert lib.atls_sb_read_ready(c_sb, cconn[1], buf, 16384, C.byref(ln)) == 254  # BrokenPipe
    assert lib.atls_sb_read_ready(c_sb, cconn[3], buf, 16384, C.byref(ln)) == 0 and bytes(buf[:ln.value]) == msg
    assert lib.atls_sb_read_ready(c_sb, cconn[3], buf, 16384, C.byref(ln)) == 254
    assert lib.atls_sb_read_ready(c_sb, cconn[2], buf, 16384, C.byref(ln)) == 254  # the partial record never completes
    assert lib.atls_sb_read(c_sb, cconn[1], buf, 16384, C.byref(ln)) == 254  # the blocking read agrees
    for i in (0, 4, 5):
        pairs[i][0].close()
    t0 = time.monotonic()
    for _ in range(5):  # every peer closed: nothing to poll, no wait
        assert lib.atls_sb_recv_all(c_sb, 1000) == 0
    assert time.monotonic() - t0 < 1.0
    for i in (0, 4, 5):
        assert lib.atls_sb_read_ready(c_sb, cconn[i], buf, 16384, C.byref(ln)) == 254
    for sb in (s_sb, c_sb):
        lib.atls_sb_destroy(sb)
    for a, b in pairs:
        b.close()
    e_s.close()
    e_c.close()
