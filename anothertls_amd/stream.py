"""Batched host socket path: TlsStream::tls_write / tls_read (net/stream.rs:32-150) for many
connections at once, over one device engine.

The reference seals one record per ``tls_write`` call and opens one record per ``tls_read``
(stream.rs:97-150), each through ``RecordPayloadProtection::{encrypt,decrypt}``
(net/record.rs:162-240). Here every connection queues its writes, and ``flush`` seals the queued
records of ALL connections in one ``atls_seal_batch`` in ATLS_MODE_WIRE: the device writes each
record's header || ciphertext || tag straight into one staging buffer, each connection's records
contiguous, and each connection's slice goes to its socket with one ``sendall``. On the way in,
bytes received per connection are split into whole records (``Record::from_raw``,
record.rs:81-102; a partial record stays buffered for the next read — the reference's
``todo!()`` at stream.rs:106-108), and ``open_pending`` opens the complete records of all
connections in one ``atls_open_batch`` (WIRE mode: the received header is the AAD,
record.rs:219).

Per connection the state is the reference's: a write key and a read key (``WriteKeys``,
key_schedule.rs:67-114) each with its own sequence number, incremented per record
(``get_per_record_nonce``, key_schedule.rs:51-64). A record that fails to open poisons its
connection with the TlsError the reference returns (DecryptError / DecodeError); ``tls_read``
returns application data only and raises UnexpectedMessage for other inner content types
(stream.rs:112-116).

Divergence (documented): writes longer than 2^14 bytes are fragmented into 2^14-byte records
(RFC 8446 §5.1); the reference emits a single over-long record. Writes up to 2^14 bytes give the
same wire bytes as the reference.
"""
import collections

import numpy as np

from . import MODE_WIRE, OPEN_RESULT_DTYPE, REC_DTYPE, TlsError, make_keys
from .record import RecordType

MAX_FRAGMENT = 1 << 14  # RFC 8446 §5.1
_RECORD_TYPES = frozenset(int(t) for t in RecordType)


def record_type_ok(b):
    return b in _RECORD_TYPES
UNEXPECTED_MESSAGE = 10  # alert.rs:22
BROKEN_PIPE = 254  # alert.rs:44 (not official)
_OVERHEAD = 5 + 1 + 16  # header, inner content type, tag


def _staging(nbytes):
    """Page-locked host buffer when torch can provide one (fast DMA), else plain numpy."""
    try:
        import torch

        if torch.cuda.is_available():
            return torch.empty(max(nbytes, 16), dtype=torch.uint8, pin_memory=True).numpy()
    except Exception:  # pinned allocation is an optimisation only
        pass
    return np.empty(max(nbytes, 16), np.uint8)


class _Buf:
    """Grow-only staging buffer."""

    def __init__(self):
        self.a = np.empty(0, np.uint8)

    def get(self, nbytes):
        if self.a.size < nbytes + 16:
            self.a = _staging(max(nbytes + 16, 2 * self.a.size))
        return self.a


class Connection:
    """One connection's application-traffic protection (RecordPayloadProtection, record.rs:116-160)."""

    def __init__(self, index, sock, write_slot, read_slot):
        self.index = index
        self.sock = sock
        self.write_slot = write_slot
        self.read_slot = read_slot
        self.write_seq = 0
        self.read_seq = 0
        self.error = None
        self._out = []  # queued (content_type, fragment) records
        self._rx = bytearray()  # received bytes not yet split into records
        self._records = []  # complete received wire records not yet opened: (bytes, record offsets)
        self._pending = 0  # records in _records
        self.inbox = collections.deque()  # opened (content_type, plaintext)

    def _check(self):
        if self.error is not None:
            raise self.error


class StreamBatch:
    """Many TLS connections sharing one engine: batched seal on flush, batched open on read.

    engine: an object with set_keys / seal_batch / open_batch of ``anothertls_amd.Engine``."""

    def __init__(self, engine):
        self.engine = engine
        self.conns = []
        self._keys = []
        self._keys_dirty = False
        self._in, self._wire, self._pt = _Buf(), _Buf(), _Buf()

    # ---- connections ------------------------------------------------------------------------
    def add_connection(self, sock, write_key, read_key):
        """write_key / read_key: (suite, key, static_iv) as Key::from_hkdf produces them."""
        c = Connection(len(self.conns), sock, len(self._keys), len(self._keys) + 1)
        self._keys += [tuple(write_key), tuple(read_key)]
        self._keys_dirty = True
        self.conns.append(c)
        return c

    def _install_keys(self):
        if self._keys_dirty:
            self.engine.set_keys(make_keys(self._keys))
            self._keys_dirty = False

    # ---- write side (stream.rs:32-58, :136-150) --------------------------------------------
    def write_record(self, conn, typ, data):
        """Queue one record's worth of content (fragmented at 2^14, RFC 8446 §5.1)."""
        conn._check()
        typ = RecordType(typ)
        data = bytes(data)
        if not data:
            conn._out.append((typ, b""))
        for i in range(0, len(data), MAX_FRAGMENT):
            conn._out.append((typ, data[i:i + MAX_FRAGMENT]))

    def tls_write(self, conn, data):
        self.write_record(conn, RecordType.ApplicationData, data)

    def flush(self):
        """Seal every queued record of every connection in one device batch and send each
        connection's records with one sendall. Returns the number of records sealed."""
        todo = [c for c in self.conns if c._out]
        if not todo:
            return 0
        self._install_keys()
        frags = [f for c in todo for _, f in c._out]
        n = len(frags)
        lens = np.fromiter(map(len, frags), np.int64, n)
        ends = np.cumsum(lens)
        wire_ends = np.cumsum(lens + _OVERHEAD)
        recs = np.zeros(n, REC_DTYPE)
        recs["in_off"] = ends - lens
        recs["out_off"] = wire_ends - (lens + _OVERHEAD)
        recs["len"] = lens
        recs["mode"] = MODE_WIRE
        recs["content_type"] = np.fromiter((int(t) for c in todo for t, _ in c._out), np.uint8, n)
        recs["key_slot"] = np.repeat([c.write_slot for c in todo], [len(c._out) for c in todo])
        recs["seq"] = np.concatenate([np.arange(c.write_seq, c.write_seq + len(c._out), dtype=np.uint64)
                                      for c in todo])
        inbuf = self._in.get(int(ends[-1]))
        for f, e in zip(frags, ends.tolist()):  # straight into the (pinned) staging buffer
            inbuf[e - len(f):e] = np.frombuffer(f, np.uint8)
        wire = self._wire.get(int(wire_ends[-1]))
        self.engine.seal_batch(recs, inbuf, np.zeros(16, np.uint8), wire, None)
        i = 0
        for c in todo:
            k = len(c._out)
            lo, hi = int(recs["out_off"][i]), int(wire_ends[i + k - 1])
            c.write_seq += k
            c._out = []
            i += k
            try:
                c.sock.sendall(memoryview(wire)[lo:hi])
            except OSError:
                c.error = TlsError(BROKEN_PIPE)
        return n

    # ---- read side (stream.rs:97-133) ------------------------------------------------------
    def feed(self, conn, data):
        """Bytes received on conn's socket."""
        if conn._rx:
            conn._rx += data
            data = bytes(conn._rx)
            conn._rx = bytearray()
        else:
            data = bytes(data)
        pos = self._split(conn, data)
        if pos < len(data):
            conn._rx += memoryview(data)[pos:]  # a partial record waits for more bytes

    def recv(self, conn, bufsize=1 << 20):
        """One socket read into conn's record buffer (stream.rs:74-79); False on EOF."""
        data = conn.sock.recv(bufsize)
        if not data:
            return False
        self.feed(conn, data)
        return True

    @staticmethod
    def _split(conn, buf):
        """Whole records at the front of buf (Record::from_raw checks, record.rs:81-102), kept as
        buf plus record offsets (no copy). Returns the bytes consumed."""
        pos, offs, end = 0, [], len(buf)
        while end - pos >= 5:
            ln = (buf[pos + 3] << 8) | buf[pos + 4]
            if end - pos < 5 + ln:
                break  # partial record
            if not record_type_ok(buf[pos]) or ln < 16:
                # RecordType::new (record.rs:23-32); a fragment shorter than a tag underflows the
                # reference's slice (record.rs:208)
                conn.error = TlsError(TlsError.DECODE_ERROR)
                break
            offs.append(pos)
            pos += 5 + ln
        if offs:
            conn._records.append((buf if pos == end else buf[:pos], offs))
            conn._pending += len(offs)
        return pos

    def open_pending(self):
        """Open every complete received record of every connection in one device batch.
        Returns the number of records opened."""
        todo = [c for c in self.conns if c._pending and c.error is None]
        if not todo:
            return 0
        self._install_keys()
        chunks = [ch for c in todo for ch in c._records]
        base = np.cumsum([0] + [len(b) for b, _ in chunks])
        in_off = np.concatenate([np.asarray(o, np.int64) + base[j] for j, (_, o) in enumerate(chunks)])
        n = len(in_off)
        wire = self._wire.get(int(base[-1]))
        for (b, _), lo in zip(chunks, base.tolist()):
            wire[lo:lo + len(b)] = np.frombuffer(b, np.uint8)
        ct_len = ((wire[in_off + 3].astype(np.int64) << 8) | wire[in_off + 4]) - 16
        pt_end = np.cumsum(ct_len)
        pt = self._pt.get(int(pt_end[-1]))
        recs = np.zeros(n, REC_DTYPE)
        recs["in_off"] = in_off
        recs["out_off"] = pt_end - ct_len
        recs["len"] = ct_len
        recs["mode"] = MODE_WIRE
        counts = [c._pending for c in todo]
        recs["key_slot"] = np.repeat([c.read_slot for c in todo], counts)
        recs["seq"] = np.concatenate([np.arange(c.read_seq, c.read_seq + k, dtype=np.uint64)
                                      for c, k in zip(todo, counts)])
        res = np.zeros(n, OPEN_RESULT_DTYPE)
        self.engine.open_batch(recs, wire, np.zeros(16, np.uint8), None, pt, res)
        st, cl, ty, po = (res["status"].tolist(), res["content_len"].tolist(), res["content_type"].tolist(),
                          recs["out_off"].tolist())
        i = 0
        for c, k in zip(todo, counts):
            c.read_seq += k
            c._records, c._pending = [], 0
            for j in range(i, i + k):
                if st[j]:  # a failed record ends the connection (the reference returns the error)
                    c.error = TlsError(st[j])
                    break
                c.inbox.append((ty[j], pt[po[j]:po[j] + cl[j]].tobytes()))
            i += k
        return n

    def tls_read(self, conn):
        """Next application-data plaintext of conn (stream.rs:97-133): receives and opens as
        needed. Raises the connection's TlsError, UnexpectedMessage for a non-application-data
        record, BrokenPipe on EOF."""
        while not conn.inbox:
            conn._check()
            if not conn._pending and not self.recv(conn):
                raise TlsError(BROKEN_PIPE)
            self.open_pending()
        typ, data = conn.inbox.popleft()
        if typ != RecordType.ApplicationData:
            raise TlsError(UNEXPECTED_MESSAGE)
        return data
