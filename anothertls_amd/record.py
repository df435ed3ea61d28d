"""TLS 1.3 record framing on the host, mirroring net/record.rs of otsmr/AnotherTLS.

* ``RecordType`` — record.rs:13-33 (``RecordType::new`` rejects unknown bytes with DecodeError).
* ``Record.new`` / ``Record.from_raw`` / ``Record.as_bytes`` — record.rs:70-114, including the
  reference's bounds check ``buf.len() < 2 + len`` (record.rs:88); where the reference would then
  panic slicing ``buf[5..5+len]`` we raise ``TlsError(DecodeError)`` (documented divergence,
  DESIGN.md §1).
* ``frame_sealed`` / ``parse_stream`` — the batched form the socket path uses around the device
  engine: an ``atls_seal_batch`` TLS-mode output (ciphertext of content || type, plus the tag)
  becomes wire records ``[23, 3, 3, n >> 8, n] || ciphertext || tag`` with n = len + 1 + 16
  (record.rs:162-198: the header is also the AEAD's AAD, which the device derives itself), and a
  received byte stream splits back into records for ``atls_open_batch``.
"""
import enum

import numpy as np

from . import TlsError


class RecordType(enum.IntEnum):
    """record.rs:13-20."""

    Invalid = 0
    ChangeCipherSpec = 20
    Alert = 21
    Handshake = 22
    ApplicationData = 23

    @classmethod
    def new(cls, byte):  # record.rs:23-32
        try:
            return cls(byte)
        except ValueError:
            raise TlsError(TlsError.DECODE_ERROR) from None


class Record:
    """record.rs:62-115 (fragment as bytes)."""

    def __init__(self, content_type, fragment, version=0x0303, header=None):
        self.content_type = RecordType(content_type)
        self.version = version
        self.fragment = bytes(fragment)
        self.len = len(self.fragment)
        self.header = bytes(header) if header is not None else bytes([int(content_type), 3, 3, 0, 0])

    @classmethod
    def new(cls, content_type, fragment):  # record.rs:71-79
        return cls(content_type, fragment)

    @classmethod
    def from_raw(cls, buf):
        """record.rs:81-102 -> (consumed, Record)."""
        buf = bytes(buf)
        if len(buf) < 5:
            raise TlsError(TlsError.DECODE_ERROR)
        content_type = RecordType.new(buf[0])
        version = (buf[1] << 8) | buf[2]
        length = (buf[3] << 8) | buf[4]
        if len(buf) < 2 + length:  # the reference's check (record.rs:88)
            raise TlsError(TlsError.DECODE_ERROR)
        if len(buf) < 5 + length:  # the reference panics here (slice out of range)
            raise TlsError(TlsError.DECODE_ERROR)
        consumed = 5 + length
        return consumed, cls(content_type, buf[5:consumed], version=version, header=buf[:5])

    def as_bytes(self):  # record.rs:103-114
        n = len(self.fragment)
        return bytes([int(self.content_type), 3, 3, (n >> 8) & 0xFF, n & 0xFF]) + self.fragment


def frame_sealed(recs, out, tags):
    """Wire bytes of sealed TLS-mode records: for record i an ApplicationData header with
    length n = len + 1 + 16, then out[out_off : out_off + len + 1] and the record's 16-byte tag."""
    recs = np.asarray(recs)
    lens = recs["len"].astype(np.int64) + 1
    wire = np.empty(int((5 + lens + 16).sum()), np.uint8)
    pos = 0
    for i in range(len(recs)):
        L = int(lens[i])
        n = L + 16
        wire[pos:pos + 5] = (23, 3, 3, (n >> 8) & 0xFF, n & 0xFF)
        o = int(recs["out_off"][i])
        wire[pos + 5:pos + 5 + L] = out[o:o + L]
        wire[pos + 5 + L:pos + 5 + n] = tags[16 * i:16 * i + 16]
        pos += 5 + n
    return wire


def parse_stream(wire):
    """Split a received byte stream into whole records with Record::from_raw (record.rs:81-102):
    returns (header offsets, fragment lengths)."""
    data = np.asarray(wire, np.uint8).tobytes()
    offs, lens = [], []
    pos = 0
    while pos + 5 <= len(data):
        consumed, rec = Record.from_raw(data[pos:])
        offs.append(pos)
        lens.append(rec.len)
        pos += consumed
    return np.array(offs, np.int64), np.array(lens, np.int64)
