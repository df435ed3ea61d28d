"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY §5 "Race detection /
sanitizers"; GPU sanitizers are not available on this pool):

* the socket path's record splitter (anothertls_amd/csrc/record_split.h, which stream.cpp uses to
  split untrusted received bytes) fed randomized record streams in random chunks, against the
  mirror of the reference's Record::from_raw (anothertls_amd/record.py, net/record.rs:81-102);
* the oracle (oracle/ref_restatement.c) over every entry point (tests/native/oracle_asan.c);
* how the socket path cuts flushes and receive rounds into engine batches (anothertls_amd/csrc/stream_batches.h)
  on random connection / record layouts (tests/native/batches_fuzz.cpp).
"""
import fcntl
import os
import random
import struct
import subprocess

import pytest

from anothertls_amd import TlsError
from anothertls_amd.record import Record

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NATIVE = os.path.join(ROOT, "tests", "native")


@pytest.fixture(scope="module")
def san_build():
    # one build at a time: pytest-xdist workers each run this fixture, and a second `make`
    # rewriting a binary the first worker is executing fails with ETXTBSY
    os.makedirs(os.path.join(NATIVE, "build"), exist_ok=True)
    with open(os.path.join(NATIVE, "build", ".lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        try:
            subprocess.check_call(["make", "-s", "-C", NATIVE, "san"])
        except (OSError, subprocess.CalledProcessError) as exc:  # no sanitizer runtime here
            pytest.skip(f"sanitizer build unavailable: {exc}")
    return os.path.join(NATIVE, "build")


def test_oracle_under_asan_ubsan(san_build):
    r = subprocess.run([os.path.join(san_build, "oracle_san")], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "OK" in r.stdout


def _model(stream):
    """Whole records of `stream` as the splitter must report them: Record::from_raw on each
    complete record (record.rs:81-102; the splitter waits for a partial one instead of failing)
    and DecodeError for a fragment shorter than a tag (record.rs:208 would underflow)."""
    recs, pos = [], 0
    while len(stream) - pos >= 5:
        n = (stream[pos + 3] << 8) | stream[pos + 4]
        if len(stream) - pos < 5 + n:
            break
        try:
            consumed, rec = Record.from_raw(stream[pos:])
        except TlsError as e:
            return recs, e.code, len(stream) - pos
        if rec.len < 16:
            return recs, TlsError.DECODE_ERROR, len(stream) - pos
        recs.append((pos, rec.len))
        pos += consumed
    return recs, None, len(stream) - pos


def _stream(rng):
    out = bytearray()
    for _ in range(rng.randint(0, 12)):
        kind = rng.random()
        n = rng.choice([16, 17, 100, 600, rng.randint(0, 700)])
        t = rng.choice([20, 21, 22, 23, 0]) if kind > 0.1 else rng.choice([1, 19, 24, 255])
        out += bytes([t, 3, 3, n >> 8, n & 255]) + bytes(rng.getrandbits(8) for _ in range(n))
    if out and rng.random() < 0.5:
        out = out[:rng.randint(0, len(out))]  # a partial record at the end
    return bytes(out)


def test_split_fuzz_matches_from_raw(san_build):
    rng = random.Random(2024)
    exe = os.path.join(san_build, "split_fuzz_san")
    for it in range(120):
        s = _stream(rng)
        cuts = sorted(rng.sample(range(len(s) + 1), min(len(s) + 1, rng.randint(1, 6))))
        pieces = [s[a:b] for a, b in zip([0] + cuts, cuts + [len(s)])]
        data = b"".join(struct.pack("<I", len(p)) + p for p in pieces)
        r = subprocess.run([exe], input=data, capture_output=True, timeout=60)
        assert r.returncode == 0, r.stderr.decode()[-2000:]
        lines = r.stdout.decode().split("\n")
        got = [tuple(int(x) for x in ln.split()[1:]) for ln in lines if ln.startswith("R ")]
        err = [int(ln.split()[1]) for ln in lines if ln.startswith("E ")]
        left = [int(ln.split()[1]) for ln in lines if ln.startswith("P ")][0]
        want, werr, wleft = _model(s)
        assert got == want, (it, got, want)
        assert (err[0] if err else None) == werr, (it, err, werr)
        assert left == wleft, (it, left, wleft)


def test_stream_batches_fuzz(san_build):
    r = subprocess.run([os.path.join(san_build, "batches_fuzz_san")], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "OK" in r.stdout
