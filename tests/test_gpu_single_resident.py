"""The resident single-call server (ATLS_SINGLE_RESIDENT=1, gcm.hip single_resident): a
workgroup that stays on the GPU and answers Cipher-trait calls of both suites through a doorbell in mapped
memory instead of a launch per call. The mode is read once per process, so the checks run in a child process
(tests/helpers/resident_check.py), in both modes (1: ChaCha20-Poly1305 through the server, AES-GCM launched;
2: both through the server): every call against the oracle (crypto/chacha20/poly1305.rs:69-104,
crypto/aes/gcm.rs:42-162), the F4 lengths, AES-GCM with 12-byte and other IVs and 128/192/256-bit keys, suites
interleaved, batch launches between calls, calls after the server left on its idle timeout, 8 threads at once;
and the process exits cleanly with its server stopped."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(180)
@pytest.mark.parametrize("mode", ["1", "2"])
def test_resident_single_calls_vs_oracle(mode):
    env = dict(os.environ, ATLS_SINGLE_RESIDENT=mode, ATLS_SINGLE_RESIDENT_IDLE_MS="5")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "helpers", "resident_check.py")], env=env,
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, (out.stdout[-2000:], out.stderr[-3000:])
    assert "resident OK" in out.stdout
