"""The built library's kernels keep the register budgets the design depends on (host-only; reads the gfx950 code
objects' metadata, tests/helpers/kernel_resources.py):
- no record kernel on a default path uses scratch (C5's planned ChaCha20-Poly1305 open spilled);
- a mixed batch's two kernels fit on one SIMD together: the AES-GCM seal instance that runs beside the ChaCha side
  kernel, and the side kernels themselves, stay within 128 VGPRs (3 AES-GCM waves + 1 ChaCha wave = 512,
  gcm.hip:1197-1204, chacha.hip ATLS_CHACHA_MINW_SIDE)."""
import os

import pytest

from helpers.kernel_resources import READELF, kernel_resources

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "anothertls_amd", "libatls.so")

# Scratch by design, off the record path: the SHA / HMAC / HKDF kernels keep per-thread message schedules in
# private arrays (once per connection); the 3-wave direct ChaCha20-Poly1305 kernel runs only
# under ATLS_CHACHA_W2=0.
ALLOWED_SCRATCH = ("hash_kernel", "derive_kernel", "key_schedule_kernel", "chacha_kernelILb0ELb0E",
                   "chacha_kernelILb1ELb0E")


@pytest.fixture(scope="module")
def res():
    if not os.path.exists(LIB):
        pytest.skip("libatls.so not built")
    if not os.path.exists(READELF):
        pytest.skip("llvm-readelf not present")
    r = kernel_resources(LIB)
    assert len(r) > 40, f"only {len(r)} kernels found"
    return r


def test_record_kernels_use_no_scratch(res):
    bad = {k: v for k, v in res.items() if v[0] and not any(a in k for a in ALLOWED_SCRATCH)}
    assert not bad, f"kernels with scratch: {bad}"


def test_mixed_batch_kernels_fit_one_simd_together(res):
    beside = [k for k in res if k.startswith("_ZN4atls10gcm_kernelILb0ELi12E") and k.endswith("ELb1EEEvNS_7GcmArgsE")]
    side = [k for k in res if k.startswith("_ZN4atls13chacha_kernelIL") and "ELb1EEEvNS_6ChArgsE" in k]
    assert len(beside) >= 2 and len(side) == 2, (beside, side)
    for k in beside + side:
        assert res[k][1] <= 128, f"{k}: {res[k][1]} VGPRs"


def test_direct_chacha_kernels_fit_two_waves(res):
    w2 = [k for k in res if "chacha_kernel_w2" in k]
    assert len(w2) == 2
    for k in w2:
        assert res[k][1] <= 256 and res[k][0] == 0, (k, res[k])
