"""GPU: the AES block cipher (AES::encrypt / AES::decrypt, crypto/aes/cipher.rs:175-215) through
atls_aes_block / atls_aes_blocks, against the reference's FIPS-197 KATs (tests/golden) and the
oracle's restatement on random blocks for all three key sizes."""
import json
import os

import numpy as np
import pytest

import oracle as ora

pytestmark = pytest.mark.gpu
KATS = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_kats.json")))
H = bytes.fromhex


@pytest.fixture(scope="module")
def atls():
    import anothertls_amd as a

    if not a.device_available():
        pytest.skip("no HIP device")
    return a


@pytest.mark.parametrize("v", KATS["aes_block"], ids=lambda v: v["name"])
def test_aes_block_kats(atls, v):
    aes = atls.AES.init(H(v["key"]))
    ct = aes.encrypt(H(v["pt"]))
    assert ct.hex() == v["ct"]
    assert aes.decrypt(ct).hex() == v["pt"]


@pytest.mark.parametrize("key_len", [16, 24, 32])
@pytest.mark.parametrize("device", [True, False], ids=["device", "host"])
def test_aes_blocks_vs_oracle(atls, key_len, device):
    import torch

    rng = np.random.default_rng(key_len)
    key = rng.integers(0, 256, key_len, dtype=np.uint8).tobytes()
    nb = 3001
    blocks = rng.integers(0, 256, 16 * nb, dtype=np.uint8)
    eng = atls.Engine(0)
    eng.set_keys(atls.make_keys([(0x1302, rng.integers(0, 256, 32, dtype=np.uint8).tobytes(), bytes(12)),
                                 (0x1301, key, bytes(12))]))
    if device:
        dev = torch.device("cuda", 0)
        d_in = torch.from_numpy(blocks).to(dev)
        d_ct = torch.empty_like(d_in)
        d_pt = torch.empty_like(d_in)
        eng.aes_blocks(False, 1, d_in, d_ct, flags=atls.FLAG_DEVICE_PTRS)
        eng.aes_blocks(True, 1, d_ct, d_pt, flags=atls.FLAG_DEVICE_PTRS)
        ct, pt = d_ct.cpu().numpy(), d_pt.cpu().numpy()
    else:
        ct, pt = np.empty_like(blocks), np.empty_like(blocks)
        eng.aes_blocks(False, 1, blocks, ct)
        eng.aes_blocks(True, 1, ct, pt)
    assert np.array_equal(pt, blocks)
    for i in list(range(0, nb, 97)) + [nb - 1]:
        rc, want = ora.aes_encrypt_block(key, blocks[16 * i:16 * i + 16].tobytes())
        assert rc == 0 and ct[16 * i:16 * i + 16].tobytes() == want, i
    eng.close()


def test_aes_blocks_rejects_non_aes_slot(atls):
    eng = atls.Engine(0)
    eng.set_keys(atls.make_keys([(0x1303, bytes(32), bytes(12))]))
    with pytest.raises(atls.TlsError) as e:
        eng.aes_blocks(False, 0, np.zeros(32, np.uint8), np.zeros(32, np.uint8))
    assert e.value.code == 47
    with pytest.raises(atls.TlsError) as e:
        eng.aes_blocks(False, 5, np.zeros(32, np.uint8), np.zeros(32, np.uint8))
    assert e.value.code == 47
    eng.close()
