"""Small bitsliced-kernel checks with per-case progress output (GPU debugging aid)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402

import anothertls_amd as atls  # noqa: E402
import oracle as ora  # noqa: E402
from anothertls_amd import workload  # noqa: E402
from test_gpu_parity import oracle_keys, oracle_recs  # noqa: E402


def case(eng, n, L, suite=0x1301):
    batch = workload.tls_batch(n, L, suite, n_keys=max(1, n // 2))
    inbuf = np.random.default_rng(n).integers(0, 256, size=batch["in_bytes"] + 16, dtype=np.uint8)
    eng.set_keys(batch["keys"])
    out = np.zeros(batch["out_bytes"] + 16, np.uint8)
    tags = np.zeros(16 * n, np.uint8)
    t0 = time.time()
    eng.seal_batch(batch["recs"], inbuf, np.zeros(16, np.uint8), out, tags)
    dt = time.time() - t0
    oout, otags = np.zeros_like(out), np.zeros_like(tags)
    ora.seal_batch(oracle_keys(batch["keys"]), oracle_recs(batch["recs"]), inbuf, np.zeros(16, np.uint8), oout,
                   otags, 8)
    ok_t = sum(tags[16 * i:16 * i + 16].tobytes() == otags[16 * i:16 * i + 16].tobytes() for i in range(n))
    bad = np.nonzero(out != oout)[0]
    print(f"n={n} L={L} suite={suite:#x}: {dt * 1e3:.1f} ms, tags ok {ok_t}/{n}, bad bytes {len(bad)}"
          + (f" first at {bad[0]}" if len(bad) else ""), flush=True)


def main():
    eng = atls.Engine(0)
    for n, L in [(1, 16384), (2, 16384), (8, 16384), (64, 16384), (512, 16384), (4096, 16384)]:
        case(eng, n, L)
    case(eng, 64, 16384, 0x1302)
    eng.close()


if __name__ == "__main__":
    main()
