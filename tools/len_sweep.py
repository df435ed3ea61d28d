"""Kernel time of one seal_batch vs record length (fixed record count): slope = per-64-slot-step
cost, intercept = per-record overhead. python tools/len_sweep.py [suite_hex] [n_records]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import anothertls_amd as atls  # noqa: E402
from anothertls_amd import workload  # noqa: E402


def main():
    suite = int(sys.argv[1], 16) if len(sys.argv) > 1 else 0x1301
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
    dev = torch.device("cuda", 0)
    eng = atls.Engine(0)
    flags = atls.FLAG_DEVICE_PTRS | atls.FLAG_DEVICE_RECS | atls.FLAG_NO_SYNC
    stream = torch.cuda.ExternalStream(eng.stream, device=dev)
    rows = []
    lens = [int(v) for v in os.environ.get("LENS", "1008,2032,4080,8176,12272,16368").split(",")]
    for clen in lens:  # default: 64, 128, 256, 512, 768, 1024 slots (+3)
        b = workload.tls_batch(n, clen, suite, n_keys=4096)
        eng.set_keys(b["keys"])
        d_in = torch.randint(0, 256, (b["in_bytes"],), dtype=torch.uint8, device=dev)
        d_out = torch.empty(b["out_bytes"], dtype=torch.uint8, device=dev)
        d_tags = torch.empty(16 * n, dtype=torch.uint8, device=dev)
        d_aux = torch.zeros(16, dtype=torch.uint8, device=dev)
        d_recs = torch.from_numpy(b["recs"].view(np.uint8).copy()).to(dev)
        for _ in range(2):
            eng.seal_batch(d_recs.data_ptr(), d_in, d_aux, d_out, d_tags, flags=flags, n=n)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(5):
            eng.seal_batch(d_recs.data_ptr(), d_in, d_aux, d_out, d_tags, flags=flags, n=n)
        e1.record(stream)
        eng.sync()
        ms = e0.elapsed_time(e1) / 5
        slots = (clen + 1 + 15) // 16 + 3
        rows.append((clen, slots, ms))
        print(f"content {clen:6d} B, {slots:5d} slots/record: {ms:.4f} ms, {b['payload'] / ms / 1e6:.1f} GB/s payload", flush=True)
    x = np.array([r[1] for r in rows], float)
    y = np.array([r[2] for r in rows], float)
    A = np.vstack([x, np.ones_like(x)]).T
    (slope, icpt), *_ = np.linalg.lstsq(A, y, rcond=None)
    print(f"fit: {slope * 64 * 1e3:.3f} us per 64-slot step (whole batch), {icpt * 1e3:.1f} us per launch fixed "
          f"({icpt / (slope * 64):.2f} step-equivalents per record)")
    eng.close()


if __name__ == "__main__":
    main()
