"""Key grouping of direct AES-GCM batches across key multiplicity and record length: device-resident
seal of n records of one length over n_keys connections (round-robin), timed with HIP events on the
engine stream, grouped (default engine) and ungrouped (ATLS_GCM_GROUP_MIN=0). One JSON line per
case. python tools/group_sweep.py [steps]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import anothertls_amd as atls  # noqa: E402
from anothertls_amd import workload  # noqa: E402


def time_seal(b, grouped, steps):
    os.environ["ATLS_GCM_GROUP_MIN"] = "2048" if grouped else "0"
    eng = atls.Engine(0)
    del os.environ["ATLS_GCM_GROUP_MIN"]
    eng.set_keys(b["keys"])
    dev = torch.device("cuda", 0)
    n = len(b["recs"])
    g = torch.Generator(device=dev).manual_seed(7)
    d_in = torch.randint(0, 256, (b["in_bytes"] + 16,), dtype=torch.uint8, device=dev, generator=g)
    d_out = torch.empty(b["out_bytes"] + 16, dtype=torch.uint8, device=dev)
    d_tags = torch.empty(16 * n, dtype=torch.uint8, device=dev)
    d_aux = torch.zeros(16, dtype=torch.uint8, device=dev)
    d_recs = torch.from_numpy(b["recs"].view(np.uint8).copy()).to(dev)
    flags = atls.FLAG_DEVICE_PTRS | atls.FLAG_DEVICE_RECS | atls.FLAG_NO_SYNC
    torch.cuda.synchronize()
    stream = torch.cuda.ExternalStream(eng.stream, device=dev)
    for _ in range(2):
        eng.seal_batch(d_recs.data_ptr(), d_in, d_aux, d_out, d_tags, flags=flags, n=n)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(steps):
        eng.seal_batch(d_recs.data_ptr(), d_in, d_aux, d_out, d_tags, flags=flags, n=n)
    e1.record(stream)
    eng.sync()
    ms = e0.elapsed_time(e1) / steps
    out = d_tags.cpu().numpy().tobytes()
    eng.close()
    return ms, out


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    for L, n in [(16384, 65536), (1536, 65536), (64, 65536), (256, 262144)]:
        for nk in (4096, n // 2, n):
            b = workload.tls_batch(n, L, 0x1301, n_keys=nk)
            mg, tg = time_seal(b, True, steps)
            mu, tu = time_seal(b, False, steps)
            gib = b["payload"] / 2**30
            print(json.dumps({"len": L, "records": n, "keys": nk, "grouped_ms": round(mg, 4), "ungrouped_ms": round(mu, 4),
                              "grouped_GiBps": round(gib / mg * 1e3, 1), "ungrouped_GiBps": round(gib / mu * 1e3, 1),
                              "tags_equal": tg == tu}), flush=True)


if __name__ == "__main__":
    main()
