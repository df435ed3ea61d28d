"""Device-resident OPEN throughput of a BASELINE config (the bench times seal): seal the batch once,
then time `steps` atls_open_batch launches with HIP events on the engine stream. Prints one JSON
line. python tools/open_bench.py [config] [steps]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import anothertls_amd as atls  # noqa: E402
from anothertls_amd import workload  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c3_chacha20poly1305_64Ki_x_1.5KiB"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    b = workload.shard_batch(cfg, 0)
    dev = torch.device("cuda", 0)
    eng = atls.Engine(0)
    eng.set_keys(b["keys"])
    n = len(b["recs"])
    g = torch.Generator(device=dev).manual_seed(workload.SEEDS["payload"])
    d_in = torch.randint(0, 256, (b["in_bytes"] + 16,), dtype=torch.uint8, device=dev, generator=g)
    d_ct = torch.empty(b["out_bytes"] + 16, dtype=torch.uint8, device=dev)
    d_tags = torch.empty(16 * n, dtype=torch.uint8, device=dev)
    d_aux = torch.zeros(16, dtype=torch.uint8, device=dev)
    eng.seal_batch(b["recs"], d_in, d_aux, d_ct, d_tags, flags=atls.FLAG_DEVICE_PTRS)
    orecs = b["recs"].copy()
    orecs["in_off"] = b["recs"]["out_off"]
    orecs["len"] = b["recs"]["len"] + 1
    d_recs = torch.from_numpy(orecs.view(np.uint8).copy()).to(dev)
    d_pt = torch.empty_like(d_ct)
    d_res = torch.empty(8 * n, dtype=torch.uint8, device=dev)
    flags = atls.FLAG_DEVICE_PTRS | atls.FLAG_DEVICE_RECS | atls.FLAG_NO_SYNC
    torch.cuda.synchronize()
    stream = torch.cuda.ExternalStream(eng.stream, device=dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for i in range(3 + steps):
        if i == 3:
            e0.record(stream)
        eng.open_batch(d_recs.data_ptr(), d_ct, d_aux, d_tags, d_pt, d_res, flags=flags, n=n)
    e1.record(stream)
    eng.sync()
    res = d_res.cpu().numpy().view(atls.OPEN_RESULT_DTYPE)
    assert (res["status"] == 0).all()
    ms = e0.elapsed_time(e1) / steps
    print(json.dumps({"config": cfg, "open_ms": round(ms, 4), "open_GiBps": round(b["payload"] / (ms * 1e-3) / 2**30, 2)}))


if __name__ == "__main__":
    main()
