"""Is the AES-GCM open kernel slower than the seal, or slower where the bench times it (after the seals)?
C2, device-resident: seal once, then alternate blocks of 20 opens and 20 seals (HIP events on the engine stream,
each block after the previous one has finished), 4 times, and print ms per launch of each block.
python tools/open_order_probe.py [config]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    import anothertls_amd as atls
    from anothertls_amd import workload

    sys.path.insert(0, ROOT)
    import bench

    name = sys.argv[1] if len(sys.argv) > 1 else "c2_aes128gcm_64Ki_x_16KiB"
    dev = torch.device("cuda", 0)
    eng = atls.Engine(0)
    batch = workload.shard_batch(name, 0)
    recs = batch["recs"]
    n = len(recs)
    eng.set_keys(batch["keys"])
    g = torch.Generator(device=dev).manual_seed(workload.SEEDS["payload"])
    d_in = torch.randint(0, 256, (batch["in_bytes"],), dtype=torch.uint8, device=dev, generator=g)
    d_out = torch.empty(batch["out_bytes"], dtype=torch.uint8, device=dev)
    d_tags = torch.empty(16 * n, dtype=torch.uint8, device=dev)
    d_aux = torch.zeros(16, dtype=torch.uint8, device=dev)
    d_recs = torch.from_numpy(recs.view(np.uint8).copy()).to(dev)
    d_orecs = torch.from_numpy(bench.open_descs(recs).view(np.uint8).copy()).to(dev)
    d_pt = torch.zeros(batch["out_bytes"], dtype=torch.uint8, device=dev)
    d_res = torch.zeros(8 * n, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize(dev)
    flags = atls.FLAG_DEVICE_PTRS | atls.FLAG_DEVICE_RECS | atls.FLAG_NO_SYNC
    P = {k: t.data_ptr() for k, t in dict(recs=d_recs, inp=d_in, aux=d_aux, out=d_out, tags=d_tags, orecs=d_orecs,
                                           pt=d_pt, res=d_res).items()}
    stream = torch.cuda.ExternalStream(eng.stream, device=dev)

    def seal():
        eng.seal_batch(P["recs"], P["inp"], P["aux"], P["out"], P["tags"], flags=flags, n=n)

    def open_():
        eng.open_batch(P["orecs"], P["out"], P["aux"], P["tags"], P["pt"], P["res"], flags=flags, n=n)

    for _ in range(100):  # the clock up under load, and sealed records to open
        seal()
    eng.sync()
    torch.cuda.synchronize(dev)
    out = []
    for rnd in range(4):
        for what, f in (("open", open_), ("seal", seal)):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            eng.join()
            e0.record(stream)
            for _ in range(20):
                f()
            eng.join()
            e1.record(stream)
            eng.sync()
            torch.cuda.synchronize(dev)
            out.append({"round": rnd, "kernel": what, "ms": round(e0.elapsed_time(e1) / 20, 4)})
    res = d_res.cpu().numpy().view(atls.OPEN_RESULT_DTYPE)
    print(json.dumps({"config": name, "blocks": out, "open_status_ok": bool((res["status"] == 0).all())}))
    eng.close()


if __name__ == "__main__":
    main()
