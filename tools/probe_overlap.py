"""Does the clock probe run beside a config's timed seals? (round 6: C4's whole batch read an idle clock and its
timed wall stretched by the probe's span, as if the probe ran after the seals.)

For each config: K seals on the engine stream with the probe enqueued on a side stream (a) before the first seal,
(b) after the first seal; HIP events give each probe's start / end relative to the window. One JSON line per case.
python tools/probe_overlap.py [--configs c2_aes128gcm_64Ki_x_16KiB:0,c4_aes256gcm_1Mi_x_16KiB:1048576]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--configs", default="c2_aes128gcm_64Ki_x_16KiB:0,c4_aes256gcm_1Mi_x_16KiB:1048576")
    p.add_argument("--steps", type=int, default=5)
    args = p.parse_args()
    import anothertls_amd as atls
    from anothertls_amd import workload

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    eng = atls.Engine(0)
    out = torch.zeros(32, dtype=torch.int64, device=dev)
    side = torch.cuda.Stream(device=dev)
    stream = torch.cuda.ExternalStream(eng.stream, device=dev)
    eng.clock_probe(out, wgs=16, delay_us=0, spin_us=1, stream=side.cuda_stream)
    torch.cuda.synchronize(dev)
    for tok in args.configs.split(","):
        name, _, recs = tok.partition(":")
        batch = workload.shard_batch(name, 0, n=int(recs) or None)
        n = len(batch["recs"])
        eng.set_keys(batch["keys"])
        d_in = torch.randint(0, 256, (batch["in_bytes"],), dtype=torch.uint8, device=dev)
        d_out = torch.empty(batch["out_bytes"], dtype=torch.uint8, device=dev)
        d_tags = torch.empty(16 * n, dtype=torch.uint8, device=dev)
        d_aux = torch.zeros(16, dtype=torch.uint8, device=dev)
        d_recs = torch.from_numpy(batch["recs"].view(np.uint8).copy()).to(dev)
        flags = atls.FLAG_DEVICE_PTRS | atls.FLAG_DEVICE_RECS | atls.FLAG_NO_SYNC
        ptrs = [t.data_ptr() for t in (d_recs, d_in, d_aux, d_out, d_tags)]

        def seal():
            eng.seal_batch(*ptrs, flags=flags, n=n)

        for _ in range(3):
            seal()
        eng.sync()
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        seal()
        e1.record(stream)
        torch.cuda.synchronize(dev)
        one = e0.elapsed_time(e1)
        for case in ("before", "after_first"):
            span_us = args.steps * one * 1e3
            w0, w1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            p0, p1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

            def probe():
                p0.record(side)
                eng.clock_probe(out, wgs=16, delay_us=int(0.15 * span_us), spin_us=max(20, int(0.7 * span_us)),
                                stream=side.cuda_stream)
                p1.record(side)

            if case == "before":
                probe()
            w0.record(stream)
            for i in range(args.steps):
                seal()
                if case == "after_first" and i == 0:
                    probe()
            w1.record(stream)
            torch.cuda.synchronize(dev)
            o = out.cpu().numpy().reshape(16, 2).astype(np.float64)
            print(json.dumps({"config": name, "records": n, "case": case, "launch_ms": round(one, 3),
                              "window_ms": round(w0.elapsed_time(w1), 3),
                              "probe_start_ms": round(w0.elapsed_time(p0), 3) if case == "after_first" else round(-p0.elapsed_time(w0), 3),
                              "probe_end_ms": round(w0.elapsed_time(p1), 3),
                              "probe_span_ms": round(p0.elapsed_time(p1), 3),
                              "sclk_MHz": round(float(np.median(100.0 * o[:, 0] / np.maximum(o[:, 1], 1))), 1)}), flush=True)
        del d_in, d_out, d_tags, d_recs
        torch.cuda.empty_cache()
    eng.close()


if __name__ == "__main__":
    main()
