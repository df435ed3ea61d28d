"""Check atls_clock_probe against the in-kernel clock (MI355X_MICROARCH.md "DVFS give-back" item 6).

Needs the diagnostic build anothertls_amd/variants/libatls_clk.so (python tools/build_variants.py
clk=ATLS_CLK_STAMPS), loaded through ATLS_LIB. For each config, after ~1 s of back-to-back seals the
kernels' own stamps (every wave's s_memtime / s_memrealtime span over the kernel body) are reset, then
`--seconds` more seals run with the probe beside them; both clocks come from the same launches.

ATLS_LIB=anothertls_amd/variants/libatls_clk.so python tools/clock_check.py > out.json"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

NAMES = {"c2": "c2_aes128gcm_64Ki_x_16KiB", "c4": "c4_aes256gcm_1Mi_x_16KiB"}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--seconds", type=float, default=2.0)
    p.add_argument("--configs", default="c2,c2z,c4,c2k")
    args = p.parse_args()
    import anothertls_amd as atls
    from anothertls_amd import workload

    lib = atls.library()
    lib.atls_debug_clk_stamps.argtypes = [ctypes.c_void_p]
    flags_build = lib.atls_build_flags()
    assert flags_build & 64, "not a -DATLS_CLK_STAMPS build (set ATLS_LIB)"
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    eng = atls.Engine(0)
    stamps = np.zeros(4, np.uint64)
    out = {"library": os.environ.get("ATLS_LIB"), "runs": []}
    for c in args.configs.split(","):
        key = c.rstrip("zk")
        zero, per_record_key = "z" in c[2:], "k" in c[2:]
        name = NAMES[key]
        n0 = workload.records_per_rank(name)
        batch = workload.shard_batch(name, 0, n_keys=n0 if per_record_key else None)
        recs = batch["recs"]
        n = len(recs)
        eng.set_keys(batch["keys"])
        g = torch.Generator(device=dev).manual_seed(workload.SEEDS["payload"])
        d_in = (torch.zeros(batch["in_bytes"], dtype=torch.uint8, device=dev) if zero else
                torch.randint(0, 256, (batch["in_bytes"],), dtype=torch.uint8, device=dev, generator=g))
        d_out = torch.empty(batch["out_bytes"], dtype=torch.uint8, device=dev)
        d_tags = torch.empty(16 * n, dtype=torch.uint8, device=dev)
        d_aux = torch.zeros(16, dtype=torch.uint8, device=dev)
        d_recs = torch.from_numpy(recs.view(np.uint8).copy()).to(dev)
        torch.cuda.synchronize(dev)
        fl = atls.FLAG_DEVICE_PTRS | atls.FLAG_DEVICE_RECS | atls.FLAG_NO_SYNC
        ptrs = [t.data_ptr() for t in (d_recs, d_in, d_aux, d_out, d_tags)]

        def launch():
            eng.seal_batch(ptrs[0], ptrs[1], ptrs[2], ptrs[3], ptrs[4], flags=fl, n=n)

        stream = torch.cuda.ExternalStream(eng.stream, device=dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(10):
            launch()
        e1.record(stream)
        eng.sync()
        k_ms = e0.elapsed_time(e1) / 10
        for _ in range(int(1.0e3 / k_ms)):  # ~1 s of load first
            launch()
        eng.sync()
        assert lib.atls_debug_clk_stamps(stamps.ctypes.data) == 0  # reset
        n_launch = max(10, int(args.seconds * 1e3 / k_ms))
        probe = torch.zeros(32, dtype=torch.int64, device=dev)
        side = torch.cuda.Stream(device=dev)
        span = n_launch * k_ms * 1e3
        eng.clock_probe(probe, wgs=16, delay_us=int(0.05 * span), spin_us=int(0.9 * span), stream=side.cuda_stream)
        e0.record(stream)
        for _ in range(n_launch):
            launch()
        e1.record(stream)
        eng.sync()
        torch.cuda.synchronize(dev)
        assert lib.atls_debug_clk_stamps(stamps.ctypes.data) == 0
        o = probe.cpu().numpy().reshape(16, 2).astype(np.float64)
        pr = (100.0 * o[:, 0] / np.maximum(o[:, 1], 1))
        ms = e0.elapsed_time(e1) / n_launch
        r = {"config": name, "zero_payload": zero, "key_per_record": per_record_key, "launches": n_launch,
             "kernel_ms": round(ms, 4), "in_kernel_MHz": round(100.0 * float(stamps[0]) / max(float(stamps[1]), 1.0), 1),
             "in_kernel_waves": int(stamps[2]), "wave_busy_frac": round(float(stamps[1]) * 10e-9 / max(stamps[2], 1) /
                                                                         (ms * 1e-3), 4),
             "probe_MHz_median": round(float(np.median(pr)), 1), "probe_MHz_all": pr.round(1).tolist()}
        print(json.dumps({k: r[k] for k in ("config", "zero_payload", "key_per_record", "kernel_ms", "in_kernel_MHz",
                                            "probe_MHz_median")}), file=sys.stderr, flush=True)
        out["runs"].append(r)
        del d_in, d_out, d_tags, d_recs
        torch.cuda.empty_cache()
    eng.close()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
