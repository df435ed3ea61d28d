"""Clock and power of the record kernels under sustained load, one config after another on one box
(why does gcm_kernel run at ~2.0 GHz where the ChaCha20-Poly1305 kernels run at ~2.36?).

For each config: seal the bench's device-resident batch back to back for --seconds while
  * a thread samples the board's hwmon files every 10 ms (sclk freq1_input, power1_input, temperatures),
  * `amd-smi metric -p -c --json` is sampled once a second (per-XCD gfx clocks, socket power),
  * the in-kernel clock probe (atls_clock_probe, 16 one-wave workgroups on a second stream beside the
    launches) reads s_memtime against s_memrealtime over the middle of the window (every workgroup kept);
the launches are timed with HIP events. Variants: the payload all zero (less toggling energy per block)
as the data-dependence check of MI355X_MICROARCH.md "DVFS give-back" (1).

python tools/clock_power.py [--seconds 4] [--configs c2,c3,...] > out.json"""
import argparse
import glob
import json
import os
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

NAMES = {"c2": "c2_aes128gcm_64Ki_x_16KiB", "c3": "c3_chacha20poly1305_64Ki_x_1.5KiB",
         "c4": "c4_aes256gcm_1Mi_x_16KiB", "c5": "c5_mixed_256Ki_x_64B-16KiB"}


def hwmon_dir():
    for d in sorted(glob.glob("/sys/class/drm/card*/device/hwmon/hwmon*")):
        if os.path.exists(os.path.join(d, "freq1_input")) and os.path.exists(os.path.join(d, "power1_input")):
            return d
    return None


def read_int(path):
    try:
        with open(path) as f:
            return int(f.read().strip())
    except (OSError, ValueError):
        return None


class Sampler(threading.Thread):
    def __init__(self, hw, period=0.01):
        super().__init__(daemon=True)
        self.hw, self.period, self.rows, self.stop = hw, period, [], threading.Event()

    def run(self):
        t0 = time.perf_counter()
        while not self.stop.is_set():
            r = [time.perf_counter() - t0]
            for f in ("freq1_input", "power1_input", "temp2_input", "temp3_input"):
                r.append(read_int(os.path.join(self.hw, f)) if self.hw else None)
            self.rows.append(r)
            time.sleep(self.period)


def amdsmi_samples(seconds, out):
    """amd-smi metric once a second (per-XCD clocks and socket power), appended to `out`."""
    t_end = time.perf_counter() + seconds
    while time.perf_counter() < t_end:
        try:
            p = subprocess.run(["amd-smi", "metric", "-p", "-c", "--json"], capture_output=True, text=True, timeout=20)
            j = json.loads(p.stdout)
            g = j["gpu_data"][0] if isinstance(j, dict) else j[0]
            clk = {k: v["clk"]["value"] for k, v in g["clock"].items() if k.startswith("gfx_") and isinstance(v, dict)}
            pw = g["power"]["socket_power"]["value"]
            out.append({"t": time.perf_counter(), "gfx_MHz": clk, "socket_W": pw,
                        "throttle": g["power"].get("throttle_status")})
        except Exception as ex:  # noqa: BLE001 -- a missing tool or format change leaves this list short
            out.append({"error": str(ex)[:200]})
            return
        time.sleep(0.5)


def stats(xs):
    xs = [x for x in xs if x is not None]
    if not xs:
        return None
    a = np.asarray(xs, np.float64)
    return {"median": float(np.median(a)), "p10": float(np.percentile(a, 10)), "p90": float(np.percentile(a, 90)),
            "n": len(xs)}


def run_one(eng, dev, key, zero, seconds, hw):
    import anothertls_amd as atls
    from anothertls_amd import workload

    name = NAMES[key]
    batch = workload.shard_batch(name, 0)
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
    flags = atls.FLAG_DEVICE_PTRS | atls.FLAG_DEVICE_RECS | atls.FLAG_NO_SYNC | atls.FLAG_LAZY_JOIN
    ptrs = [t.data_ptr() for t in (d_recs, d_in, d_aux, d_out, d_tags)]

    def launch():
        eng.seal_batch(ptrs[0], ptrs[1], ptrs[2], ptrs[3], ptrs[4], flags=flags, n=n)

    for _ in range(20):
        launch()
    eng.sync()
    stream = torch.cuda.ExternalStream(eng.stream, device=dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    eng.join()
    e0.record(stream)
    for _ in range(10):
        launch()
    eng.join()
    e1.record(stream)
    torch.cuda.synchronize(dev)
    k_ms = e0.elapsed_time(e1) / 10
    n_launch = max(10, int(seconds * 1e3 / k_ms))
    probe = torch.zeros(32, dtype=torch.int64, device=dev)
    side = torch.cuda.Stream(device=dev)
    span_us = n_launch * k_ms * 1e3
    samp = Sampler(hw)
    smi = []
    th = threading.Thread(target=amdsmi_samples, args=(seconds * 0.9, smi), daemon=True)
    samp.start()
    time.sleep(0.3)  # idle-ish baseline rows before the load starts
    t_load0 = samp.rows[-1][0] if samp.rows else 0.0
    eng.clock_probe(probe, wgs=16, delay_us=int(0.25 * span_us), spin_us=int(0.5 * span_us), stream=side.cuda_stream)
    eng.join()
    e0.record(stream)
    th.start()  # amd-smi samples from the first launch on (the enqueue loop below blocks once the queue is full)
    for _ in range(n_launch):
        launch()
    eng.join()
    e1.record(stream)
    torch.cuda.synchronize(dev)
    t_load1 = samp.rows[-1][0]
    time.sleep(0.3)
    samp.stop.set()
    samp.join()
    th.join(timeout=30)
    ms = e0.elapsed_time(e1) / n_launch
    o = probe.cpu().numpy().reshape(16, 2).astype(np.float64)
    probe_mhz = (100.0 * o[:, 0] / np.maximum(o[:, 1], 1)).round(1).tolist()
    # hwmon rows over the middle half of the load window
    a, b = t_load0 + 0.25 * (t_load1 - t_load0), t_load0 + 0.75 * (t_load1 - t_load0)
    mid = [r for r in samp.rows if a <= r[0] <= b]
    alg = 2 * batch["payload"] + 16 * n
    xcd = {}
    for s in smi:
        for k, v in s.get("gfx_MHz", {}).items():
            xcd.setdefault(k, []).append(v)
    res = {"config": name, "zero_payload": zero, "launches": n_launch, "kernel_ms": round(ms, 4),
           "frac_hbm": round(alg / (ms * 1e-3) / 8e12, 4),
           "probe_MHz_median": float(np.median(probe_mhz)), "probe_MHz_all": probe_mhz,
           "hwmon_sclk_MHz": stats([r[1] / 1e6 if r[1] else None for r in mid]),
           "hwmon_power_W": stats([r[2] / 1e6 if r[2] else None for r in mid]),
           "hwmon_temp2_mC": stats([r[3] for r in mid]), "hwmon_temp3_mC": stats([r[4] for r in mid]),
           "amdsmi_socket_W": stats([s.get("socket_W") for s in smi]),
           "amdsmi_gfx_MHz_median_per_xcd": {k: float(np.median(v)) for k, v in sorted(xcd.items())},
           "amdsmi_samples": len(smi), "hwmon_rows_mid": len(mid)}
    del d_in, d_out, d_tags, d_recs
    torch.cuda.empty_cache()
    return res


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--seconds", type=float, default=8.0)
    p.add_argument("--configs", default="c2,c3,c2z,c3z,c4,c5")
    args = p.parse_args()
    import anothertls_amd as atls

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    eng = atls.Engine(0)
    hw = hwmon_dir()
    out = {"hwmon": hw, "power1_cap_W": (read_int(os.path.join(hw, "power1_cap")) or 0) / 1e6 if hw else None,
           "device": torch.cuda.get_device_name(dev), "runs": []}
    # bring the clock out of idle first
    x = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
    for _ in range(200):
        x.add_(1)
    torch.cuda.synchronize(dev)
    del x
    for c in args.configs.split(","):
        key, zero = c.rstrip("z"), c.endswith("z")
        r = run_one(eng, dev, key, zero, args.seconds, hw)
        print(json.dumps({k: r[k] for k in ("config", "zero_payload", "kernel_ms", "probe_MHz_median")}),
              file=sys.stderr, flush=True)
        out["runs"].append(r)
    eng.close()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
