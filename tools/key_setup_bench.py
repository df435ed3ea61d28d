"""Key installs (atls_update_keys -> csrc/keysetup.hip, one wave per key): the cost of a new key, which the
reference pays on every Cipher call (crypto/aes/gcm.rs:49-56 expands the key and computes H per call).
Prints one JSON object: host microseconds of a 1-key update (launch only, and launch + completion), a
4-key update, a 4,096-key install (staged copy + kernel + wait), and the key-setup kernel's own time from
HIP events on the engine stream for 1 and 4,096 AES-128 / AES-256 keys. Run under `rocprofv3 --kernel-trace
--stats` for the per-kernel averages (profiles/r04/keysetup_*). Needs a GPU."""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import anothertls_amd as atls  # noqa: E402
from anothertls_amd import workload  # noqa: E402


def _median_us(fn, reps):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return round(statistics.median(ts) * 1e6, 2)


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.init()
    out = {"what": "key installs: host us (median) and key-setup kernel ms (HIP events, engine stream)"}
    for suite, klen, name in [(0x1301, 16, "aes128"), (0x1302, 32, "aes256")]:
        keys = workload.make_keys(4096, np.full(4096, suite, np.uint16), key_lens=np.full(4096, klen))
        eng = atls.Engine(0)
        eng.set_keys(keys)
        it = {"i": 0}
        stream = torch.cuda.ExternalStream(eng.stream, device=dev)
        done = torch.cuda.Event()

        def one(wait, n=1):
            it["i"] = (it["i"] + 1) % 4000
            eng.update_keys(it["i"], keys[it["i"]:it["i"] + n])
            if wait:  # until the new schedule is in HBM: an event after the kernel (atls_engine_sync would
                done.record(stream)  # add its sticky-error-word read, a synchronous 4-byte copy)
                done.synchronize()

        out[f"{name}_update1_launch_us"] = _median_us(lambda: one(False), 500)
        eng.sync()
        out[f"{name}_update1_end_to_end_us"] = _median_us(lambda: one(True), 500)
        out[f"{name}_update4_end_to_end_us"] = _median_us(lambda: one(True, 4), 200)
        out[f"{name}_set4096_end_to_end_us"] = _median_us(lambda: eng.set_keys(keys), 50)
        for n, reps in ((1, 200), (4096, 20)):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            eng.sync()
            e0.record(stream)
            for r in range(reps):
                eng.update_keys(0, keys[:n])  # n = 4096: staged copy + kernel per call, waits each time
            e1.record(stream)
            eng.sync()
            torch.cuda.synchronize(dev)
            out[f"{name}_setup{n}_stream_ms"] = round(e0.elapsed_time(e1) / reps, 4)
        eng.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
