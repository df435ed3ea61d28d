"""Time one engine batch from page-locked host memory in the shapes the socket path uses (C1 at scale: 64
connections x 64 WIRE records of 16 KiB per flush, a key slot pair per connection), against the bench's
C2-from-pinned-memory shape, to find what bounds atls_sb_flush / atls_sb_open_pending.
python tools/host_batch_probe.py -> JSON lines."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def pinned(n):
    return torch.empty(max(n, 16), dtype=torch.uint8, pin_memory=True).numpy()


def main():
    import anothertls_amd as atls
    from anothertls_amd import workload

    eng = atls.Engine(0)
    for conns, keys_per_conn, mode in ((64, 2, "wire"), (64, 2, "tls"), (64, 1, "wire"), (1, 1, "wire")):
        n = conns * 64
        # records of connection c are 64 consecutive entries, all with its write slot 2c
        b = workload.tls_batch(n, 16384, 0x1301, n_keys=conns * keys_per_conn)
        r = b["recs"]
        r["key_slot"] = (np.arange(n) // 64) * keys_per_conn
        r["seq"] = np.arange(n) % 64
        if mode == "wire":
            b = workload.wire_batch(b)
            r = b["recs"]
        eng.set_keys(b["keys"])
        h_in, h_out, h_tags = pinned(b["in_bytes"] + 16), pinned(b["out_bytes"] + 16), pinned(16 * n)
        h_in[:] = np.random.default_rng(1).integers(0, 256, h_in.size, dtype=np.uint8)
        aux = np.zeros(16, np.uint8)
        for _ in range(2):
            eng.seal_batch(r, h_in, aux, h_out, h_tags)
        t0 = time.perf_counter()
        reps = 10
        for _ in range(reps):
            eng.seal_batch(r, h_in, aux, h_out, h_tags)
        dt = (time.perf_counter() - t0) / reps
        print(json.dumps({"conns": conns, "key_slots": conns * keys_per_conn, "mode": mode, "records": n,
                          "ms_per_batch": round(dt * 1e3, 3), "GBps": round(b["in_bytes"] / dt / 1e9, 2)}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
