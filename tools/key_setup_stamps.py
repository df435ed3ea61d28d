"""Where a single key install's time goes (round 4): run with ATLS_LIB pointing at a -DATLS_KS_STAMPS build.
Lane 0 of the first workgroup adds the shader clock at each phase end of the key-setup kernel (after its
memory operations) to a device array; the real-time clock calibrates. Prints one JSON object per key size:
host microseconds of update_keys(1 key) + a wait on an event behind it, and the kernel's phases. Needs a GPU."""
import ctypes
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

PHASES = ["t0_table_to_lds", "key_args_chacha_words", "expansion_and_H", "round_key_stores", "scan_level_1",
          "scan_levels_2_to_6", "seeds_and_stores"]


def main():
    lib = atls.library()
    lib.atls_debug_ks_stamps.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
    buf = (ctypes.c_ulonglong * 16)()
    if lib.atls_debug_ks_stamps(buf) != 0:
        sys.exit("not a -DATLS_KS_STAMPS build (set ATLS_LIB)")
    dev = torch.device("cuda", 0)
    out = {"what": "atls_update_keys of one key slot: host us (update + event wait) and kernel phases (us)",
           "lib": os.path.basename(atls.LIB_PATH)}
    for suite, klen, name in [(0x1301, 16, "aes128"), (0x1302, 32, "aes256")]:
        keys = workload.make_keys(64, np.full(64, suite, np.uint16), key_lens=np.full(64, klen))
        eng = atls.Engine(0)
        eng.set_keys(keys)
        stream = torch.cuda.ExternalStream(eng.stream, device=dev)
        ev = torch.cuda.Event()
        it = {"i": 0}

        def one():
            it["i"] = (it["i"] + 1) % 64
            eng.update_keys(it["i"], keys[it["i"]:it["i"] + 1])
            ev.record(stream)
            ev.synchronize()

        for _ in range(20):
            one()
        lib.atls_debug_ks_stamps(buf)
        ts = []
        for _ in range(300):
            t0 = time.perf_counter()
            one()
            ts.append(time.perf_counter() - t0)
        assert lib.atls_debug_ks_stamps(buf) == 0
        v = list(buf)
        calls = v[13]
        rt_us = (v[15] - v[14]) / calls / 100.0
        cyc = (v[7] - v[0]) / calls
        mhz = cyc / rt_us if rt_us else 0.0
        out[name] = {"host_median_us": round(statistics.median(ts) * 1e6, 2), "launches": calls,
                     "kernel_entry_to_exit_us": round(rt_us, 3), "shader_clock_MHz": round(mhz, 1),
                     "phases_us": {PHASES[i - 1]: round((v[i] - v[i - 1]) / calls / mhz, 3) for i in range(1, 8)}}
        eng.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
