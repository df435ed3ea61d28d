"""Phase clocks of the AES-GCM single call (gcm_single, one record per call) from a -DATLS_TT_STAMPS build
(ATLS_LIB=anothertls_amd/variants/libatls_ttstamps.so): shader-clock cycles per call in the record's setup
(GHASH table, counter cache), fast steps, general steps and lane combine + tag, and the host median per
call. Prints one JSON object. Needs a GPU."""
import ctypes
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import anothertls_amd as atls  # noqa: E402


def main():
    fn = atls.library().atls_debug_tt_stamps
    fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
    buf = (ctypes.c_ulonglong * 16)()
    if fn(buf) != 0:
        sys.exit("not a -DATLS_TT_STAMPS build (set ATLS_LIB)")
    out = {"what": "AES-GCM single call: shader-clock cycles per call by phase (gcm_record TT_STAMPS)"}
    for klen in (16, 32):
        c = atls.Gcm()
        key, iv, aad = bytes(range(klen)), bytes(12), b"\x17\x03\x03\x06\x11"
        for n in (64, 1537, 3000):
            pt = os.urandom(n)
            for _ in range(20):
                c.encrypt(key, iv, pt, aad)
            fn(buf)
            ts = []
            for _ in range(300):
                t0 = time.perf_counter()
                c.encrypt(key, iv, pt, aad)
                ts.append(time.perf_counter() - t0)
            fn(buf)
            r = buf[4] or 1
            out[f"aes{klen * 8}_{n}"] = {"host_median_us": round(statistics.median(ts) * 1e6, 2), "calls": buf[4],
                                        "fast_steps_per_call": buf[5] / r, "general_steps_per_call": buf[6] / r,
                                        "cycles": {nm: round(buf[i] / r) for i, nm in
                                                   enumerate(["setup", "fast_steps", "general_steps", "combine_tag"])}}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
