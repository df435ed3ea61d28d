"""Where a single ChaCha20-Poly1305 Cipher-trait call's time goes: run with ATLS_LIB pointing
at a -DATLS_LAT_STAMPS build (anothertls_amd/variants/libatls_latstamps.so, tools/recipes/r4_single.sh).
The kernel's lane 0 adds the shader clock at each phase end to a device array (after waiting for its
outstanding memory operations); the real-time clock at entry / exit calibrates cycles to microseconds.
Prints one JSON object: the host-side median per call and the mean kernel phases. Needs a GPU.
The phase stamps sit in the one-wave record (chacha_record G = 64), which the single call used until the
4-wave record replaced it later in round 4 (G = 256); profiles/r04/single_call_stamps.json is from then."""
import ctypes
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import anothertls_amd as atls  # noqa: E402

PHASES = ["args_and_key_schedule", "data_loads", "keystream", "r_powers", "slot_xor_store_mac", "combine_tag",
          "stores_drained"]


def main():
    lib = atls.library()
    lib.atls_debug_lat_stamps.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
    buf = (ctypes.c_ulonglong * 16)()
    if lib.atls_debug_lat_stamps(buf) != 0:
        sys.exit("not a -DATLS_LAT_STAMPS build (set ATLS_LIB)")
    out = {"what": "ChaCha20-Poly1305 atls_seal / atls_open of one record, phase clocks of the single-call kernel"}
    c = atls.Poly1305()
    key, iv, aad = bytes(range(32)), bytes(12), b"\x17\x03\x03\x06\x11"
    for n in (64, 1537, 3000):
        pt = os.urandom(n)
        for op in ("seal", "open"):
            ct, tag = c.encrypt(key, iv, pt, aad)
            call = (lambda: c.encrypt(key, iv, pt, aad)) if op == "seal" else (lambda: c.decrypt(key, iv, ct, aad, tag))
            for _ in range(20):
                call()
            lib.atls_debug_lat_stamps(buf)  # reset
            ts = []
            for _ in range(500):
                t0 = time.perf_counter()
                call()
                ts.append(time.perf_counter() - t0)
            assert lib.atls_debug_lat_stamps(buf) == 0
            v = list(buf)
            calls = v[15]
            assert calls == 500, calls
            cyc = (v[7] - v[0]) / calls
            rt_us = (v[9] - v[8]) / calls / 100.0  # 100 MHz real-time clock
            mhz = cyc / rt_us if rt_us else 0.0
            ph = {PHASES[i - 1]: round((v[i] - v[i - 1]) / calls / mhz, 3) for i in range(1, 8)}
            out[f"{op}_{n}"] = {"host_median_us": round(statistics.median(ts) * 1e6, 2),
                                "kernel_entry_to_exit_us": round(rt_us, 3), "shader_clock_MHz": round(mhz, 1),
                                "phases_us": ph}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
