"""Time the key-grouping plan (plan.hip atls_launch_group: count, scan, scatter) alone on the device
for n records over n_keys slots, with HIP events on a torch stream. python tools/group_plan_time.py"""
import ctypes
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
    lib = atls.library()
    lib.atls_group_hdr_offset.restype = ctypes.c_size_t
    lib.atls_group_hdr_offset.argtypes = [ctypes.c_uint32]
    lib.atls_launch_group.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(device=dev)
    for n, nk in [(65536, 4096), (65536, 32768), (65536, 65536), (262144, 4096), (262144, 262144)]:
        b = workload.tls_batch(n, 64, 0x1301, n_keys=nk)
        d_recs = torch.from_numpy(b["recs"].view(np.uint8).copy()).to(dev)
        cnt = torch.zeros(2 * (nk + 1), dtype=torch.int32, device=dev)
        aux = torch.zeros(lib.atls_group_hdr_offset(nk) // 4 + 16 + n, dtype=torch.int32, device=dev)
        gidx = torch.zeros(n, dtype=torch.int32, device=dev)
        torch.cuda.synchronize()
        with torch.cuda.stream(s):
            args = (d_recs.data_ptr(), n, nk, cnt.data_ptr(), aux.data_ptr(), gidx.data_ptr(), 256, s.cuda_stream)
            lib.atls_launch_group(*args)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(20):
                lib.atls_launch_group(*args)
            e1.record(s)
        torch.cuda.synchronize()
        perm = np.sort(gidx.cpu().numpy())
        print(json.dumps({"records": n, "keys": nk, "plan_us": round(e0.elapsed_time(e1) / 20 * 1e3, 1),
                          "permutation": bool((perm == np.arange(n)).all())}), flush=True)


if __name__ == "__main__":
    main()
