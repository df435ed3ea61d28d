"""Co-residency experiment: the real AES-GCM seal kernel (C2 batch, engine stream) launched
together with a VALU-only bitsliced-AES burn kernel (tools/ubench/libbs_burn.so) on a second
stream. Prints each alone and both together (ms). Build the burn library first:
hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/ubench/bs_burn.hip -o tools/ubench/libbs_burn.so"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import anothertls_amd as atls  # noqa: E402
from anothertls_amd import workload  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    burn = ctypes.CDLL(os.path.join(ROOT, "tools", "ubench", "libbs_burn.so"))
    burn.bs_burn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    b = workload.config_batch("c2_aes128gcm_64Ki_x_16KiB")
    n = len(b["recs"])
    eng = atls.Engine(0)
    eng.set_keys(b["keys"])
    d_in = torch.randint(0, 256, (b["in_bytes"],), dtype=torch.uint8, device=dev)
    d_out = torch.empty(b["out_bytes"], dtype=torch.uint8, device=dev)
    d_tags = torch.empty(16 * n, dtype=torch.uint8, device=dev)
    d_aux = torch.zeros(16, dtype=torch.uint8, device=dev)
    d_recs = torch.from_numpy(b["recs"].view(np.uint8).copy()).to(dev)
    masks = torch.full((1024,), 0x5a5a5a5a, dtype=torch.int32, device=dev)
    bout = torch.empty(256 * 64 * 1024, dtype=torch.int32, device=dev)
    flags = atls.FLAG_DEVICE_PTRS | atls.FLAG_DEVICE_RECS | atls.FLAG_NO_SYNC
    s_gcm = torch.cuda.ExternalStream(eng.stream, device=dev)
    s_b = torch.cuda.Stream(device=dev)
    g = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    grid = int(sys.argv[2]) if len(sys.argv) > 2 else 512
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 8

    def gcm():
        eng.seal_batch(d_recs.data_ptr(), d_in, d_aux, d_out, d_tags, flags=flags, n=n)

    def bs():
        burn.bs_burn(s_b.cuda_stream, g, grid, iters, masks.data_ptr(), bout.data_ptr())

    def timed(fn_list, reps=5):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        s_gcm.wait_event(e0)
        s_b.wait_event(e0)
        for _ in range(reps):
            for f in fn_list:
                f()
        ea, eb = torch.cuda.Event(), torch.cuda.Event()
        ea.record(s_gcm)
        eb.record(s_b)
        torch.cuda.current_stream().wait_event(ea)
        torch.cuda.current_stream().wait_event(eb)
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps

    timed([gcm, bs], 1)
    ta, tb, tab = timed([gcm]), timed([bs]), timed([gcm, bs])
    print(f"G={g} grid={grid} iters={iters}: gcm {ta:.3f} ms, bs {tb:.3f} ms, together {tab:.3f} ms "
          f"(sum {ta + tb:.3f}, max {max(ta, tb):.3f})", flush=True)
    eng.close()


if __name__ == "__main__":
    main()
