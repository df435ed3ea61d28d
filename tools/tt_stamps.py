"""Phase breakdown of the T-table AES-GCM kernel (gcm.hip built with -DATLS_TT_STAMPS).

python tools/tt_stamps.py [config [n_keys]]   (build first on the host:
python -c "import anothertls_amd._build as b; b.build(defines=('ATLS_TT_STAMPS',),
out='anothertls_amd/variants/libatls_ttstamps.so')")
Prints average shader-clock cycles per record (per wave) in each phase."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("ATLS_LIB", os.path.join(ROOT, "anothertls_amd", "variants", "libatls_ttstamps.so"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import anothertls_amd as atls  # noqa: E402
from anothertls_amd import workload  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c2_aes128gcm_64Ki_x_16KiB"
    batch = workload.config_batch(cfg, n_keys=int(sys.argv[2]) if len(sys.argv) > 2 else None)
    n = len(batch["recs"])
    dev = torch.device("cuda", 0)
    eng = atls.Engine(0)
    eng.set_keys(batch["keys"])
    d_in = torch.randint(0, 256, (batch["in_bytes"],), dtype=torch.uint8, device=dev)
    d_out = torch.empty(batch["out_bytes"], dtype=torch.uint8, device=dev)
    d_tags = torch.empty(16 * n, dtype=torch.uint8, device=dev)
    d_aux = torch.zeros(16, dtype=torch.uint8, device=dev)
    d_recs = torch.from_numpy(batch["recs"].view("u1").copy()).to(dev)
    torch.cuda.synchronize()
    fn = atls.library().atls_debug_tt_stamps
    fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
    buf = (ctypes.c_ulonglong * 16)()
    flags = atls.FLAG_DEVICE_PTRS | atls.FLAG_DEVICE_RECS
    eng.seal_batch(d_recs.data_ptr(), d_in, d_aux, d_out, d_tags, flags=flags, n=n)
    assert fn(buf) == 0, "library was not built with -DATLS_TT_STAMPS"
    for _ in range(3):
        eng.seal_batch(d_recs.data_ptr(), d_in, d_aux, d_out, d_tags, flags=flags, n=n)
    fn(buf)
    recs = buf[4] or 1
    print(f"{cfg} ({len(batch['keys'])} keys): {recs} record-runs, {buf[5] / recs:.2f} fast + {buf[6] / recs:.2f} general steps per record")
    tot = sum(buf[i] for i in range(4))
    for i, nm in enumerate(["setup", "fast steps", "general steps", "combine+tag"]):
        print(f"  {nm:14s} {buf[i] / recs:10.0f} cycles/record  {100 * buf[i] / max(tot, 1):5.1f} %")
    print(f"  per fast step {buf[1] / max(buf[5], 1):8.0f} cycles, per general step {buf[2] / max(buf[6], 1):8.0f}")
    print(f"  {'total':14s} {tot / recs:10.0f} cycles/record")
    g0 = buf[12] or 1
    gl = max(buf[6] - buf[12], 1)
    print(f"  general steps: first {buf[8] / g0:8.0f} cycles ({buf[12]}), later {buf[9] / gl:8.0f} cycles ({buf[6] - buf[12]});"
          f" per general step: loads landed after {buf[10] / max(buf[6], 1):8.0f}, AES {buf[11] / max(buf[6], 1):8.0f}")
    eng.close()


if __name__ == "__main__":
    main()
