"""Phase breakdown of the bitsliced AES-GCM kernel (gcm_bs.hip built with -DATLS_BS_STAMPS).

python tools/bs_stamps.py   (builds anothertls_amd/variants/libatls_stamps.so on the host first:
python -c "import anothertls_amd._build as b; b.build(defines=('ATLS_BS_STAMPS',),
out='anothertls_amd/variants/libatls_stamps.so')")
Prints the average shader-clock cycles per record pair and wave in each phase."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("ATLS_LIB", os.path.join(ROOT, "anothertls_amd", "variants", "libatls_stamps.so"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import anothertls_amd as atls  # noqa: E402
from anothertls_amd import workload  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c2_aes128gcm_64Ki_x_16KiB"
    batch = workload.config_batch(cfg)
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
    lib = atls.library()
    fn = lib.atls_debug_bs_stamps
    fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
    buf = (ctypes.c_ulonglong * 8)()
    flags = atls.FLAG_DEVICE_PTRS | atls.FLAG_DEVICE_RECS
    eng.seal_batch(d_recs.data_ptr(), d_in, d_aux, d_out, d_tags, flags=flags, n=n)
    assert fn(buf) == 0, "library was not built with -DATLS_BS_STAMPS"
    for _ in range(3):
        eng.seal_batch(d_recs.data_ptr(), d_in, d_aux, d_out, d_tags, flags=flags, n=n)
    fn(buf)
    pairs = buf[5] or 1
    names = ["setup", "rounds+transpose", "data+ghash", "tails", "combine"]
    tot = sum(buf[i] for i in range(5))
    print(f"{cfg}: {pairs} pair-runs")
    for i, nm in enumerate(names):
        print(f"  {nm:18s} {buf[i] / pairs:12.0f} cycles/pair  {100 * buf[i] / max(tot, 1):5.1f} %")
    print(f"  {'total':18s} {tot / pairs:12.0f} cycles/pair")
    eng.close()


if __name__ == "__main__":
    main()
