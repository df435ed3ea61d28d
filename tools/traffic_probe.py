"""Diagnostic for HBM write / read amplification (run under rocprofv3 --pmc): seals a C3- or C2-shaped
batch, device-resident, with a chosen output stride and key count, so FETCH / WRITE request counts can
be compared between the config's packed layout (16-B aligned records) and line-aligned ones.
python tools/traffic_probe.py --config c3 --out-align 128 --keys 4096 --steps 3"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--config", default="c3")
    p.add_argument("--out-align", type=int, default=16)
    p.add_argument("--in-align", type=int, default=16)
    p.add_argument("--keys", type=int, default=4096)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--in-shift", type=int, default=0, help="bytes added to every record's input offset")
    p.add_argument("--out-shift", type=int, default=0, help="bytes added to every record's output offset")
    p.add_argument("--op", default="seal", choices=["seal", "open", "reseal"],
                   help="open: seal once, then time opens of the sealed records into a second buffer; "
                        "reseal: seal once, then seal again reading the first seal's output")
    p.add_argument("--raw", type=int, default=0,
                   help="RAW-mode records of exactly this many bytes (no type byte: every 16-B / 64-B piece whole)")
    a = p.parse_args()
    import anothertls_amd as atls
    from anothertls_amd import workload

    name = {"c2": "c2_aes128gcm_64Ki_x_16KiB", "c3": "c3_chacha20poly1305_64Ki_x_1.5KiB",
            "c5": "c5_mixed_256Ki_x_64B-16KiB"}[a.config]
    b = workload.config_batch(name, n=workload.records_per_rank(name), n_keys=a.keys)  # bench.py's rank-0 share
    recs = b["recs"].copy()
    mixed = a.config == "c5"  # the config's own packed layout (mixed lengths, planned batch)
    n = len(recs)
    aux = np.zeros(16, np.uint8)
    if a.raw:  # RAW: nonce (12 B) || no AAD from aux for every record
        recs["len"] = a.raw
        recs["mode"] = atls.MODE_RAW
        recs["iv_len"] = 12
        recs["aad_len"] = 0
        recs["aux_off"] = 0
    L = recs["len"].astype(np.int64)
    if mixed:
        istr = ostr = (int(recs["out_off"][-1]) + int(L[-1]) + 17 + n - 1) // n
    else:
        istr = (L[0] + a.in_align - 1) // a.in_align * a.in_align
        ostr = (L[0] + (0 if a.raw else 1) + a.out_align - 1) // a.out_align * a.out_align
        recs["in_off"] = np.arange(n, dtype=np.uint64) * np.uint64(istr) + np.uint64(a.in_shift)
        recs["out_off"] = np.arange(n, dtype=np.uint64) * np.uint64(ostr) + np.uint64(a.out_shift)
    dev = torch.device("cuda", 0)
    eng = atls.Engine(0)
    eng.set_keys(b["keys"])
    d_in = torch.randint(0, 256, (n * istr + 64 + a.in_shift,), dtype=torch.uint8, device=dev)
    d_out = torch.empty(n * ostr + 64 + a.out_shift, dtype=torch.uint8, device=dev)
    d_tags = torch.empty(16 * n, dtype=torch.uint8, device=dev)
    d_aux = torch.zeros(16, dtype=torch.uint8, device=dev)
    d_recs = torch.from_numpy(recs.view(np.uint8).copy()).to(dev)
    torch.cuda.synchronize()
    fl = atls.FLAG_DEVICE_PTRS | atls.FLAG_DEVICE_RECS | atls.FLAG_NO_SYNC
    seal = lambda r, i, o: eng.seal_batch(r.data_ptr(), i.data_ptr(), d_aux.data_ptr(), o.data_ptr(), d_tags.data_ptr(), flags=fl, n=n)
    if a.op == "seal":
        for _ in range(a.steps):
            seal(d_recs, d_in, d_out)
    else:
        seal(d_recs, d_in, d_out)
        d_pt = torch.zeros_like(d_out)
        o = recs.copy()
        o["in_off"] = recs["out_off"]
        if not a.raw:
            o["len"] = recs["len"] + 1
        if a.op == "reseal":  # the sealed bytes as plaintext, read where the open reads them
            o["len"] = recs["len"]
        d_o = torch.from_numpy(o.view(np.uint8).copy()).to(dev)
        d_res = torch.zeros(8 * n, dtype=torch.uint8, device=dev)
        for _ in range(a.steps):
            if a.op == "open":
                eng.open_batch(d_o.data_ptr(), d_out.data_ptr(), d_aux.data_ptr(), d_tags.data_ptr(), d_pt.data_ptr(),
                               d_res.data_ptr(), flags=fl, n=n)
            else:
                seal(d_o, d_out, d_pt)
        eng.sync()
        if a.op == "open":
            st = d_res.cpu().numpy().view(atls.OPEN_RESULT_DTYPE)["status"]
            print(f"open statuses ok: {bool((st == 0).all())}")
    eng.sync()
    print(f"{a.config} {a.op} in stride {istr} out stride {ostr} keys {a.keys}: payload {int(L.sum()) + n} B per launch")
    eng.close()


if __name__ == "__main__":
    main()
