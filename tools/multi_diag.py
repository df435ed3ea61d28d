"""Diagnose atls_multi on one GPU at C4's full size: seal the whole 1 Mi x 16 KiB batch with one engine
(reference) and with MultiEngine([0] * parts) in three transports -- device copies, RCCL self with
transfers cut into ATLS_MULTI_CHUNK_MB pieces, RCCL self in whole ranges (ATLS_MULTI_CHUNK_MB=0) --
and print, per transport, which parts' tags / ciphertext differ from the reference. Each transport
runs in its own process (the chunk size is read once per process). Needs a GPU."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(mode, parts, n):
    sys.path.insert(0, ROOT)
    import numpy as np
    import torch

    import anothertls_amd as atls
    from anothertls_amd import workload

    b = workload.config_batch("c4_aes256gcm_1Mi_x_16KiB", n=n)
    recs = b["recs"]
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(1)
    d_in = torch.randint(0, 256, (b["in_bytes"] + 16,), dtype=torch.uint8, device=dev, generator=g)
    d_aux = torch.zeros(16, dtype=torch.uint8, device=dev)
    ref_out = torch.zeros(b["out_bytes"] + 16, dtype=torch.uint8, device=dev)
    ref_tags = torch.zeros(16 * len(recs), dtype=torch.uint8, device=dev)
    eng = atls.Engine(0)
    eng.set_keys(b["keys"])
    eng.seal_batch(recs, d_in, d_aux, ref_out, ref_tags, flags=atls.FLAG_DEVICE_PTRS)
    eng.close()
    if mode != "copies":
        os.environ["ATLS_MULTI_RCCL_SELF"] = "1"
    m = atls.MultiEngine([0] * parts)
    out = torch.zeros_like(ref_out)
    tags = torch.zeros_like(ref_tags)
    m.set_keys(b["keys"])
    m.seal_batch(recs, d_in, d_aux, out, tags, flags=atls.FLAG_DEVICE_PTRS)
    torch.cuda.synchronize()
    first = atls.partition(recs, parts)
    t_ok = (tags.view(-1, 16) == ref_tags.view(-1, 16)).all(dim=1).cpu().numpy()
    res = {"mode": mode, "uses_rccl": m.uses_rccl, "parts": parts, "records": len(recs), "per_part": []}
    so = int(recs["out_off"][1] - recs["out_off"][0])
    for p in range(parts):
        a, bb = int(first[p]), int(first[p + 1])
        bad = np.flatnonzero(~t_ok[a:bb])
        ct_same = bool(torch.equal(out[a * so:bb * so], ref_out[a * so:bb * so]))
        res["per_part"].append({"p": p, "records": bb - a, "bad_tags": int(len(bad)),
                                "first_bad": int(a + bad[0]) if len(bad) else None, "ct_equal": ct_same})
    m.close()
    print(json.dumps(res), flush=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "child":
        return child(sys.argv[2], int(sys.argv[3]), int(sys.argv[4]))
    n = int(os.environ.get("DIAG_RECORDS", "1048576"))
    for mode, chunk in (("rccl_chunked", "1024"), ("rccl_whole", "0"), ("copies", "1024")):
        env = dict(os.environ, ATLS_MULTI_CHUNK_MB=chunk)
        r = subprocess.run([sys.executable, __file__, "child", mode, "8", str(n)], env=env, capture_output=True,
                           text=True, timeout=300)
        print(r.stdout.strip() or r.stderr[-1500:], flush=True)


if __name__ == "__main__":
    main()
