"""Reduce the rocprofv3 PMC passes of tools/profile_round.sh into profiles/traffic.json.

python tools/traffic.py <profiles dir with c{2,3,4}_pmc_{fetch,write}.csv>
FETCH_SIZE / WRITE_SIZE are KiB per dispatch; FETCH_SIZE is doubled (gfx950 reports half of wide
streaming reads, MI355X_MICROARCH.md §HBM). Each config's dominant kernel is the one with the
largest traffic per dispatch among the record kernels (atls::gcm_kernel / atls::chacha_kernel);
values are averaged over its dispatches."""
import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CONFIGS = {"c2": "c2_aes128gcm_64Ki_x_16KiB", "c3": "c3_chacha20poly1305_64Ki_x_1.5KiB",
           "c4": "c4_aes256gcm_1Mi_x_16KiB", "c5": "c5_mixed_256Ki_x_64B-16KiB"}


def per_kernel(path, counter):
    vals = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            vals[r["Kernel_Name"]].append(float(r["Counter_Value"]) * 1024)
    return vals


def main():
    from anothertls_amd import workload

    d = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "profiles", "r03")
    out = {"_about": "HBM traffic per launch of the dominant kernel from rocprofv3 PMC passes (separate --pmc "
                     "FETCH_SIZE / WRITE_SIZE runs of `bench.py --config <cfg> --steps 20 --warmup 3`, "
                     "tools/profile_round.sh; CSVs in " + os.path.relpath(d, ROOT) + ", reduced by tools/traffic.py; seal kernels, and under "
                     "'open' the open kernels of the same runs). FETCH_SIZE is "
                     "doubled (gfx950 reports 1/2 of wide streaming reads, MI355X_MICROARCH.md §HBM), WRITE_SIZE as "
                     "reported. Averaged over the kernel's dispatches. Units: bytes."}
    for tag, cfg in CONFIGS.items():
        if not os.path.exists(os.path.join(d, f"{tag}_pmc_fetch.csv")):
            continue
        f = per_kernel(os.path.join(d, f"{tag}_pmc_fetch.csv"), "FETCH_SIZE")
        w = per_kernel(os.path.join(d, f"{tag}_pmc_write.csv"), "WRITE_SIZE")
        b = workload.shard_batch(cfg, 0)
        alg = 2 * b["payload"] + 16 * len(b["recs"])

        def reduce(opening):
            # the record kernels of one direction: <false, ...> seals, <true, ...> opens (bench.py runs
            # both); a mixed batch's AES-GCM and ChaCha20-Poly1305 kernels each take their records of
            # the same launch (two streams), so C5's traffic is the sum of both
            flag = "<true" if opening else "<false"
            rec = [n for n in f if ("atls::gcm_kernel" in n or "atls::chacha_kernel" in n) and flag in n and n in w]
            if not rec:
                return None
            if tag == "c5":
                k = " + ".join(sorted(rec))
                fetch = sum(2 * sum(f[n]) / len(f[n]) for n in rec)
                write = sum(sum(w[n]) / len(w[n]) for n in rec)
            else:
                k = max(rec, key=lambda n: sum(f[n]) / len(f[n]))
                fetch = 2 * sum(f[k]) / len(f[k])
                write = sum(w[k]) / len(w[k])
            return {"kernel": k, "fetch_bytes": round(fetch), "write_bytes": round(write),
                    "hbm_bytes_per_launch": round(fetch + write), "algorithmic_bytes_per_launch": alg,
                    "ratio": round((fetch + write) / alg, 4)}

        out[cfg] = reduce(False)
        op = reduce(True)
        if out[cfg] is not None and op is not None:
            out[cfg]["open"] = op
    json.dump(out, open(os.path.join(ROOT, "profiles", "traffic.json"), "w"), indent=1)
    print(json.dumps({k: v.get("ratio") for k, v in out.items() if k != "_about"}))


if __name__ == "__main__":
    main()
