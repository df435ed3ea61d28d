"""HBM traffic of one kernel per variant from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (round-4 A/Bs):
python tools/ab_traffic.py <dir> <kernel substring> <algorithmic bytes per launch> <variant>...
expects <dir>/<variant>_fetch/**/run_counter_collection.csv and <variant>_write/...; FETCH_SIZE doubled
(MI355X_MICROARCH.md §HBM), both KiB per dispatch. Prints one JSON object: per variant bytes per launch and
(FETCH + WRITE) / algorithmic."""
import collections
import csv
import glob
import json
import os
import sys


def avg(path_glob, counter, kern):
    vals = collections.defaultdict(float)
    for path in glob.glob(path_glob, recursive=True):
        for r in csv.DictReader(open(path)):
            if r["Counter_Name"] == counter and kern in r["Kernel_Name"]:
                vals[r["Dispatch_Id"]] += float(r["Counter_Value"]) * 1024
    v = sorted(vals.values())
    return sum(v) / len(v) if v else None, len(v)


def main():
    d, kern, alg = sys.argv[1], sys.argv[2], float(sys.argv[3])
    out = {"kernel": kern, "alg_bytes": alg}
    for var in sys.argv[4:]:
        f, nf = avg(os.path.join(d, f"{var}_fetch", "**", "*counter_collection.csv"), "FETCH_SIZE", kern)
        w, nw = avg(os.path.join(d, f"{var}_write", "**", "*counter_collection.csv"), "WRITE_SIZE", kern)
        if f is None or w is None:
            out[var] = None
            continue
        out[var] = {"fetch_bytes": round(2 * f), "write_bytes": round(w), "dispatches": [nf, nw],
                    "traffic_over_alg": round((2 * f + w) / alg, 4), "write_over_alg_write": None}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
