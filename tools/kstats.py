"""Steady-state kernel times from a rocprofv3 --kernel-trace CSV: per kernel, the dispatches after
the first `warmup` ones (bench.py's untimed warm-up steps), so averages compare with bench.py's
HIP-event kernel_ms. python tools/kstats.py <run_kernel_trace.csv> [warmup] -> JSON on stdout."""
import collections
import csv
import json
import sys


def main():
    path = sys.argv[1]
    warmup = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    t = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        t[r["Kernel_Name"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    out = {}
    for k, v in t.items():
        if "atls::" not in k:  # the engine's kernels only (not torch's fills and copies)
            continue
        v.sort()
        d = [(e - s) / 1e6 for s, e in v]  # ns -> ms
        steady = d[warmup:] if len(d) > warmup else d
        out[k] = {"dispatches": len(d), "steady_dispatches": len(steady),
                  "steady_avg_ms": round(sum(steady) / len(steady), 5), "steady_min_ms": round(min(steady), 5),
                  "steady_max_ms": round(max(steady), 5), "all_avg_ms": round(sum(d) / len(d), 5)}
    print(json.dumps(dict(sorted(out.items(), key=lambda kv: -kv[1]["steady_avg_ms"] * kv[1]["dispatches"])),
                     indent=1))


if __name__ == "__main__":
    main()
