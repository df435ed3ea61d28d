"""Reduce a rocprofv3 --pmc counter_collection CSV to per-kernel averages over the dispatches after
the first `skip` of that kernel, with the derived ratios used in DESIGN.md: LDS array busy =
SQ_LDS_IDX_ACTIVE / (CUs x cycles), cycles = GRBM_GUI_ACTIVE / 8 (XCDs); wave-state shares of
SQ_WAVE_CYCLES. python tools/pmc_summary.py <run_counter_collection.csv> [kernel-substring] [skip]"""
import collections
import csv
import json
import sys


def main():
    path = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else "gcm_kernel"
    skip = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    per = collections.defaultdict(lambda: collections.defaultdict(dict))
    for r in csv.DictReader(open(path)):
        if sub not in r["Kernel_Name"]:
            continue
        per[r["Kernel_Name"]][int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
        per[r["Kernel_Name"]][int(r["Dispatch_Id"])]["_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    out = {}
    for k, disp in per.items():
        ids = sorted(disp)[skip:] or sorted(disp)
        avg = {c: sum(disp[i].get(c, 0.0) for i in ids) / len(ids) for c in disp[ids[0]]}
        d = {"dispatches": len(ids), "avg": {c: round(v, 1) for c, v in avg.items()}}
        cyc = avg.get("GRBM_GUI_ACTIVE", 0) / 8
        if cyc:
            d["clock_GHz"] = round(cyc / avg["_ns"], 3)
            if "SQ_LDS_IDX_ACTIVE" in avg:
                d["lds_array_busy"] = round(avg["SQ_LDS_IDX_ACTIVE"] / (256 * cyc), 4)
        wc = avg.get("SQ_WAVE_CYCLES")
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
            if wc and c in avg:
                d[c + "_share"] = round(avg[c] / wc, 4)
        out[k] = d
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
