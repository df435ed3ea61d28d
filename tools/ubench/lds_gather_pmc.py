"""Reduce a rocprofv3 --pmc pass of tools/ubench/lds_gather_ubench to one line per (pattern, waves, dependent):
SQ_LDS_IDX_ACTIVE per LDS wave-instruction (what the counter charges), its share of the CUs' cycles (the "array
busy" figure the AES-GCM PMC reports), and the CU-cycles actually spent per LDS wave-instruction.
python tools/ubench/lds_gather_pmc.py <run_counter_collection.csv>"""
import collections
import csv
import re
import sys

PATS = ["b32_tt", "b32_lin", "b32_bcast", "b32_64bank", "b64_tt", "b128_gh", "mix"]


def main():
    per = collections.defaultdict(dict)
    for r in csv.DictReader(open(sys.argv[1])):
        k = (int(r["Dispatch_Id"]), r["Kernel_Name"])
        per[k][r["Counter_Name"]] = float(r["Counter_Value"])
        per[k]["_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    best = {}
    for (_, name), d in per.items():
        if "k<" not in name:
            continue
        # the timed launch of each kernel (the warm-up runs 64 iterations)
        if name not in best or d.get("SQ_INSTS_LDS", 0) > best[name].get("SQ_INSTS_LDS", 0):
            best[name] = d
    rows = []
    for name, d in best.items():
        p, w, dep = (int(v) for v in re.findall(r"<(\d+), (\d+), (\d+)>", name)[0])
        cyc = d.get("GRBM_GUI_ACTIVE", 0) / 8  # per XCD
        rows.append((p, dep, w, f"{PATS[p]:11s} waves={w:2d} dependent={dep} us={d['_ns'] / 1e3:8.1f} "
                                f"IDX_ACTIVE/instr={d['SQ_LDS_IDX_ACTIVE'] / d['SQ_INSTS_LDS']:.3f} "
                                f"array_busy={d['SQ_LDS_IDX_ACTIVE'] / (256 * cyc):.3f} "
                                f"CU_cycles/instr={256 * cyc / d['SQ_INSTS_LDS']:.3f} "
                                f"wait_inst_lds={d.get('SQ_WAIT_INST_LDS', 0) / max(d.get('SQ_WAVE_CYCLES', 1), 1):.3f}"))
    for r in sorted(rows):
        print(r[3])


if __name__ == "__main__":
    main()
