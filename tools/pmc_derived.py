#!/usr/bin/env python3
"""Per-kernel derived PMC metrics from two rocprofv3 --pmc passes (tools/gpu_r4h.sh):
duration (kernel trace), effective clock (GRBM_GUI_ACTIVE / 8 XCDs / duration),
MFMA busy (SQ_VALU_MFMA_BUSY_CYCLES / (clock cycles x 4 SIMDs x CUs)), VALU/MFMA and
LDS/MFMA instruction ratios, LDS bank-conflict share. Usage: pmc_derived.py <pass1 dir> <pass2 dir> [cus]"""
import collections
import csv
import statistics
import sys


def load(d):
    dur = {}
    for r in csv.DictReader(open(d + "/p_kernel_trace.csv")):
        dur[r["Dispatch_Id"]] = (r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
    ctr = collections.defaultdict(dict)
    for r in csv.DictReader(open(d + "/p_counter_collection.csv")):
        ctr[r["Dispatch_Id"]][r["Counter_Name"]] = ctr[r["Dispatch_Id"]].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return dur, ctr


def main():
    d1, d2 = sys.argv[1], sys.argv[2]
    cus = int(sys.argv[3]) if len(sys.argv) > 3 else 256
    per = collections.defaultdict(list)
    for d in (d1, d2):
        dur, ctr = load(d)
        for k, (name, us) in dur.items():
            if k in ctr:
                per[name].append((us, ctr[k]))
    rows = []
    for name, lst in per.items():
        agg = collections.defaultdict(list)
        for us, c in lst:
            agg["us"].append(us)
            for cn, v in c.items():
                agg[cn].append(v)
        m = {k: statistics.median(v) for k, v in agg.items()}
        if "GRBM_GUI_ACTIVE" not in m or "SQ_INSTS_MFMA" not in m or m["SQ_INSTS_MFMA"] == 0:
            continue
        clk = m["GRBM_GUI_ACTIVE"] / 8 / m["us"] * 1e-3
        busy = m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (m["GRBM_GUI_ACTIVE"] / 8 * 4 * cus)
        valu = m.get("SQ_INSTS_VALU", 0) / m["SQ_INSTS_MFMA"]
        lds = m.get("SQ_INSTS_LDS", 0) / m["SQ_INSTS_MFMA"]
        conf = m.get("SQ_LDS_BANK_CONFLICT", 0) / max(m.get("SQ_LDS_IDX_ACTIVE", 1), 1)
        rows.append((m["us"], f"{m['us']:8.1f} us  clk {clk:4.2f} GHz  MFMA busy {100 * busy:5.1f}%  VALU/MFMA {valu:5.2f}  "
                              f"LDS/MFMA {lds:4.2f}  LDS conflict cycles {100 * conf:4.1f}%  n={len(lst)}  {name[:110]}"))
    for _, line in sorted(rows, reverse=True):
        print(line)


if __name__ == "__main__":
    main()
