#!/usr/bin/env python3
"""Average rocprofv3 counter values per dispatch for kernels matching a name
filter. Usage: pmc_summary.py <filter> <dir> [<dir> ...]"""
import collections
import csv
import sys


def main():
    filt, dirs = sys.argv[1], sys.argv[2:]
    for d in dirs:
        agg = collections.defaultdict(float)
        disp = collections.defaultdict(set)
        for r in csv.DictReader(open(d + "/p_counter_collection.csv")):
            if filt not in r["Kernel_Name"]:
                continue
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            disp[r["Counter_Name"]].add(r["Dispatch_Id"])
        for c in sorted(agg):
            print(f"{c:28s} {agg[c] / len(disp[c]):16.0f}")


if __name__ == "__main__":
    main()
