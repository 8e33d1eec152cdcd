#!/usr/bin/env python3
"""One forward's kernel timeline from a rocprofv3 --kernel-trace CSV: start
offset, duration and gap to the previous kernel's end (negative = overlap),
for the forward that starts at the N-th-from-last stem kernel.

Usage: timeline.py <run_kernel_trace.csv> [first-kernel substring] [which (-1 = last)]"""
import csv
import sys


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    key = sys.argv[2] if len(sys.argv) > 2 else "stem_conv_pool"
    which = int(sys.argv[3]) if len(sys.argv) > 3 else -2
    starts = [i for i, r in enumerate(rows) if key in r["Kernel_Name"]]
    i0 = starts[which]
    i1 = starts[which + 1] if which + 1 < 0 or which + 1 < len(starts) else len(rows)
    t0 = int(rows[i0]["Start_Timestamp"])
    prev_end = t0
    for r in rows[i0:i1]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} gap {(s - prev_end) / 1e3:6.1f}  {r['Kernel_Name'][:90]}")
        prev_end = max(prev_end, e)
    print(f"forward span {(prev_end - t0) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
