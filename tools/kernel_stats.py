#!/usr/bin/env python3
"""Per-forward kernel time summary from a rocprofv3 --kernel-trace CSV or
its default SQLite output (``*_results.db``).

Usage: kernel_stats.py <run_kernel_trace.csv | run_results.db> <forwards> [header line]
Prints total us per forward, call count and median us per call for each
kernel, sorted by total (the format of profiles/r1_v*_kernel_stats.txt)."""
import collections
import csv
import statistics
import sys


def main():
    path, fwd = sys.argv[1], int(sys.argv[2])
    head = sys.argv[3] if len(sys.argv) > 3 else None
    dur = collections.defaultdict(list)
    if path.endswith(".db"):
        import sqlite3
        for name, t0, t1 in sqlite3.connect(path).execute("select name, start, end from kernels"):
            dur[name].append((int(t1) - int(t0)) / 1000.0)
    else:
        for r in csv.DictReader(open(path)):
            dur[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
    if head:
        print(head)
    print("# per-forward total, calls, median per call")
    total = 0.0
    for name, d in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        s = sum(d) / fwd
        total += s
        print(f"{s:8.1f} us/fwd  n={len(d):4d}  median={statistics.median(d):8.1f} us  {name[:110]}")
    print(f"{total:8.1f} us/fwd total")


if __name__ == "__main__":
    main()
