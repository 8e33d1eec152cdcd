#!/usr/bin/env python3
"""Per-kernel medians of a bench.py rocprofv3 kernel trace, split by phase:
the single-lane latency phase (unpipelined steps: kernels isolated, one
forward at a time) and the batch-1 queries. The phases are told apart by
time: the last `--lat` stem launches at batch 256 are the latency steps.

Usage: lane_stats.py run_kernel_trace.csv [--lat 50]"""
import argparse
import collections
import csv
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--lat", type=int, default=50)
    a = ap.parse_args()
    rows = []
    for r in csv.DictReader(open(a.trace)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                     int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0), int(r.get("Workgroup_Size_X", 0) or 0)))
    rows.sort()
    stems = [r for r in rows if "stem" in r[2] and r[3] >= 256 * 64]
    if len(stems) < a.lat:
        stems = [r for r in rows if "stem" in r[2]]
    t_lat = stems[-a.lat][0]
    # end of latency phase: next kernel of a small grid after the last stem of the phase... use all kernels after
    # t_lat whose grid is that of the big-batch forward (grid >= 64 workgroups) up to the first batch-1 stem
    lat = [r for r in rows if r[0] >= t_lat]
    small_stem = [r for r in lat if "stem" in r[2] and r[3] < 256 * 64]
    if small_stem:
        t_end = small_stem[0][0]
        b1 = [r for r in lat if r[0] >= t_end]
        lat = [r for r in lat if r[0] < t_end]
    else:
        b1 = []
    for title, ph, n in (("single-lane latency phase", lat, a.lat), ("batch-1 queries", b1, None)):
        if not ph:
            continue
        d = collections.defaultdict(list)
        for s, e, name, g, w in ph:
            d[name].append((e - s) / 1000.0)
        nf = n or max(1, sum(len(v) for k, v in d.items() if "stem" in k))  # one stem per forward
        print(f"## {title}: per forward ({nf} forwards)")
        tot = 0.0
        for name, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
            per = sum(v) / nf
            tot += per
            print(f"{per:8.1f} us/fwd n={len(v):4d} med {statistics.median(v):7.1f}  {name[:120]}")
        span = (ph[-1][1] - ph[0][0]) / 1000.0 / nf
        print(f"{tot:8.1f} us/fwd kernel total; wall span per forward {span:.1f} us")


if __name__ == "__main__":
    main()
