#!/usr/bin/env python3
"""GPU busy fraction from a rocprofv3 --kernel-trace SQLite db (``*_results.db``):
the union of all kernel intervals over a window, vs the window's wall time.
With two compute lanes the forwards overlap, so the sum of kernel times
exceeds the wall time; idle gaps in the union are time the GPU ran nothing.

Usage: gpu_busy.py <run_results.db> [window_ms=20] (the last window_ms of the trace)"""
import sqlite3
import sys


def main():
    path = sys.argv[1]
    window = float(sys.argv[2]) if len(sys.argv) > 2 else 20.0
    rows = sorted(sqlite3.connect(path).execute("select start, end, name from kernels"))
    t_end = max(e for _, e, _ in rows)
    t0 = t_end - window * 1e6
    iv = [(max(s, t0), e) for s, e, _ in rows if e > t0]
    iv.sort()
    busy, cur_s, cur_e = 0, None, None
    gaps = []
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
                gaps.append(s - cur_e)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    span = t_end - max(t0, iv[0][0])
    kern = sum(e - s for s, e in iv)
    gaps.sort(reverse=True)
    print(f"window {span / 1e6:.2f} ms: busy {busy / span * 100:.1f}%  kernel-time/wall {kern / span:.2f}  "
          f"{len(gaps)} gaps, largest (us): {[round(g / 1e3, 1) for g in gaps[:8]]}")


if __name__ == "__main__":
    main()
