#!/usr/bin/env python3
"""AlexNet forward latency at query batch sizes (graph replay, host-timed
including the D2H of the answers) and the classifier's share of it; run
under rocprofv3 --kernel-trace for per-kernel times (fc_small_kernel per
classifier layer vs its HBM floor: 75.5 / 33.6 / 8.2 MB of bf16 weights).
usage: python tools/alexnet_bench.py [--batches 1,8,16] [--iters 200]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from dmlc.runtime import InferenceEngine


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="1,8,16")
    ap.add_argument("--iters", type=int, default=200)
    a = ap.parse_args()
    for B in [int(x) for x in a.batches.split(",")]:
        eng = InferenceEngine("alexnet", device=0, max_batch=B, seed=1)
        img = torch.randint(0, 256, (B, 224, 224, 3), dtype=torch.uint8, device="cuda")
        out = (torch.empty(B, dtype=torch.int32, device="cuda"), torch.empty(B, device="cuda"))
        for _ in range(20):
            eng.predict(img, out=out)
        torch.cuda.synchronize()
        lat = []
        for _ in range(a.iters):
            t = time.perf_counter()
            eng.predict(img, out=out)
            _ = out[0][0].item()
            lat.append((time.perf_counter() - t) * 1e3)
        lat.sort()
        prof = eng.profile(img)
        fc = sum(t for n, t in prof if n.startswith("classifier"))
        print(f"alexnet B={B}: p50 {lat[len(lat) // 2]:.3f} ms  p95 {lat[int(len(lat) * 0.95)]:.3f} ms  "
              f"({B / lat[len(lat) // 2] * 1e3:.0f} img/s); eager per-op classifier sum {fc:.3f} ms: "
              + ", ".join(f"{n}={t:.3f}" for n, t in prof if n.startswith("classifier")), flush=True)


if __name__ == "__main__":
    main()
