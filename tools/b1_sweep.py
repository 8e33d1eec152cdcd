#!/usr/bin/env python3
"""Batch-1 (query-sized) implicit-GEMM tile x split-K sweep for the ResNet18
convs of layers 2-4: each (tile, split) replayed from a graph (tools/
conv_bench.py's timer), the split-K reduce kernel included. Picks the
per-layer configuration the batch-1 path should use."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from conv_bench import time_us, warm_gpu  # noqa: E402

from dmlc import ops  # noqa: E402

LAYERS = [("l2", 28, 128, 128, 1), ("l2.c1", 56, 64, 128, 2), ("l3", 14, 256, 256, 1), ("l3.c1", 28, 128, 256, 2),
          ("l4", 7, 512, 512, 1), ("l4.c1", 14, 256, 512, 2)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--tiles", default="0,2,7,8")
    ap.add_argument("--splits", default="1,2,4,8,16,32,64")
    ap.add_argument("--iters", type=int, default=30)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    warm_gpu(0.5)
    for name, H, Cin, Cout, s in LAYERS:
        x = (torch.randn(a.batch, H, H, Cin, device=dev) * 0.5).bfloat16()
        w = torch.randn(Cout, Cin, 3, 3) / (Cin * 9) ** 0.5
        wp = ops.pack_conv_weight(w, device=dev)
        bias = torch.zeros(Cout, device=dev)
        row = []
        best = None
        for t in [int(v) for v in a.tiles.split(",")]:
            for sp in [int(v) for v in a.splits.split(",")]:
                try:
                    f = lambda: ops.conv2d(x, wp, Cout, 3, 3, s, 1, bias=bias, relu=True, tile=t, split_k=sp)
                    us = time_us(f, a.iters)
                except Exception as e:  # noqa: BLE001
                    row.append(f"t{t}s{sp}=ERR")
                    continue
                row.append(f"t{t}s{sp}={us:.1f}")
                if best is None or us < best[0]:
                    best = (us, t, sp)
        print(f"{name:6s} B={a.batch} best t{best[1]} s{best[2]} {best[0]:.1f}us | " + " ".join(row), flush=True)


if __name__ == "__main__":
    main()
