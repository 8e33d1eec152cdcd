#!/usr/bin/env python3
"""Microbenchmark of ResNet18's fused stem (stem_pool.hip: conv7x7/s2 + BN +
ReLU + maxpool, u8 images in) at B=256, graph-replayed (tools/conv_bench.py's
timer), with parts knocked out (stem_conv_pool_set_dbg bits, see the kernel's
DBG) and against the bf16 paired-image variant (conversion done by a separate
preprocess kernel, not timed here). Random operands: timing only."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dmlc  # noqa: E402
from dmlc import ops  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from conv_bench import time_us, warm_gpu  # noqa: E402

NAMES = {0: "full", 1: "no h-pool epilogue", 2: "no u8 conversion", 4: "no v-max/stores", 6: "no conv, no v-max",
         7: "MFMA + loads only", 8: "no MFMA", 14: "epilogue only"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--dbg", default="0,1,2,4,6,7,8,14")
    ap.add_argument("--stagger", default="0,1,2,3,4,6")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(3)
    B = args.batch
    img = torch.randint(0, 256, (B, 224, 224, 3), generator=g, dtype=torch.uint8).to(dev)
    w = torch.randn(64, 3, 7, 7, generator=g) / 12
    wp = ops.pack_stem_pool_weight(w, device=dev)
    bias = (torch.randn(64, generator=g) * 0.1).to(dev)
    C = dmlc.native()
    flop = 2 * B * 112 * 112 * 64 * 147
    warm_gpu()
    for d in [int(t) for t in args.dbg.split(",")] * 2:
        C.stem_conv_pool_set_dbg(d)
        try:
            us = time_us(lambda: ops.stem_conv_pool_u8(img, wp, bias, 28), args.iters)
        finally:
            C.stem_conv_pool_set_dbg(0)
        print(f"u8 dbg={d:2d} {NAMES.get(d, ''):22s} {us:7.1f} us  {flop / us / 1e6:6.0f} TFLOP/s (147-deep K)", flush=True)
    for st in [int(t) for t in args.stagger.split(",")]:  # second half of the grid started ~st us late
        C.stem_conv_pool_set_dbg(((st + 1) << 16) | 1024)  # (0 = the default stagger)
        try:
            us = time_us(lambda: ops.stem_conv_pool_u8(img, wp, bias, 28), args.iters)
        finally:
            C.stem_conv_pool_set_dbg(0)
        print(f"u8 stagger={st:2d} {us:7.1f} us", flush=True)
    us = time_us(lambda: ops.stem_conv_pool_u8(img, wp, bias), args.iters)
    print(f"u8 default (role-split, one workgroup per image at B >= CUs) {us:7.1f} us", flush=True)
    C.stem_conv_pool_set_dbg(1024)
    try:
        us = time_us(lambda: ops.stem_conv_pool_u8(img, wp, bias, 28), args.iters)
    finally:
        C.stem_conv_pool_set_dbg(0)
    print(f"u8 strip kernel (strip 28, 2 workgroups per CU, staggered) {us:7.1f} us", flush=True)
    xp = ops.preprocess_u8(img, 224, 3, paired=True)
    us = time_us(lambda: ops.stem_conv_pool(xp, wp, bias), args.iters)
    print(f"bf16 paired input          {us:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
