#!/usr/bin/env python3
"""ResNet stem microbenchmark: fused conv7x7/s2 + maxpool (stem_pool.hip) vs
the two-kernel path (implicit-GEMM stem conv on the packed image + maxpool).
Median of --iters hipEvent timings, B=256 by default."""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dmlc import ops  # noqa: E402


def _time(f, iters):
    f()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
        e0.record()
        f()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--size", type=int, default=224)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--strips", default="0,56,28,14")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    B, S = a.batch, a.size
    img = torch.randint(0, 256, (B, S, S, 3), dtype=torch.uint8, device=dev)
    w = torch.randn(64, 3, 7, 7) / 147 ** 0.5
    bias = torch.zeros(64, device=dev)
    flops = 2.0 * B * (S // 2) ** 2 * 64 * 147
    xp = ops.preprocess_u8(img, S, 3, (S + 6 + 7) // 8 * 8, paired=True)
    wp = ops.pack_stem_pool_weight(w, device=dev)
    for st in [int(s) for s in a.strips.split(",")]:
        ms = _time(lambda: ops.stem_conv_pool(xp, wp, bias, S, st or None), a.iters)
        print(f"fused strip={st or 'auto'}: {ms * 1e3:7.1f} us  ({flops / ms / 1e9:5.0f} TF conv-equivalent)")
    for st in [int(s) for s in a.strips.split(",")]:
        ms = _time(lambda: ops.stem_conv_pool_u8(img, wp, bias, st or None), a.iters)
        print(f"fused u8 strip={st or 'auto'}: {ms * 1e3:7.1f} us  ({flops / ms / 1e9:5.0f} TF conv-equivalent)")
    wr = ops.stem_row_width(S, 3, 7, 2)
    xr = ops.preprocess_u8(img, S, 3, wr)
    wr_p = ops.pack_conv_weight(w, stem=True, device=dev)
    ho = S // 2

    def two():
        y = ops.conv2d(xr, wr_p, 64, 7, 7, 2, 3, bias=bias, relu=True, stem=True, out_hw=(ho, ho))
        return ops.maxpool2d(y, 3, 2, 1)

    ms = _time(two, a.iters)
    print(f"conv+maxpool (2 kernels): {ms * 1e3:7.1f} us")
    pp = _time(lambda: ops.preprocess_u8(img, S, 3, (S + 6 + 7) // 8 * 8, paired=True), a.iters)
    pr = _time(lambda: ops.preprocess_u8(img, S, 3, wr), a.iters)
    print(f"preprocess paired: {pp * 1e3:7.1f} us   packed: {pr * 1e3:7.1f} us")


if __name__ == "__main__":
    main()
