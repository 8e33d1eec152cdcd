#!/usr/bin/env python3
"""Microbenchmark of ResNet18 layer2.0.conv1 + downsample at B=256:
conv3x3_s2rows.hip vs the stream conv's register-weight fused-downsample
variant (what the engine ran before); event-timed, median over --iters event
pairs of --reps launches each (native calls, operands prepared outside the
timed region)."""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dmlc  # noqa: E402
from dmlc import ops  # noqa: E402


def timed(fn, iters):
    ts = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--reps", type=int, default=10, help="launches per timed event pair")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(1)
    B = args.batch
    x = torch.randn(B, 56, 56, 64, generator=g).bfloat16().to(dev)
    w = (torch.randn(128, 64, 3, 3, generator=g) / 24).bfloat16().float()
    wd = (torch.randn(128, 64, 1, 1, generator=g) / 8).bfloat16().float()
    b1 = (torch.randn(128, generator=g) * 0.1).to(dev)
    bd = (torch.randn(128, generator=g) * 0.1).to(dev)
    wp, wdp = ops.pack_conv_weight(w, device=dev), ops.pack_conv_weight(wd, device=dev)
    C = dmlc.native()
    wf, wdf = ops.stream_weight_frag(wp), ops.stream_weight_frag(wdp)
    y = torch.empty(B, 28, 28, 128, dtype=torch.bfloat16, device=dev)
    yd = torch.empty_like(y)
    zero = ops._zero_page(dev)
    P = ops._ptr
    flop = 2 * B * 28 * 28 * 128 * (576 + 64)

    def rows():
        def run():
            for _ in range(args.reps):
                C.conv3x3_s2rows(P(x), P(wf), P(b1), P(wdf), P(bd), P(y), P(yd), P(zero), B, True, ops._stream())
        return run

    def stream():
        for _ in range(args.reps):
            C.conv3x3_stream(P(x), P(wp), P(b1), 0, P(y), P(zero), B, 56, 56, 64, 128, 2, True, ops._stream(), 0,
                             P(wdp), P(bd), P(yd))

    runs = [("s2rows", rows()), ("stream+ds", stream)]
    for name, fn in runs:
        fn()
        torch.cuda.synchronize()
        us = timed(fn, args.iters) / args.reps
        print(f"{name:10s} {us:8.1f} us  {flop / us / 1e6:7.1f} TFLOP/s", flush=True)


if __name__ == "__main__":
    main()
