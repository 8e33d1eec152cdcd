#!/usr/bin/env python3
"""Microbenchmark of ResNet18's layer2 stride-1 conv (28x28x128 -> 128) at
B=256: conv3x3_rows28.hip (weight-stationary, row-streaming) vs the stream
conv the engine ran before, with and without the residual; event-timed,
median over --iters event pairs of --reps launches (native calls, operands
prepared outside the timed region)."""
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
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(1)
    B = args.batch
    x = torch.randn(B, 28, 28, 128, generator=g).bfloat16().to(dev)
    r = torch.randn(B, 28, 28, 128, generator=g).bfloat16().to(dev)
    w = (torch.randn(128, 128, 3, 3, generator=g) / 34).bfloat16().float()
    b1 = (torch.randn(128, generator=g) * 0.1).to(dev)
    wp = ops.pack_conv_weight(w, device=dev)
    wf = ops.stream_weight_frag(wp)
    C = dmlc.native()
    y = torch.empty_like(x)
    zero = ops._zero_page(dev)
    P = ops._ptr
    flop = 2 * B * 28 * 28 * 128 * 1152

    def rows(res):
        def run():
            for _ in range(args.reps):
                C.conv3x3_rows28(P(x), P(wf), P(b1), P(res), P(y), B, True, ops._stream())
        return run

    def stream(res):
        def run():
            for _ in range(args.reps):
                C.conv3x3_stream(P(x), P(wp), P(b1), P(res), P(y), P(zero), B, 28, 28, 128, 128, 1, True,
                                 ops._stream())
        return run

    runs = [("rows28", rows(None)), ("rows28+res", rows(r)), ("stream", stream(None)), ("stream+res", stream(r))]
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from conv_bench import warm_gpu
    warm_gpu()
    for rnd in range(2):  # two passes: the spread between them is the noise
        for name, fn in runs:
            fn()
            torch.cuda.synchronize()
            us = timed(fn, args.iters) / args.reps
            print(f"pass {rnd} {name:11s} {us:8.1f} us  {flop / us / 1e6:7.1f} TFLOP/s", flush=True)


if __name__ == "__main__":
    main()
