#!/usr/bin/env python3
"""Microbenchmark of the fused layer1 basic block (conv3x3_block.hip) at
B=256 vs the two register-weight row convs it replaces; event-timed, median
over --iters event pairs of --reps launches each (native calls, operands
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
    ap.add_argument("--reps", type=int, default=10, help="launches per timed event pair")
    ap.add_argument("--rows", action="store_true", help="also time the two row convs")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(1)
    x = torch.randn(args.batch, 56, 56, 64, generator=g).bfloat16().to(dev)
    w1 = (torch.randn(64, 64, 3, 3, generator=g) / 24).bfloat16().float()
    w2 = (torch.randn(64, 64, 3, 3, generator=g) / 24).bfloat16().float()
    b1 = (torch.randn(64, generator=g) * 0.1).to(dev)
    b2 = (torch.randn(64, generator=g) * 0.1).to(dev)
    wp1, wp2 = ops.pack_conv_weight(w1, device=dev), ops.pack_conv_weight(w2, device=dev)
    C = dmlc.native()
    wf1, wf2 = ops.stream_weight_frag(wp1), ops.stream_weight_frag(wp2)
    y = torch.empty_like(x)
    zero = ops._zero_page(dev)
    P = ops._ptr

    def block():
        for _ in range(args.reps):
            C.conv3x3_block(P(x), P(wf1), P(b1), P(wf2), P(b2), P(y), P(zero), args.batch, ops._stream())

    block()
    timed(block, 5)  # clocks up: the first timed launches read ~5-10% slow
    torch.cuda.synchronize()
    print(f"fused block: {timed(block, args.iters) / args.reps:8.1f} us", flush=True)
    if args.rows:
        t = torch.empty_like(x)
        strip = C.conv3x3_rows_pick_strip(args.batch, 56, 2 * torch.cuda.get_device_properties(dev).multi_processor_count)

        def two():
            for _ in range(args.reps):
                C.conv3x3_rows(P(x), P(wp1), P(b1), 0, P(t), P(zero), args.batch, 56, 56, 64, True, strip,
                               ops._stream(), P(wf1))
                C.conv3x3_rows(P(t), P(wp2), P(b2), P(x), P(y), P(zero), args.batch, 56, 56, 64, True, strip,
                               ops._stream(), P(wf2))
        two()
        print(f"two row convs:   {timed(two, args.iters) / args.reps:8.1f} us")


if __name__ == "__main__":
    main()
