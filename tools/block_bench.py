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
    ap.add_argument("--dbg", default="0", help="comma list of conv3x3_block dbg variants (1 no loop DMA, 2 no "
                    "residual loads, 4 no y stores, 7 none of them)")
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

    ref = None
    for dbg in (int(d) for d in args.dbg.split(",")):
        if dbg in (0, 16, 32):  # result-preserving variants: compare with the first one
            C.conv3x3_block(P(x), P(wf1), P(b1), P(wf2), P(b2), P(y), P(zero), args.batch, ops._stream(), dbg)
            torch.cuda.synchronize()
            if ref is None:
                ref = y.float().clone()
            else:
                d = (y.float() - ref).abs()
                print(f"dbg={dbg}: max abs diff vs the first variant {d.max().item():.4g} "
                      f"(max |ref| {ref.abs().max().item():.3g}, bf16 ulps differing "
                      f"{(d > 0).float().mean().item() * 100:.3f}%)", flush=True)

        def block():
            for _ in range(args.reps):
                C.conv3x3_block(P(x), P(wf1), P(b1), P(wf2), P(b2), P(y), P(zero), args.batch, ops._stream(), dbg)

        block()
        timed(block, 5)  # clocks up: the first timed launches read ~5-10% slow
        torch.cuda.synchronize()
        print(f"fused block dbg={dbg:2d}: {timed(block, args.iters) / args.reps:8.1f} us", flush=True)
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
