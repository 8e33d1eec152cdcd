#!/usr/bin/env python3
"""Microbenchmark of the fused ResNet50 layer1 bottleneck (bottleneck56.hip)
at B=256: event-timed, median over --iters event pairs of --reps launches
each (its phase knock-outs: profiles/r3_bottleneck_*.txt). Random operands
(timing only; numerics are tests/test_engine_gpu.py's)."""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dmlc  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=15)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    B = args.batch
    g = torch.Generator().manual_seed(1)

    def f8(*shape):
        return (torch.randn(*shape, generator=g) * 0.5).to(torch.float8_e4m3fn).view(torch.uint8).to(dev)

    x = f8(B, 56, 56, 256)
    y = torch.empty_like(x)
    w1 = f8(64, 256)
    a1 = torch.full((64,), 0.05, device=dev)
    b1 = (torch.randn(64, generator=g) * 0.1).to(dev)
    wf2 = (torch.randn(2 * 18 * 2 * 64 * 8, generator=g) / 24).bfloat16().to(dev)
    b2 = (torch.randn(64, generator=g) * 0.1).to(dev)
    wf3 = (torch.randn(8 * 2 * 2 * 64 * 8, generator=g) / 8).bfloat16().to(dev)
    b3 = (torch.randn(256, generator=g) * 0.1).to(dev)
    C = dmlc.native()
    P = [t.data_ptr() for t in (x, w1, a1, b1, wf2, b2, wf3, b3, y)]
    torch.cuda.synchronize()
    for _rnd in range(2):  # two passes: the spread between them is the noise
        def run():
            for _ in range(args.reps):
                C.bottleneck56(*P, 1.0, 1.0, B, 0)
        run()
        torch.cuda.synchronize()
        ts = []
        for _ in range(args.iters):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            run()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3 / args.reps)
        print(f"bottleneck56  {statistics.median(ts):8.1f} us", flush=True)


if __name__ == "__main__":
    main()
