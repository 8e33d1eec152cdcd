#!/usr/bin/env python3
"""Microbenchmark of the fused ResNet50 identity bottleneck (bottleneck_img.hip)
for layer2 / layer3 / layer4 at B=256 with parts knocked out (--dbg bits, see
BiArgs::dbg): event-timed, median over --iters event pairs of --reps launches.
Random operands (timing only; numerics are tests/test_engine_gpu.py's)."""
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
    ap.add_argument("--layers", default="2,3,4")
    ap.add_argument("--dbg", default="0,1,2,4,8,15")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    B = args.batch
    g = torch.Generator().manual_seed(1)
    C = dmlc.native()
    shapes = {2: (28, 512, 128), 3: (14, 1024, 256), 4: (7, 2048, 512)}

    def f8(*shape):
        return (torch.randn(*shape, generator=g) * 0.5).to(torch.float8_e4m3fn).view(torch.uint8).to(dev)

    for layer in (int(l) for l in args.layers.split(",")):
        H, Cc, M = shapes[layer]
        x = f8(B, H, H, Cc)
        y = torch.empty_like(x)
        w1 = f8(M, Cc)
        a1 = torch.full((M,), 0.05, device=dev)
        b1 = (torch.randn(M, generator=g) * 0.1).to(dev)
        wf2 = (torch.randn(M * 9 * M, generator=g) / 24).bfloat16().to(dev)
        b2 = (torch.randn(M, generator=g) * 0.1).to(dev)
        w3 = (torch.randn(Cc * M, generator=g) / 8).bfloat16().to(dev)
        b3 = (torch.randn(Cc, generator=g) * 0.1).to(dev)
        P = [t.data_ptr() for t in (x, w1, a1, b1, wf2, b2, w3, b3, y)]
        torch.cuda.synchronize()
        for dbg in (int(d) for d in args.dbg.split(",")):
            def run():
                for _ in range(args.reps):
                    C.bottleneck_img(*P, 1.0, 1.0, B, H, Cc, M, 0, dbg)
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
            print(f"layer{layer} dbg={dbg:2d}  {statistics.median(ts):8.1f} us", flush=True)


if __name__ == "__main__":
    main()
