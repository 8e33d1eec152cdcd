#!/usr/bin/env python3
"""AlexNet classifier FCs at B=256 on the implicit-GEMM conv (conv_igemm.hip)
by tile config and split-K count: graph-replayed launches (tools/conv_bench.py's
timer), answers checked against fp32 torch. The engine's pick: tile -1 (auto),
split-K from conv_pick_split_k.

  python tools/fc_bench.py [--tiles 0,1] [--splits 0,4,8,16]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dmlc  # noqa: E402
from dmlc import ops  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from conv_bench import time_us, warm_gpu  # noqa: E402

SHAPES = [("classifier.1", 9216, 4096, True), ("classifier.4", 4096, 4096, True), ("classifier.6", 4096, 1000, False)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--tiles", default="-1,0,1,2,7,8,b0,b1", help="conv_igemm tile ids; b0 / b1: conv_bigtile 256x256 / 256x128")
    ap.add_argument("--splits", default="0,2,4,8,16")
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(7)
    C = dmlc.native()
    warm_gpu()
    for name, K, N, relu in SHAPES:
        x = (torch.randn(a.batch, K, generator=g) * 0.5).bfloat16()
        w = (torch.randn(N, K, generator=g) / K ** 0.5).bfloat16()
        b = torch.randn(N, generator=g) * 0.1
        ref = x.float() @ w.float().t() + b
        if relu:
            ref = ref.relu()
        wp = ops.pack_conv_weight(w.float().view(N, K, 1, 1), device=dev)
        xg = x.view(a.batch, 1, 1, K).to(dev)
        bg = b.to(dev)
        flop = 2.0 * a.batch * K * N
        tiles = [C.CONV_BIGTILE0 + int(v[1:]) if v.startswith("b") else int(v) for v in a.tiles.split(",")]
        for t in tiles:
            for s in (int(v) for v in a.splits.split(",")):
                try:
                    def run():
                        return ops.conv2d(xg, wp, N, 1, 1, bias=bg, relu=relu, split_k=s, tile=t)
                    y = run()
                    torch.cuda.synchronize()
                except Exception as e:  # (unsupported tile / split for the shape)
                    print(f"{name} tile {t:2d} split {s:2d}: {type(e).__name__}: {e}", flush=True)
                    continue
                rel = ((y.float().cpu().view(a.batch, N) - ref).norm() / ref.norm()).item()
                us = time_us(run, a.iters)
                print(f"{name} K={K} N={N} tile {t:2d} split {s:2d}: {us:7.1f} us  {flop / us / 1e6:7.1f} TF/s  "
                      f"{(K * N * 2) / us / 1e6:5.2f} TB/s weights  rel {rel:.1e}", flush=True)


if __name__ == "__main__":
    main()
