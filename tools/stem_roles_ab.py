#!/usr/bin/env python3
"""Knock-out timings of the role-split ResNet stem (stem_pool.hip
stem_roles_kernel<7, V>, V bits: 1 16-B raw-row DMA, 2 dense K (5 K steps a
fragment instead of 7), 4 no u8 conversion, 8 no conv rows, 16 no
pooling epilogue, 32 no DMA / vertical max / stores) at B=256, 224x224 u8
images, graph-replayed, interleaved over --rounds rounds in one process
(tools/conv_bench.py's timer). The variants this tool A/B'd in round 4
(pipelined operand reloads, rotated helper stores, the packed pooling
epilogue) are in profiles/r4_stem_roles.txt."""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dmlc  # noqa: E402
from dmlc import ops  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from conv_bench import time_us, warm_gpu  # noqa: E402

NAMES = {0: "paired, 4-B DMA", 1: "paired (round 5 default)", 3: "dense K (default)", 7: "dense, KO u8 conversion",
         19: "dense, KO h-pool epilogue", 43: "dense, conversion only", 55: "dense, MFMA only", 4: "KO u8 conversion", 8: "KO conv rows", 9: "KO conv rows, 16-B raw DMA",
         16: "KO h-pool epilogue", 36: "MFMA + h-pool only", 52: "MFMA only", 40: "conversion only",
         -1: "4-B raw-row DMA (round 4)"}
KNOCKOUTS = {4, 8, 9, 16, 36, 52, 40, 7, 19, 43, 55}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", default="1,3,55,19,7")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(5)
    B = args.batch
    img = torch.randint(0, 256, (B, 224, 224, 3), generator=g, dtype=torch.uint8).to(dev)
    w = torch.randn(64, 3, 7, 7, generator=g) / 12
    wp = ops.pack_stem_pool_weight(w, device=dev)
    wd = ops.pack_stem_dense_weight(w, device=dev)
    bias = (torch.randn(64, generator=g) * 0.1).to(dev)
    C = dmlc.native()
    vs = [int(t) for t in args.variants.split(",")]

    def run(v):
        C.stem_conv_pool_set_dbg(2048 if v == -1 else v << 24)
        try:
            return ops.stem_conv_pool_u8(img, wp, bias, 56, w_dense=wd if v > 0 and v & 2 else None)
        finally:
            C.stem_conv_pool_set_dbg(0)

    ref = run(0).clone()
    torch.cuda.synchronize()
    for v in vs:
        if v in KNOCKOUTS:  # timing only
            continue
        out = run(v)
        torch.cuda.synchronize()
        same = torch.equal(out.view(torch.int16), ref.view(torch.int16))
        diff = (out.float() - ref.float()).abs()
        print(f"variant {v} ({NAMES.get(v, '')}): bit-identical to variant 0: {same} "
              f"(max abs diff {diff.max().item():.3g}, {(diff > 0).float().mean().item():.2%} differ)", flush=True)
        # dense K sums the same products in another order: one bf16 ulp at most
        if not same and not (v & 2 and bool((diff <= ref.float().abs() * 2.0 ** -7 + 1e-6).all())):
            raise SystemExit(f"variant {v} differs: max abs {diff.max().item()}")
    warm_gpu()
    res = {v: [] for v in vs}
    for _ in range(args.rounds):
        for v in vs:
            res[v].append(time_us(lambda: run(v), args.iters))
    for v in vs:
        print(f"variant {v} {NAMES.get(v, ''):28s} median {statistics.median(res[v]):7.1f} us  "
              f"all {' '.join(f'{t:.1f}' for t in res[v])}", flush=True)


if __name__ == "__main__":
    main()
