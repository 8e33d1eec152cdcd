#!/usr/bin/env python3
"""A/B of the role-split ResNet stem (stem_pool.hip stem_roles_kernel<7, V>)
variants at B=256, 224x224 u8 images: each variant's output must be
bit-identical to the default's (same arithmetic, only the issue order and the
helpers' store order differ), then graph-replayed timings, interleaved over
--rounds rounds in one process (tools/conv_bench.py's timer)."""
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

NAMES = {0: "default", 1: "pipelined operand reloads", 2: "rotated helper stores", 3: "both",
         4: "KO u8 conversion", 8: "KO conv rows", 16: "KO h-pool epilogue",
         36: "MFMA + h-pool only", 52: "MFMA only", 40: "conversion only",
         64: "packed bf16 pooling"}
KNOCKOUTS = {4, 8, 16, 36, 52, 40}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", default="0,1,2,3")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(5)
    B = args.batch
    img = torch.randint(0, 256, (B, 224, 224, 3), generator=g, dtype=torch.uint8).to(dev)
    w = torch.randn(64, 3, 7, 7, generator=g) / 12
    wp = ops.pack_stem_pool_weight(w, device=dev)
    bias = (torch.randn(64, generator=g) * 0.1).to(dev)
    C = dmlc.native()
    vs = [int(t) for t in args.variants.split(",")]

    def run(v):
        C.stem_conv_pool_set_dbg(v << 24)
        try:
            return ops.stem_conv_pool_u8(img, wp, bias, 56)
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
        print(f"variant {v} ({NAMES.get(v, '')}): bit-identical to the default: {same}", flush=True)
        if v & 64:  # bias accumulated from the start: rounding may differ by an ulp
            d = (out.float() - ref.float()).abs()
            rel = (d / ref.float().abs().clamp_min(1e-3)).max().item()
            print(f"  max abs diff {d.max().item():.4g}, max rel {rel:.3g}, differing {(d > 0).float().mean().item():.4%}")
            if d.max().item() > 0.05 * ref.float().abs().max().item():
                raise SystemExit(f"variant {v} out of tolerance")
            continue
        if not same:
            raise SystemExit(f"variant {v} differs: max abs {(out.float() - ref.float()).abs().max().item()}")
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
