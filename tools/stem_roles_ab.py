#!/usr/bin/env python3
"""A/B of the one-image-per-workgroup ResNet stem (stem_pool.hip
stem_roles_kernel) at B=256, 224x224 u8 images, graph-replayed, interleaved
over --rounds rounds in one process (tools/conv_bench.py's timer): the paired
layout (7 K steps a fragment, round 5) against the dense-K layout (5 K steps,
the engine's default: ops.stem_conv_pool_u8(..., w_dense=...)), and the 4-B
raw-row DMA form of the paired kernel. The phase knock-outs of both layouts
are in profiles/r4_stem_roles.txt and profiles/r6_stem_dense.txt."""
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

VARIANTS = {"paired": (512, False), "dense": (512, True), "paired4": (512 | 2048, False)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", default="paired,dense,paired4")
    ap.add_argument("--stamps", action="store_true",
                    help="per-step phase stamps of each variant (stem_conv_pool_set_stamps), after the timing")
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
    vs = args.variants.split(",")

    def run(v):
        dbg, dense = VARIANTS[v]
        C.stem_conv_pool_set_dbg(dbg)
        try:
            return ops.stem_conv_pool_u8(img, wp, bias, 56, w_dense=wd if dense else None)
        finally:
            C.stem_conv_pool_set_dbg(0)

    ref = run("paired").clone()
    torch.cuda.synchronize()
    for v in vs:
        out = run(v)
        torch.cuda.synchronize()
        diff = (out.float() - ref.float()).abs()
        print(f"{v}: max abs diff vs paired {diff.max().item():.3g}, {(diff > 0).float().mean().item():.3%} differ",
              flush=True)
        # dense K sums the same products in another order: one bf16 ulp at most
        if not bool((diff <= ref.float().abs() * 2.0 ** -7 + 1e-6).all()):
            raise SystemExit(f"{v} differs beyond one bf16 ulp")
    warm_gpu()
    res = {v: [] for v in vs}
    for _ in range(args.rounds):
        for v in vs:
            res[v].append(time_us(lambda: run(v), args.iters))
    for v in vs:
        print(f"{v:8s} median {statistics.median(res[v]):7.1f} us  all {' '.join(f'{t:.1f}' for t in res[v])}",
              flush=True)
    if args.stamps:
        steps = 56 // 2 + 2
        for v in vs:
            st = torch.zeros(16 * steps * 4, dtype=torch.int64, device=dev)
            for _ in range(3):  # (the last launch's stamps, warm)
                C.stem_conv_pool_set_stamps(st.data_ptr())
                run(v)
                C.stem_conv_pool_set_stamps(0)
            torch.cuda.synchronize()
            a = st.view(16, steps, 4).double().cpu() * 10e-3  # 100 MHz ticks -> us
            t0 = a[:, 0, 0].view(16, 1)
            start = a[:, :, 0] - t0
            mfma = a[:, :, 1] - a[:, :, 0]
            helper = a[:, :, 2] - a[:, :, 0]
            hwait = a[:, :, 3] - a[:, :, 2]
            step = torch.cat([start[:, 1:] - start[:, :-1], torch.zeros(16, 1)], 1)

            def med(x, j):
                return x[:, j].median().item()

            print(f"{v}: per-step medians over 16 workgroups (us): step t / step length / MFMA wave 0 phase / "
                  "helper wave 4 work issued / helper waits", flush=True)
            for j in range(steps):
                print(f"  t={j:2d} start {med(start, j):6.2f} len {med(step, j):5.2f} mfma {med(mfma, j):5.2f} "
                      f"helper {med(helper, j):5.2f} wait {med(hwait, j):5.2f}")
            end = a[:, steps - 1, 3] - a[:, 0, 0]
            print(f"  total (start to last helper wait) median {end.median().item():.2f} us", flush=True)


if __name__ == "__main__":
    main()
