#!/usr/bin/env python3
"""Whole-forward A/B of kernel variants inside the engine (ResNet18 / ResNet50
at B=256, random-init weights, u8 224x224 images): each variant is a set of
native tuning hooks (kernel variant / debug bits) applied around an eager
forward captured REP times in a graph and replayed (tools/conv_bench.py's
timer), variants interleaved over --rounds rounds in one process. Answers of
every non-default variant are checked bit-identical to the default first
(a variant that changes numerics fails unless --allow-diff).

  python tools/engine_ab.py --model resnet18 --variants "stream=0;stream=64"

Hooks: stream (conv3x3_stream_set_variant), stream8 (conv3x3_stream8_set_variant),
stem (stem_conv_pool_set_dbg), stag_<family>=N (kernel_stagger_set: workgroup
start stagger of stream / block / rows28 / s2rows / stem / stream8 / conv1x1 /
bottleneck kernels), comma-separated within a variant."""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dmlc  # noqa: E402
from dmlc.models import build, state_dict_f32  # noqa: E402
from dmlc.runtime import InferenceEngine  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from conv_bench import time_us, warm_gpu  # noqa: E402

HOOKS = {"stream": "conv3x3_stream_set_variant", "stream8": "conv3x3_stream8_set_variant",
         "stem": "stem_conv_pool_set_dbg"}
# workgroup start stagger per kernel family (kernels.h StaggerKernel): stag_<family>=N
STAG = {"stag_stream": 0, "stag_block": 1, "stag_rows28": 2, "stag_s2rows": 3, "stag_stem": 4, "stag_stream8": 5,
        "stag_conv1x1": 6, "stag_bottleneck": 7}


def parse(spec):
    out = {}
    for kv in filter(None, spec.split(",")):
        k, v = kv.split("=")
        if k not in HOOKS and k not in STAG:
            raise SystemExit(f"unknown hook {k} (known: {', '.join(HOOKS)})")
        out[k] = int(v, 0)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet18")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", default="stream=0;stream=64")
    ap.add_argument("--allow-diff", action="store_true")
    a = ap.parse_args()
    C = dmlc.native()
    dev = torch.device("cuda", 0)
    sd = state_dict_f32(build(a.model, seed=3, randomize_bn=True))
    eng = InferenceEngine(a.model, sd, device=0, max_batch=a.batch)
    g = torch.Generator().manual_seed(4)
    img = torch.randint(0, 256, (a.batch, 224, 224, 3), generator=g, dtype=torch.uint8).to(dev)
    variants = [v.strip() for v in a.variants.split(";") if v.strip()]

    def run(spec):
        hooks = parse(spec)
        for k, v in hooks.items():
            if k in STAG:
                C.kernel_stagger_set(STAG[k], v)
            else:
                getattr(C, HOOKS[k])(v)
        try:
            return eng.predict(img, use_graph=False)
        finally:
            for k in hooks:
                if k in STAG:
                    C.kernel_stagger_set(STAG[k], -1)
                else:
                    getattr(C, HOOKS[k])(0)

    ref = [t.clone() for t in run("")]
    torch.cuda.synchronize()
    for v in variants:
        out = run(v)
        torch.cuda.synchronize()
        same = all(torch.equal(x, y) for x, y in zip(out, ref))
        print(f"variant [{v}]: answers bit-identical to the default: {same}", flush=True)
        if not same and not a.allow_diff:
            raise SystemExit(f"variant [{v}] changes the answers")
    warm_gpu()
    res = {v: [] for v in variants}
    for _ in range(a.rounds):
        for v in variants:
            res[v].append(time_us(lambda: run(v), a.iters))
    for v in variants:
        med = statistics.median(res[v])
        print(f"{a.model} b{a.batch} [{v:24s}] forward median {med:8.1f} us  ({a.batch / med * 1e6:9.0f} img/s "
              f"single lane)  all {' '.join(f'{t:.1f}' for t in res[v])}", flush=True)


if __name__ == "__main__":
    main()
