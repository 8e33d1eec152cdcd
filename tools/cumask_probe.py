#!/usr/bin/env python3
"""EXPERIMENT: two B=128 ResNet18 engines on CU-masked streams (each half of
the CUs) running concurrently vs the two-lane B=256 scheme (two B=256
engines alternating on plain streams). Images/s over --iters iterations."""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--layout", default="halves", choices=["halves", "interleave", "xcd"])
    a = ap.parse_args()
    import dmlc
    from dmlc.models import build, state_dict_f32
    from dmlc.runtime import InferenceEngine
    C = dmlc.native()
    dev = torch.device("cuda", 0)
    sd = state_dict_f32(build("resnet18", seed=0))
    img = torch.randint(0, 256, (256, 224, 224, 3), dtype=torch.uint8, device=dev)
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count

    def run(engs, streams, halves):
        outs = [(torch.empty(256, dtype=torch.int32, device=dev), torch.empty(256, dtype=torch.float32, device=dev))
                for _ in engs]
        def it(i):
            if halves:
                for k, (e, s) in enumerate(zip(engs, streams)):
                    with torch.cuda.stream(s):
                        e.predict(img[128 * k:128 * (k + 1)], out=(outs[k][0][:128], outs[k][1][:128]))
            else:
                k = i % 2
                with torch.cuda.stream(streams[k]):
                    engs[k].predict(img, out=outs[k])
        for i in range(20):
            it(i)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for i in range(a.iters):
            it(i)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        n = 256 * a.iters if halves else 256 * a.iters
        return n / dt

    base = [InferenceEngine("resnet18", sd, device=0, max_batch=256) for _ in range(2)]
    plain = [torch.cuda.Stream(), torch.cuda.Stream()]
    print(f"two lanes B=256 alternating: {run(base, plain, False):,.0f} img/s", flush=True)
    del base
    os.environ["DMLC_EXP_NUM_CUS"] = str(ncu // 2)
    halfe = [InferenceEngine("resnet18", sd, device=0, max_batch=128) for _ in range(2)]
    words = (ncu + 31) // 32
    for layout in ["halves", "interleave", "xcd"]:
        masks = []
        for k in range(2):
            m = [0] * words
            for c in range(ncu):
                if layout == "halves":
                    on = (c < ncu // 2) == (k == 0)
                elif layout == "interleave":
                    on = (c % 2) == k
                else:  # alternate groups of 16
                    on = ((c // 16) % 2) == k
                if on:
                    m[c // 32] |= 1 << (c % 32)
            masks.append(m)
        ss = [torch.cuda.ExternalStream(C.cu_masked_stream(0, m)) for m in masks]
        print(f"two B=128 engines on CU-masked halves ({layout}): {run(halfe, ss, True):,.0f} img/s", flush=True)
    plain2 = [torch.cuda.Stream(), torch.cuda.Stream()]
    print(f"two B=128 engines, unmasked streams: {run(halfe, plain2, True):,.0f} img/s", flush=True)
    base = [InferenceEngine("resnet18", sd, device=0, max_batch=256) for _ in range(2)]
    os.environ.pop("DMLC_EXP_NUM_CUS")
    print(f"(engines built with 128 CUs) two lanes B=256 alternating: {run(base, plain, False):,.0f} img/s", flush=True)


if __name__ == "__main__":
    main()
