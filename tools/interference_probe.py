#!/usr/bin/env python3
"""How much does a concurrent kernel on another stream slow the ResNet18
forward? (Rehearses what an RCCL scatter/gather kernel does to a rank's
compute in the N>1 bench, on one GPU.)

Modes, each timed over graph-replayed b256 forwards:
  none     forward alone
  sleepK   K single-wave spin kernels (torch.cuda._sleep) on K side streams,
           each lasting about one forward: K CUs partly held the whole time,
           like a long-lived RCCL p2p kernel with K blocks
  copy     a side-stream D2D copy of 7 x 38.5 MB per forward (HBM traffic of
           the coordinator's u8 shards at N=8)
  rcclK    real RCCL kernels: a one-rank communicator (CTA cap K, 0 = RCCL's
           default) moves 7 x 38.5 MB to itself by grouped send/recv on a
           high-priority side stream per forward -- the coordinator's
           scatter legs, with their CTA/LDS footprint, minus the xGMI hop
  rcclK:L  the same with L legs (L = 1: what a receiving rank runs per step)

--batches b1,b2,...: every mode at each forward batch (the coordinator's
weighted share vs a worker's full batch: bench.py --coord-weight).
--leg-images: images per leg (default: the batch).
"""
import argparse
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--modes", default="none,sleep1,sleep4,sleep16,sleep32,copy")
    ap.add_argument("--batches", default="")
    ap.add_argument("--leg-images", type=int, default=0)
    args = ap.parse_args()
    for b in ([int(x) for x in args.batches.split(",")] if args.batches else [args.batch]):
        print(f"## batch {b}", flush=True)
        run(args, b)


def run(args, B):
    import dmlc
    from dmlc.runtime import InferenceEngine
    dev = torch.device("cuda", 0)
    eng = InferenceEngine("resnet18", None, device=0, max_batch=B)
    LB = args.leg_images or B
    img = torch.randint(0, 256, (B, 224, 224, 3), dtype=torch.uint8, device=dev)
    out = (torch.empty(B, dtype=torch.int32, device=dev), torch.empty(B, dtype=torch.float32, device=dev))
    main_s = torch.cuda.current_stream()
    side = [torch.cuda.Stream() for _ in range(32)]
    src = torch.empty(7 * LB * 224 * 224 * 3, dtype=torch.uint8, device=dev)
    dst = torch.empty_like(src)
    hi = torch.cuda.Stream(priority=-1)
    loops = {}

    def fwd():
        eng.predict(img, out=out)

    for _ in range(10):
        fwd()
    torch.cuda.synchronize()
    # cycles per ms for _sleep: calibrate
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    torch.cuda._sleep(1_000_000)
    e1.record()
    torch.cuda.synchronize()
    cyc_per_ms = 1_000_000 / e0.elapsed_time(e1)

    base = None
    for mode in args.modes.split(","):
        times = []
        for it in range(args.iters):
            torch.cuda.synchronize()
            ev = torch.cuda.Event()
            ev.record(main_s)
            if mode.startswith("sleep"):
                k = int(mode[5:])
                for j in range(k):
                    side[j].wait_event(ev)
                    with torch.cuda.stream(side[j]):
                        torch.cuda._sleep(int(cyc_per_ms * 1.3))
            elif mode.startswith("rccl"):
                spec = mode[4:].split(":")
                k = int(spec[0])
                legs = int(spec[1]) if len(spec) > 1 else 7
                if k not in loops:
                    loops[k] = dmlc.native().RcclLoop(0, k)
                if mode not in loops:
                    loops[mode] = True
                    ts = []
                    for _ in range(6):  # the legs alone
                        x0, x1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        x0.record(hi)
                        loops[k].issue(hi.cuda_stream, src.data_ptr(), dst.data_ptr(), LB * 224 * 224 * 3, legs)
                        x1.record(hi)
                        torch.cuda.synchronize()
                        ts.append(x0.elapsed_time(x1))
                    print(f"{mode:8s} {legs} x {LB * 224 * 224 * 3 / 1e6:.1f} MB self send/recv alone: "
                          f"{sorted(ts[1:])[2]:.3f} ms", flush=True)
                hi.wait_event(ev)
                loops[k].issue(hi.cuda_stream, src.data_ptr(), dst.data_ptr(), LB * 224 * 224 * 3, legs)
            elif mode == "copy":
                side[0].wait_event(ev)
                with torch.cuda.stream(side[0]):
                    dst.copy_(src)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(main_s)
            fwd()
            b.record(main_s)
            torch.cuda.synchronize()
            times.append(a.elapsed_time(b))
        times.sort()
        med = times[len(times) // 2]
        if base is None:
            base = med
        print(f"{mode:8s} forward median {med:.3f} ms  ({med / base:.2f}x)  min {times[0]:.3f}", flush=True)


if __name__ == "__main__":
    main()
