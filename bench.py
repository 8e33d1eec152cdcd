#!/usr/bin/env python3
"""Headline benchmark: ResNet18 ImageNet-shaped batch inference, images/s for
the whole node plus p50/p95 query latency (BASELINE.json metric).

One process per GPU (torchrun for N>1, RCCL = torch.distributed "nccl").
Each step of the timed loop is the whole serving path of the north star:

  rank 0 holds the staged image pool (u8 [*,224,224,3], HBM-resident)
   -> RCCL scatter of one u8 shard (per_gpu_batch images) to every rank
   -> on every GPU: preprocess + ResNet18 (hand-written MFMA kernels,
      hipGraph replay) + fused softmax/top-1
   -> RCCL gather of (top-1 class, probability) back to rank 0.

The scatter of step i+1 is issued before the forward of step i, so the xGMI
transfer overlaps compute (double-buffered input slots). ``--input-mode local``
skips the scatter (each rank reads its own HBM-resident shard).

Reference numbers (CS425MP4Report.pdf p.2): ResNet18 mean query latency
158.94 ms on CPU VMs, i.e. 6.29 images/s for one query stream; there is no
published images/s figure, so ``vs_baseline`` divides by that derived rate
and ``vs_baseline_latency`` compares latency directly.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

REF_MEAN_LATENCY_MS = 158.94  # ResNet18, CS425MP4Report.pdf p.2 §1a
REF_STREAM_IMG_S = 1000.0 / REF_MEAN_LATENCY_MS


def pct(xs, q):
    xs = sorted(xs)
    if not xs:
        return None
    k = (len(xs) - 1) * q / 100.0
    lo, hi = int(k), min(int(k) + 1, len(xs) - 1)
    return xs[lo] + (xs[hi] - xs[lo]) * (k - lo)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--model", default="resnet18")
    ap.add_argument("--batch", type=int, default=256, help="images per GPU per step")
    ap.add_argument("--input-mode", choices=["scatter", "local"], default="scatter")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--latency-queries", type=int, default=200, help="batch-1 queries for query latency")
    ap.add_argument("--profile-ops", action="store_true", help="print per-op times of one eager forward")
    ap.add_argument("--force-dist", action="store_true",
                    help="use the process group (RCCL scatter/gather) even for one rank: rehearses the N>1 path")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}; launch N>1 with torchrun")
    if world > 1:
        # Under the concurrent RCCL scatter/gather kernels a grid that exactly
        # fills the CUs loses a whole round when a few slots are taken: finer
        # row-conv strips (1792 instead of 512 workgroups) cost ~1% alone and
        # halve that loss (profiles/r1_interference.txt).
        os.environ.setdefault("DMLC_ROWS_STRIP", "8")
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    distributed = world > 1 or args.force_dist
    if distributed:
        dist.init_process_group("nccl", device_id=dev)

    from dmlc.models import build, state_dict_f32
    from dmlc.parallel import DPInference, broadcast_state_dict
    from dmlc.runtime import InferenceEngine

    B = args.batch
    # Rank 0 owns the weights (random init: the reference's .ot files are LFS
    # stubs) and broadcasts them over RCCL, like `train` distributing a model.
    sd = state_dict_f32(build(args.model, seed=0)) if rank == 0 else None
    sd = broadcast_state_dict(sd, 0, dev) if distributed else sd
    eng = InferenceEngine(args.model, sd, device=local_rank, max_batch=B)
    use_graph = not args.no_graph

    # Staged input pool (two global batches of distinct synthetic images) in
    # the coordinator's HBM, or every rank's own shard in local mode.
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    pool = None
    if rank == 0 or args.input_mode == "local":
        n_pool = 2 * (B * world if args.input_mode == "scatter" else B)
        pool = torch.randint(0, 256, (n_pool, 224, 224, 3), dtype=torch.uint8, device=dev, generator=g)

    dp = DPInference(lambda imgs, out: eng.predict(imgs, use_graph=use_graph, out=out), B, dev,
                     input_mode=args.input_mode)

    # Warmup (also captures the hipGraphs and warms RCCL channels).
    dp.run(pool, 0, args.warmup)
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    dp.run(pool, args.warmup, args.steps, stamps=False)
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if distributed:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()

    # Per-batch latency (scatter issue -> gathered top-1) from event stamps, in
    # a separate pass: the stamps' stream barriers would otherwise sit inside
    # the throughput measurement.
    n_lat = min(args.steps, 50)
    lat0 = args.warmup + args.steps
    dp.run(pool, lat0, n_lat)
    torch.cuda.synchronize()
    batch_lat = [dp.latency_ms(i) for i in range(lat0, lat0 + n_lat)]

    # Sanity: the coordinator's gathered outputs are valid class ids / probabilities.
    if rank == 0:
        ids, probs = dp.results(lat0 + n_lat - 1)
        assert ids.numel() == B * world
        assert int(ids.min()) >= 0 and int(ids.max()) < 1000, "bad class ids"
        assert float(probs.min()) > 0 and float(probs.max()) <= 1.0001, "bad probabilities"

    # Batch-1 query latency (hipGraph replay of preprocess+forward+top-1 for
    # one image, host-timed end to end including the D2H of the answer).
    qlat = []
    if rank == 0 and args.latency_queries > 0:
        q_eng = InferenceEngine(args.model, sd, device=local_rank, max_batch=1)
        qimg = pool[:1].contiguous()
        qout = (torch.empty(1, dtype=torch.int32, device=dev), torch.empty(1, dtype=torch.float32, device=dev))
        for i in range(args.latency_queries + 20):
            torch.cuda.synchronize()
            t = time.perf_counter()
            q_eng.predict(qimg, out=qout)
            _ = qout[0].item()
            if i >= 20:
                qlat.append((time.perf_counter() - t) * 1e3)

    ops_profile = None
    if rank == 0 and args.profile_ops:
        ops_profile = eng.profile(pool[:B].contiguous())

    if rank == 0:
        n_img = B * world * args.steps
        value = n_img / elapsed
        res = {
            "metric": "images/sec (whole node) + p50/p95 query latency, "
                      + ("ResNet18" if args.model == "resnet18" else args.model) + " ImageNet",
            "value": round(value, 1),
            "unit": "images/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(value / REF_STREAM_IMG_S, 1) if args.model == "resnet18" else None,
            "dtype": "fp8" if args.model.endswith("_fp8") else "bf16",
            "data": "synthetic u8 224x224x3 images (HBM-staged on rank 0), random-init weights",
            "config": {
                "model": args.model,
                "global_batch": B * world,
                "per_gpu_batch": B,
                "seq_len": None,
                "image_size": 224,
                "parallelism": f"dp{world}",
                "input_mode": args.input_mode,
                "hipgraph": use_graph,
                "baseline": "6.29 img/s = one query stream at the reference's 158.94 ms mean ResNet18 latency "
                            "(CS425MP4Report.pdf p.2; no images/s is published)",
            },
            "batch_latency_p50_ms": round(pct(batch_lat, 50), 3),
            "batch_latency_p95_ms": round(pct(batch_lat, 95), 3),
            "query_latency_p50_ms": round(pct(qlat, 50), 4) if qlat else None,
            "query_latency_p95_ms": round(pct(qlat, 95), 4) if qlat else None,
            "vs_baseline_latency": round(REF_MEAN_LATENCY_MS / pct(qlat, 50), 1) if qlat else None,
            "tflops_effective": round(value * eng.gflop_per_image / 1e3, 1),
        }
        if ops_profile:
            print("# per-op (ms): " + ", ".join(f"{n}={t:.3f}" for n, t in ops_profile), file=sys.stderr)
        print(json.dumps(res), flush=True)

    if distributed:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
