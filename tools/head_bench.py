#!/usr/bin/env python3
"""Time the pooled classifier head (head.hip) alone: graph-replayed launches,
per-launch GPU time, by class split count and knock-out bits (ko 2: no fc
weight loads). usage: python tools/head_bench.py [K (512: ResNet18, 2048:
ResNet50)]"""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import dmlc

C = dmlc.native()
B, N, NP = 256, 1000, 1008
K = int(sys.argv[1]) if len(sys.argv) > 1 else 512
dev = torch.device("cuda", 0)
pooled = torch.randn(B, K, device=dev).to(torch.bfloat16)
w = (torch.randn(NP, K, device=dev) * 0.05).to(torch.bfloat16)
bias = torch.randn(NP, device=dev)
logits = torch.empty(B, N, device=dev)
idx = torch.empty(B, dtype=torch.int32, device=dev)
prob = torch.empty(B, device=dev)
wsb = C.head_ws_bytes(B)
ws = torch.zeros(wsb, dtype=torch.uint8, device=dev)
cus = torch.cuda.get_device_properties(0).multi_processor_count


def run(ns, ko, reps=200):
    """Back-to-back eager launches (host launch ~5 us < kernel time), timed by events."""
    s = torch.cuda.current_stream().cuda_stream
    f = lambda: C.head_pooled(pooled.data_ptr(), w.data_ptr(), bias.data_ptr(), B, K, N, K, NP, logits.data_ptr(),
                              idx.data_ptr(), prob.data_ptr(), ws.data_ptr(), wsb, cus, s, ns, ko)
    for _ in range(5):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


ref = torch.softmax(pooled.float() @ w[:N].float().t() + bias[:N], -1)
for ns in (0, 4, 8, 16):
    us = run(ns, 0)
    ok = torch.equal(idx.long().cpu(), ref.argmax(-1).cpu())
    print(f"ns={ns or 'auto'}: {us:.2f} us/launch  top1 ok={ok}  (ko=2: {run(ns, 2):.2f} us)")
