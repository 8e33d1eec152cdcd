#!/usr/bin/env python3
"""Framework baseline on the same GPU: the torch.nn ResNet18 (our reference
model definition) in PyTorch-ROCm eager bf16, channels_last (MIOpen convs,
hipBLASLt FC), including input normalisation and softmax/top-1, batch 256.
For comparison with bench.py (hand-written HIP engine)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dmlc.models import build  # noqa: E402


def main():
    B = int(os.environ.get("B", "256"))
    steps = int(os.environ.get("STEPS", "30"))
    dev = torch.device("cuda", 0)
    m = build("resnet18").to(dev).bfloat16().to(memory_format=torch.channels_last).eval()
    imgs = torch.randint(0, 256, (B, 224, 224, 3), dtype=torch.uint8, device=dev)
    mean = torch.tensor([0.485, 0.456, 0.406], device=dev).view(1, 3, 1, 1)
    std = torch.tensor([0.229, 0.224, 0.225], device=dev).view(1, 3, 1, 1)

    def step():
        with torch.no_grad():
            x = ((imgs.permute(0, 3, 1, 2).float() / 255 - mean) / std).bfloat16().contiguous(
                memory_format=torch.channels_last)
            p = torch.softmax(m(x).float(), -1)
            return p.max(-1)

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / steps
    print(json.dumps({"baseline": "pytorch-eager-bf16-channels_last (MIOpen)", "model": "resnet18", "batch": B,
                      "ms_per_step": round(dt * 1e3, 3), "images_per_s": round(B / dt, 1)}))


if __name__ == "__main__":
    main()
