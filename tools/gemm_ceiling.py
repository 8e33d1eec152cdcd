#!/usr/bin/env python3
"""Library-GEMM ceiling for ResNet18's b256 3x3 convs: times torch.mm
(hipBLASLt) in bf16 on each conv's implicit-GEMM shape [B*Ho*Wo, 9*Cin] x
[9*Cin, Cout] (the im2col copy itself not included), to price what an MFMA
GEMM of that shape reaches on this GPU vs the direct convs' times."""
import statistics

import torch

SHAPES = [  # name, M, K, N
    ("layer1 3x3 56x56x64", 256 * 56 * 56, 576, 64),
    ("layer2.0 conv1 s2 ->28x28x128", 256 * 28 * 28, 576, 128),
    ("layer2 3x3 28x28x128", 256 * 28 * 28, 1152, 128),
    ("layer3.0 conv1 s2 ->14x14x256", 256 * 14 * 14, 1152, 256),
    ("layer3 3x3 14x14x256", 256 * 14 * 14, 2304, 256),
    ("layer4.0 conv1 s2 ->7x7x512", 256 * 7 * 7, 2304, 512),
    ("layer4 3x3 7x7x512", 256 * 7 * 7, 4608, 512),
]


def main():
    dev = torch.device("cuda", 0)
    for name, M, K, N in SHAPES:
        a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        b = torch.randn(K, N, device=dev, dtype=torch.bfloat16)
        for _ in range(3):
            torch.mm(a, b)
        torch.cuda.synchronize()
        ts = []
        for _ in range(15):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                torch.mm(a, b)
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3 / 5)
        us = statistics.median(ts)
        print(f"{name:32s} M={M:7d} K={K:5d} N={N:4d}  {us:7.1f} us  {2 * M * K * N / us / 1e6:7.1f} TFLOP/s",
              flush=True)
        del a, b


if __name__ == "__main__":
    main()
