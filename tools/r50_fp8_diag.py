#!/usr/bin/env python3
"""ResNet50 e4m3 engine variants vs the fp32 reference at a batch size:
relative logit error and top-1 agreement on the first 16 images (diagnostic
for the e4m3 3x3-output option)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from dmlc.models import build, state_dict_f32  # noqa: E402
from dmlc.runtime import InferenceEngine  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
model = build("resnet50", seed=63, randomize_bn=True).eval()
sd = state_dict_f32(model)
g = torch.Generator().manual_seed(64)
img = torch.randint(0, 256, (B, 224, 224, 3), generator=g, dtype=torch.uint8)
x = img.to("cuda")
with torch.no_grad():
    mean = torch.tensor([0.485, 0.456, 0.406]).view(1, 3, 1, 1)
    std = torch.tensor([0.229, 0.224, 0.225]).view(1, 3, 1, 1)
    ref = model((img[:16].permute(0, 3, 1, 2).float() / 255 - mean) / std)
variants = {"fp8_3x3_out off": {"fp8_3x3_out": False},
            "fp8_3x3_out on": {"fp8_3x3_out": True},
            "fp8_3x3_out on, no ds_into_expand": {"fp8_3x3_out": True, "ds_into_expand": False},
            "fp8_3x3_out on, no stream_conv": {"fp8_3x3_out": True, "stream_conv": False},
            "fp8_3x3_out on, strided too": {"fp8_3x3_out": True, "fp8_3x3_out_s2": True}}
out = {}
for name, opts in variants.items():
    eng = InferenceEngine("resnet50_fp8", sd, max_batch=B, options=opts)
    for graph in (False, True):
        i, p, lg = eng.predict(x, return_logits=True, use_graph=graph)
        torch.cuda.synchronize()
        lg = lg.float().cpu()
        rel = ((lg[:16] - ref).norm() / ref.norm()).item()
        agree = (lg[:16].argmax(-1) == ref.argmax(-1)).float().mean().item()
        out[(name, graph)] = i.cpu()
        print(f"B={B} {name:36s} graph={graph}: rel {rel:.4f} top1 vs fp32 {agree:.3f}", flush=True)
base = out[("fp8_3x3_out off", True)]
for k, v in out.items():
    print(f"  top1 agreement with fp8_3x3_out off (graph): {k}: {(v == base).float().mean().item():.3f}")
