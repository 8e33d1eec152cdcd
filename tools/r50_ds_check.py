#!/usr/bin/env python3
"""Diagnostic: ResNet50 (bf16 / fp8) logits vs the fp32 torch model with the
layer1.0 downsample folded into its expand conv (ds_into_expand) on and off,
eager and graph, at two batch sizes."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from dmlc.models import build, state_dict_f32  # noqa: E402
from dmlc.runtime import InferenceEngine  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    model = build("resnet50", seed=63, randomize_bn=True)
    sd = state_dict_f32(model)
    g = torch.Generator().manual_seed(64)
    img = torch.randint(0, 256, (32, 224, 224, 3), generator=g, dtype=torch.uint8)
    x = img.permute(0, 3, 1, 2).float() / 255.0
    mean = torch.tensor([0.485, 0.456, 0.406]).view(1, 3, 1, 1)
    std = torch.tensor([0.229, 0.224, 0.225]).view(1, 3, 1, 1)
    with torch.no_grad():
        ref = model((x - mean) / std).float()
    for arch in ("resnet50", "resnet50_fp8"):
        for on in (1, 0):
            for mb in (16, 64):
                eng = InferenceEngine(arch, sd, max_batch=mb, options={"ds_into_expand": bool(on)})
                for graph in (False, True):
                    outs = []
                    for b0 in range(0, 32, 16):
                        _, _, lg = eng.predict(img[b0:b0 + 16].to(dev), return_logits=True, use_graph=graph)
                        outs.append(lg.float().cpu())
                    lg = torch.cat(outs)
                    rel = ((lg - ref).norm() / ref.norm()).item()
                    print(f"{arch:13s} ds_into_expand={on} max_batch={mb} graph={int(graph)} rel={rel:.4f}", flush=True)
                del eng
                torch.cuda.synchronize()


if __name__ == "__main__":
    main()
