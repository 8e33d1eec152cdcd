"""GPU inference engine (Python face of csrc/runtime/engine.cpp).

Reference counterpart: ``Member::predict`` (src/services.rs:475-497) — one
image per call, CPU libtorch, model mutex. Here one call classifies a whole
batch of u8 images already resident in HBM: on-device preprocess, the
hand-written MFMA conv stack, fused softmax+top-1, all replayed from a
hipGraph captured on first use.
"""
from __future__ import annotations

import torch

from . import native
from .models import build, state_dict_f32


def require_gpu() -> None:
    if not torch.cuda.is_available():
        raise RuntimeError("dmlc GPU engine needs a ROCm GPU (torch.cuda.is_available() is False)")


class InferenceEngine:
    """Batched classifier on one GPU.

    weights: None (random init of ``arch`` with ``seed``), a state dict, or a
    path to a ``.ot`` checkpoint. options: kernel-path switches by name
    (csrc/runtime/engine.h EngineOptions, e.g. {"fused_block": False}); the
    defaults are the fastest measured paths.
    """

    def __init__(self, arch: str = "resnet18", weights=None, device: int = 0, max_batch: int = 256,
                 num_classes: int = 1000, image_size: int = 224, seed: int = 0, options: dict | None = None):
        require_gpu()
        C = native()
        self.arch = arch
        self.device = torch.device("cuda", device)
        if isinstance(weights, str):
            self._e = C.Engine.from_ot(arch, weights, device, num_classes, image_size, dict(options or {}))
        else:
            sd = weights if weights is not None else state_dict_f32(build(arch, num_classes, seed=seed))
            self._e = C.Engine(arch, {k: v.detach().cpu().float().numpy() for k, v in sd.items()},
                               device, num_classes, image_size, dict(options or {}))
        self._e.reserve(max_batch)
        self.max_batch = max_batch
        self.num_classes = num_classes
        self.image_size = image_size

    @property
    def gflop_per_image(self) -> float:
        return self._e.gflop_per_image

    @property
    def weight_bytes(self) -> int:
        return self._e.weight_bytes

    def predict(self, images: torch.Tensor, use_graph: bool = True, out=None, return_logits: bool = False):
        """images: uint8 [B,H,W,3] on this engine's GPU. Returns (idx int32 [B],
        prob f32 [B]) (+ logits f32 [B,num_classes] if return_logits)."""
        if images.device != self.device or images.dtype != torch.uint8 or images.dim() != 4 or images.shape[-1] != 3:
            raise ValueError(f"expected uint8 [B,H,W,3] on {self.device}, got {images.dtype} {tuple(images.shape)} "
                             f"on {images.device}")
        if not images.is_contiguous():
            raise ValueError("images must be contiguous")
        B, H, W, _ = images.shape
        if out is None:
            idx = torch.empty(B, dtype=torch.int32, device=self.device)
            prob = torch.empty(B, dtype=torch.float32, device=self.device)
        else:
            idx, prob = out
        logits = torch.empty(B, self.num_classes, dtype=torch.float32, device=self.device) if return_logits else None
        self._e.forward(images.data_ptr(), B, H, W, idx.data_ptr(), prob.data_ptr(),
                        0 if logits is None else logits.data_ptr(),
                        torch.cuda.current_stream(self.device).cuda_stream, use_graph)
        return (idx, prob, logits) if return_logits else (idx, prob)

    def profile(self, images: torch.Tensor) -> list[tuple[str, float]]:
        """Per-op GPU time (ms) of one eager forward (hipEvent pairs)."""
        B, H, W, _ = images.shape
        return self._e.profile(images.data_ptr(), B, H, W, torch.cuda.current_stream(self.device).cuda_stream)
