"""libtorch ``.ot`` checkpoint I/O — the format of the reference's
``pretrained_models/{resnet18,alexnet}.ot`` (loaded with ``VarStore::load`` at
src/services.rs:516,522). The archive is written/read by the native
``torch::serialize`` code in csrc/runtime/ot_io.cpp; keys use ``|`` for ``.``.
"""
from __future__ import annotations

import os

import numpy as np
import torch


def save_ot(path: str, state: dict) -> None:
    from .. import native
    arrs = {k: (v.detach().cpu().float().numpy() if isinstance(v, torch.Tensor) else np.asarray(v, np.float32))
            for k, v in state.items()}
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    native().ot_save(path, arrs)


def load_ot(path: str) -> dict[str, torch.Tensor]:
    from .. import native
    if not os.path.exists(path):
        raise FileNotFoundError(path)
    return {k: torch.from_numpy(v) for k, v in native().ot_load(path).items()}


def load_ot_jit(path: str) -> dict[str, torch.Tensor]:
    """Independent reader (TorchScript loader), used to cross-check the
    native archive writer in tests."""
    m = torch.jit.load(path, map_location="cpu")
    out = {k.replace("|", "."): v.detach() for k, v in m.named_parameters()}
    out.update({k.replace("|", "."): v.detach() for k, v in m.named_buffers()})
    return out


def write_random_checkpoint(arch: str, path: str, seed: int = 0, num_classes: int = 1000,
                            randomize_bn: bool = False) -> str:
    """Random-init weights of ``arch`` written as ``.ot`` (the reference's real
    weights are git-LFS pointer stubs, pretrained_models/*.ot:1-3).
    randomize_bn: non-trivial BN statistics, so predictions vary by image."""
    from ..models import build, state_dict_f32
    save_ot(path, state_dict_f32(build(arch, num_classes, seed=seed, randomize_bn=randomize_bn)))
    return path
