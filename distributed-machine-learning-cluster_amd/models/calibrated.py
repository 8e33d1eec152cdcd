"""Discriminating test models and inputs for the whole-model numerics tests.

A random-init network with arbitrary BN statistics maps every image to nearly
the same pooled features: on uniform-noise inputs the per-image part of the
logits is ~2% of their norm and the argmax is one class for the whole batch,
so an engine that returned the batch-mean logits would pass a relative-error
or top-1 check. The models here are calibrated on structured images instead:

* ResNets: BN statistics re-estimated on a calibration batch (train-mode
  forward, cumulative averages), so every layer's output is standardised and
  the features keep the input's structure;
* AlexNet (no BN): data-dependent init, each conv / linear layer in turn
  rescaled and re-biased so its pre-activations have zero mean and unit
  variance per channel over the calibration batch, then a random per-channel
  gain and shift (what a trained BN would leave) is applied;
* every model's classifier the same way (logits standardised per class), so
  the argmax follows the per-image part of the features, not the fc bias.

`discrimination()` measures what a test needs to know: how many distinct
top-1 classes a batch has and how large the per-image part of the logits is.
Used by tests/test_engine_gpu.py and __graft_entry__.smoke().
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from .reference import AlexNet, BasicBlock, Bottleneck, build

BRANCH_GAIN = 0.15
MEAN = torch.tensor([0.485, 0.456, 0.406]).view(1, 3, 1, 1)
STD = torch.tensor([0.229, 0.224, 0.225]).view(1, 3, 1, 1)


def normalize(u8: torch.Tensor) -> torch.Tensor:
    """uint8 [B,H,W,3] -> float [B,3,H,W], ImageNet mean / std (what the engine's stem does)."""
    return (u8.permute(0, 3, 1, 2).float() / 255 - MEAN) / STD


def pattern_images(n: int, seed: int = 0, size: int = 224) -> torch.Tensor:
    """uint8 [n,size,size,3]: per image, per channel a plane wave of random
    frequency, orientation and phase, plus a few random flat rectangles."""
    g = torch.Generator().manual_seed(seed)
    yy, xx = torch.meshgrid(torch.arange(size, dtype=torch.float32), torch.arange(size, dtype=torch.float32),
                            indexing="ij")
    out = torch.empty(n, size, size, 3, dtype=torch.uint8)
    for i in range(n):
        r = torch.rand(3, 4, generator=g)
        chans = []
        for c in range(3):
            f = 0.01 + 0.2 * r[c, 0].item() ** 2
            th = 2 * math.pi * r[c, 1].item()
            ph = 2 * math.pi * r[c, 2].item()
            amp = 0.3 + 0.7 * r[c, 3].item()
            chans.append(0.5 + 0.5 * amp * torch.sin((xx * math.cos(th) + yy * math.sin(th)) * f + ph))
        img = torch.stack(chans, -1)
        for _ in range(int(torch.randint(0, 4, (1,), generator=g))):
            y0, x0 = torch.randint(0, size - 16, (2,), generator=g).tolist()
            h, w = torch.randint(16, size // 2, (2,), generator=g).tolist()
            img[y0:y0 + h, x0:x0 + w] = torch.rand(3, generator=g)
        out[i] = (img * 255).clamp(0, 255).to(torch.uint8)
    return out


def noise_images(n: int, seed: int = 0, size: int = 224) -> torch.Tensor:
    return torch.randint(0, 256, (n, size, size, 3), dtype=torch.uint8, generator=torch.Generator().manual_seed(seed))


def mixed_images(n: int, seed: int = 0, size: int = 224, noise_frac: float = 0.25) -> torch.Tensor:
    """Structured images with a share of uniform-noise ones mixed in (interleaved)."""
    k = int(n * noise_frac)
    imgs = torch.cat([pattern_images(n - k, seed, size), noise_images(k, seed + 7919, size)])
    perm = torch.randperm(n, generator=torch.Generator().manual_seed(seed + 1))
    return imgs[perm].contiguous()


@torch.no_grad()
def _calibrate_bn(model: nn.Module, x: torch.Tensor) -> None:
    # Damp every residual branch (its last BN's gain and shift) before the
    # statistics are taken. A random-init BN network calibrated on its batch
    # is chaotic: a perturbation grows layer after layer, so a plain torch bf16
    # forward of ResNet50 was 31% off fp32 (ResNet34 8%, ResNet18 3.3%) and no
    # reduced-precision bar could be tight. With the branches at 0.15 of the
    # identity path (as trained ResNets' last-BN gains tend to be small, and
    # SkipInit / Fixup start them near zero) torch bf16 is 2.7% / 2.3% / 2.0%
    # off, while every layer still contributes.
    for mod in model.modules():
        if isinstance(mod, (BasicBlock, Bottleneck)):
            last = mod.bn3 if isinstance(mod, Bottleneck) else mod.bn2
            last.weight.mul_(BRANCH_GAIN)
            last.bias.mul_(BRANCH_GAIN)
    for mod in model.modules():
        if isinstance(mod, nn.BatchNorm2d):
            mod.reset_running_stats()
            mod.momentum = None
    model.train()
    for chunk in x.split(32):
        model(chunk)
    model.eval()


@torch.no_grad()
def _lsuv(model: nn.Module, layers: list[nn.Module], x: torch.Tensor, seed: int) -> None:
    """Data-dependent init of `layers` in order (each has a bias; the last is the classifier)."""
    g = torch.Generator().manual_seed(seed + 101)
    model.eval()
    for li, layer in enumerate(layers):
        captured = []
        h = layer.register_forward_hook(lambda m, i, o: captured.append(o.detach().clone()))  # before the in-place ReLU
        model(x)
        h.remove()
        y = captured[0]
        dims = [0, 2, 3] if y.dim() == 4 else [0]
        mu, sd = y.mean(dims), y.std(dims).clamp_min(1e-6)
        last = li == len(layers) - 1
        gain = torch.full_like(sd, 2.0) if last else 0.5 + torch.rand(sd.shape, generator=g)
        shift = torch.zeros_like(mu) if last else (torch.rand(mu.shape, generator=g) - 0.5) * 0.4
        shape = (-1,) + (1,) * (layer.weight.dim() - 1)
        layer.weight.mul_((gain / sd).view(shape))
        layer.bias.copy_((layer.bias - mu) * gain / sd + shift)


def calibrated(arch: str, seed: int = 0, n_calib: int = 64, num_classes: int = 1000) -> nn.Module:
    """Random-init `arch` (``_fp8`` suffix ignored) calibrated on structured +
    noise images so its top-1 and logits vary by image (module docstring)."""
    model = build(arch, num_classes, seed=seed, randomize_bn=True)
    x = normalize(mixed_images(n_calib, seed=10_000 + seed))
    if isinstance(model, AlexNet):
        _lsuv(model, [m for m in list(model.features) + list(model.classifier)
                      if isinstance(m, (nn.Conv2d, nn.Linear))], x, seed)
    else:
        _calibrate_bn(model, x)
        _lsuv(model, [model.fc], x, seed)  # standardise the logits per class too
    return model.eval()


def discrimination(logits: torch.Tensor) -> tuple[int, float]:
    """(distinct top-1 classes, per-image share of the logit norm
    ||L - mean_batch(L)|| / ||L||) of a [B, classes] batch of logits."""
    L = logits.float()
    share = ((L - L.mean(0, keepdim=True)).norm() / L.norm().clamp_min(1e-12)).item()
    return len(set(L.argmax(-1).tolist())), share


@torch.no_grad()
def e4m3_emulated_logits(model: nn.Module, images_u8: torch.Tensor, calib_u8: torch.Tensor | None = None) -> torch.Tensor:
    """The logits of an ideal e4m3 version of a ResNet: every conv's input
    (but the stem's) and the last block's output (what the pooled head reads)
    rounded to OCP e4m3 with a per-tensor scale amax / 448 taken on
    `calib_u8` (default: 8 uniform-noise images, as the engine calibrates),
    weights rounded to e4m3 with per-output-channel scales, fp32 arithmetic
    otherwise. The e4m3 engine's accuracy is judged against this floor: e4m3
    keeps 3 mantissa bits, so on a discriminating model even the ideal
    rounding moves the logits by ~20% of their per-image part."""
    import copy

    if calib_u8 is None:
        calib_u8 = noise_images(8, seed=12345, size=images_u8.shape[1])
    ref = copy.deepcopy(model).eval()
    sites = [(n, m) for n, m in ref.named_modules() if isinstance(m, nn.Conv2d) and n != "conv1"]
    amax: dict[str, float] = {}

    def track(name):
        def f(mod, inp):
            amax[name] = max(amax.get(name, 0.0), inp[0].abs().max().item())
        return f
    hs = [m.register_forward_pre_hook(track(n)) for n, m in sites]
    last = ref.layer4
    hs.append(last.register_forward_hook(lambda mod, i, o: amax.__setitem__("out", max(amax.get("out", 0.0),
                                                                                         o.abs().max().item()))))
    ref(normalize(calib_u8))
    for h in hs:
        h.remove()

    def q(t, s):
        return (t / s).clamp(-448, 448).to(torch.float8_e4m3fn).float() * s
    for n, m in sites:
        w = m.weight.data
        m.weight.data = q(w, w.abs().amax((1, 2, 3), keepdim=True).clamp_min(1e-12) / 448)
        s_in = max(amax[n], 1e-6) / 448
        m.register_forward_pre_hook(lambda mod, inp, s=s_in: (q(inp[0], s),))
    s_out = max(amax["out"], 1e-6) / 448
    last.register_forward_hook(lambda mod, i, o: q(o, s_out))
    return torch.cat([ref(normalize(c)) for c in images_u8.split(64)])
