"""Python entry points to the hand-written gfx950 HIP kernels (csrc/kernels).

Every op runs the native kernel on the caller's current HIP stream; there is
no PyTorch fallback. Calling on CPU tensors, or without the built extension,
raises — a GPU test can never pass on a silent eager path.

Layout conventions: activations are bf16 NHWC; conv/linear weights are packed
``[Npad, Kpad]`` bf16 with k = (kh*KW + kw)*Cin + c (see ``pack_conv_weight``).
"""
from __future__ import annotations

import torch

from .. import native


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _need_cuda(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("dmlc.ops kernels need CUDA/HIP tensors (no CPU fallback)")


def _ptr(t):
    return 0 if t is None else t.data_ptr()


def conv_kpad(cin_eff: int, kh: int, kw: int) -> int:
    return native().conv_kpad(cin_eff, kh, kw)


def conv_npad(n: int) -> int:
    return native().conv_npad(n)


def pack_conv_weight(w: torch.Tensor, scale: torch.Tensor | None = None, cin_eff: int | None = None,
                     device=None) -> torch.Tensor:
    """[Cout, Cin, KH, KW] fp32 -> packed bf16 [Npad, Kpad] (per-row scale
    folded in, e.g. a BN scale). ``cin_eff`` = 4 for the 3-channel stem."""
    cout, cin, kh, kw = w.shape
    ce = cin_eff or cin
    kpad, npad = conv_kpad(ce, kh, kw), conv_npad(cout)
    w = w.float()
    if scale is not None:
        w = w * scale.float().view(-1, 1, 1, 1)
    wp = torch.zeros(cout, kh, kw, ce)
    wp[..., :cin] = w.permute(0, 2, 3, 1)
    out = torch.zeros(npad, kpad)
    out[:cout, : kh * kw * ce] = wp.reshape(cout, -1)
    return out.to(torch.bfloat16).to(device) if device is not None else out.to(torch.bfloat16)


def conv2d(x: torch.Tensor, w_packed: torch.Tensor, cout: int, kh: int, kw: int, stride: int = 1,
           pad: int = 0, bias: torch.Tensor | None = None, res: torch.Tensor | None = None,
           relu: bool = False, out_f32: bool = False, split_k: int = 1, tile: int = -1,
           out: torch.Tensor | None = None) -> torch.Tensor:
    """Implicit-GEMM conv on MFMA. x: bf16 NHWC [B,H,W,Cin] (Cin=4 or %64==0).
    Returns [B,Ho,Wo,cout] (bf16, or fp32 if out_f32)."""
    _need_cuda(x, w_packed, bias, res)
    C = native()
    B, H, W, Cin = x.shape
    Ho, Wo = C.conv_out_dim(H, kh, stride, pad), C.conv_out_dim(W, kw, stride, pad)
    if out is None:
        out = torch.empty(B, Ho, Wo, cout, device=x.device, dtype=torch.float32 if out_f32 else torch.bfloat16)
    ws = None
    if split_k > 1:
        ws = torch.empty(split_k * B * Ho * Wo * w_packed.shape[0], device=x.device, dtype=torch.float32)
    if bias is not None:
        bias = bias.float().contiguous()
        if bias.numel() < w_packed.shape[0]:
            bias = torch.nn.functional.pad(bias, (0, w_packed.shape[0] - bias.numel()))
    C.conv2d(x=_ptr(x.contiguous()), w=_ptr(w_packed), bias=_ptr(bias), res=_ptr(res), y=_ptr(out), B=B, H=H,
             W=W, Cin=Cin, KH=kh, KW=kw, stride=stride, pad=pad, N=cout, Npad=w_packed.shape[0],
             Kpad=w_packed.shape[1], ldo=cout, relu=relu, out_f32=out_f32, split_k=split_k, ws=_ptr(ws),
             tile=tile, stream=_stream())
    return out


def maxpool2d(x: torch.Tensor, k: int = 3, stride: int = 2, pad: int = 1) -> torch.Tensor:
    _need_cuda(x)
    C = native()
    B, H, W, Ch = x.shape
    Ho, Wo = C.conv_out_dim(H, k, stride, pad), C.conv_out_dim(W, k, stride, pad)
    y = torch.empty(B, Ho, Wo, Ch, device=x.device, dtype=torch.bfloat16)
    C.maxpool2d(_ptr(x.contiguous()), _ptr(y), B, H, W, Ch, k, stride, pad, _stream())
    return y


def avgpool_global(x: torch.Tensor) -> torch.Tensor:
    _need_cuda(x)
    B, H, W, Ch = x.shape
    y = torch.empty(B, Ch, device=x.device, dtype=torch.bfloat16)
    native().avgpool_global(_ptr(x.contiguous()), _ptr(y), B, H * W, Ch, _stream())
    return y


def avgpool_adaptive(x: torch.Tensor, ho: int, wo: int) -> torch.Tensor:
    _need_cuda(x)
    B, H, W, Ch = x.shape
    y = torch.empty(B, ho, wo, Ch, device=x.device, dtype=torch.bfloat16)
    native().avgpool_adaptive(_ptr(x.contiguous()), _ptr(y), B, H, W, Ch, ho, wo, _stream())
    return y


def preprocess_u8(images: torch.Tensor, size: int = 224) -> torch.Tensor:
    """u8 [B,H,W,3] -> bf16 NHWC4 [B,size,size,4] (resize/crop/normalise)."""
    _need_cuda(images)
    if images.dtype != torch.uint8 or images.dim() != 4 or images.shape[-1] != 3:
        raise ValueError("preprocess_u8 expects uint8 [B,H,W,3]")
    B, H, W, _ = images.shape
    y = torch.empty(B, size, size, 4, device=images.device, dtype=torch.bfloat16)
    native().preprocess_u8(_ptr(images.contiguous()), _ptr(y), B, H, W, size, _stream())
    return y


def softmax_top1(logits: torch.Tensor, n: int | None = None) -> tuple[torch.Tensor, torch.Tensor]:
    _need_cuda(logits)
    if logits.dtype != torch.float32:
        raise ValueError("softmax_top1 expects fp32 logits")
    B, ld = logits.shape
    n = ld if n is None else n
    idx = torch.empty(B, device=logits.device, dtype=torch.int32)
    prob = torch.empty(B, device=logits.device, dtype=torch.float32)
    native().softmax_top1(_ptr(logits.contiguous()), B, n, ld, _ptr(idx), _ptr(prob), _stream())
    return idx, prob
