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


def conv_kpad(cin: int, kh: int, kw: int, pair_stem: bool = False) -> int:
    return native().conv_kpad(cin, kh, kw, pair_stem)


def conv_npad(n: int) -> int:
    return native().conv_npad(n)


_ZERO = {}


def _zero_page(device) -> torch.Tensor:
    z = _ZERO.get(device)
    if z is None:
        z = _ZERO[device] = torch.zeros(64, dtype=torch.float32, device=device)
    return z


def pack_conv_weight(w: torch.Tensor, scale: torch.Tensor | None = None, pair_stem: bool = False,
                     device=None) -> torch.Tensor:
    """[Cout, Cin, KH, KW] fp32 -> packed bf16 [Npad, Kpad] (per-row scale
    folded in, e.g. a BN scale). k = (kh*KW + kw)*Cin + c; for the 3-channel
    stem (``pair_stem``) k = (kh*KWP + kw//2)*8 + (kw%2)*4 + c."""
    cout, cin, kh, kw = w.shape
    kpad, npad = conv_kpad(8 if pair_stem else cin, kh, kw, pair_stem), conv_npad(cout)
    w = w.float()
    if scale is not None:
        w = w * scale.float().view(-1, 1, 1, 1)
    out = torch.zeros(npad, kpad)
    if pair_stem:
        kwp = (kw + 1) // 2
        wp = torch.zeros(cout, kh, kwp * 2, 4)
        wp[:, :, :kw, :cin] = w.permute(0, 2, 3, 1)
        out[:cout, : kh * kwp * 8] = wp.reshape(cout, -1)
    else:
        out[:cout, : kh * kw * cin] = w.permute(0, 2, 3, 1).reshape(cout, -1)
    return out.to(torch.bfloat16).to(device) if device is not None else out.to(torch.bfloat16)


def pair_image(x_nhwc3: torch.Tensor, pad: int) -> torch.Tensor:
    """Reference construction of the stem's pair image from an NHWC RGB
    tensor: [B, H+2p, W+2p, 8], position (h,w) = RGB0 of pixels (h-p, w-p)
    and (h-p, w-p+1), zeros outside the image."""
    B, H, W, _ = x_nhwc3.shape
    px = torch.zeros(B, H + 2 * pad, W + 2 * pad + 1, 4, dtype=x_nhwc3.dtype, device=x_nhwc3.device)
    px[:, pad:pad + H, pad:pad + W, :3] = x_nhwc3
    return torch.cat([px[:, :, :-1], px[:, :, 1:]], dim=-1).contiguous()


def conv2d(x: torch.Tensor, w_packed: torch.Tensor, cout: int, kh: int, kw: int, stride: int = 1,
           pad: int = 0, bias: torch.Tensor | None = None, res: torch.Tensor | None = None,
           relu: bool = False, out_f32: bool = False, split_k: int = 1, tile: int = -1,
           out: torch.Tensor | None = None, pair_stem: bool = False) -> torch.Tensor:
    """Implicit-GEMM conv on MFMA. x: bf16 NHWC [B,H,W,Cin] (Cin % 64 == 0),
    or with ``pair_stem`` the padded pair image (``pair_image``; pad ignored).
    Returns [B,Ho,Wo,cout] (bf16, or fp32 if out_f32)."""
    _need_cuda(x, w_packed, bias, res)
    C = native()
    B, H, W, Cin = x.shape
    if pair_stem:
        pad = 0
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
             tile=tile, zero=_ptr(_zero_page(x.device)), pair_stem=pair_stem, stream=_stream())
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


def preprocess_u8(images: torch.Tensor, size: int = 224, pad: int = 0) -> torch.Tensor:
    """u8 [B,H,W,3] -> bf16 pair image [B,size+2p,size+2p,8] (resize, crop,
    normalise; see ``pair_image``)."""
    _need_cuda(images)
    if images.dtype != torch.uint8 or images.dim() != 4 or images.shape[-1] != 3:
        raise ValueError("preprocess_u8 expects uint8 [B,H,W,3]")
    B, H, W, _ = images.shape
    P = size + 2 * pad
    y = torch.empty(B, P, P, 8, device=images.device, dtype=torch.bfloat16)
    native().preprocess_u8(_ptr(images.contiguous()), _ptr(y), B, H, W, size, pad, _stream())
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
