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


def conv_kpad(cin: int, kh: int, kw: int, stem: bool = False) -> int:
    return native().conv_kpad(cin, kh, kw, stem)


def stem_row_width(size: int, pad: int, kw: int, stride: int) -> int:
    return native().stem_row_width(size, pad, kw, stride)


def conv_npad(n: int) -> int:
    return native().conv_npad(n)


_ZERO = {}


def _zero_page(device) -> torch.Tensor:
    z = _ZERO.get(device)
    if z is None:
        z = _ZERO[device] = torch.zeros(64, dtype=torch.float32, device=device)
    return z


def pack_conv_weight(w: torch.Tensor, scale: torch.Tensor | None = None, stem: bool = False,
                     device=None) -> torch.Tensor:
    """[Cout, Cin, KH, KW] fp32 -> packed bf16 [Npad, Kpad] (per-row scale
    folded in, e.g. a BN scale). k = (kh*KW + kw)*Cin + c; for the 3-channel
    stem k = kh*CPK*8 + kw*3 + c with CPK = ceil(3*KW/8)."""
    cout, cin, kh, kw = w.shape
    kpad, npad = conv_kpad(cin, kh, kw, stem), conv_npad(cout)
    w = w.float()
    if scale is not None:
        w = w * scale.float().view(-1, 1, 1, 1)
    out = torch.zeros(npad, kpad)
    if stem:
        cpk = (kw * 3 + 7) // 8
        wp = torch.zeros(cout, kh, cpk * 8)
        wp[:, :, : kw * 3] = w.permute(0, 2, 3, 1).reshape(cout, kh, kw * 3)
        out[:cout, : kh * cpk * 8] = wp.reshape(cout, -1)
    else:
        out[:cout, : kh * kw * cin] = w.permute(0, 2, 3, 1).reshape(cout, -1)
    return out.to(torch.bfloat16).to(device) if device is not None else out.to(torch.bfloat16)


def stem_image(x_nhwc3: torch.Tensor, pad: int, row_width: int) -> torch.Tensor:
    """Reference construction of the stem's input: [B, H+2p, row_width, 3]
    with the image at (p, p) and zeros elsewhere."""
    B, H, W, _ = x_nhwc3.shape
    out = torch.zeros(B, H + 2 * pad, row_width, 3, dtype=x_nhwc3.dtype, device=x_nhwc3.device)
    out[:, pad:pad + H, pad:pad + W] = x_nhwc3
    return out.contiguous()


def fc(x: torch.Tensor, w_packed: torch.Tensor, cout: int, bias: torch.Tensor | None = None, relu: bool = False,
       out_f32: bool = False, splits: int = 0) -> torch.Tensor:
    """Fully connected layer at M <= 256 rows on fc_gemm.hip: x bf16 [M, K]
    (K = w_packed.shape[1], a multiple of 64), w_packed [Npad, K] (Npad % 128
    == 0) -> [M, cout] bf16 (fp32 with out_f32). splits: K slices (0: the
    engine's choice), fp32 partials reduced with the bias and ReLU."""
    _need_cuda(x, w_packed, bias)
    C = native()
    M, K = x.shape
    if K != w_packed.shape[1]:
        raise ValueError("fc: x's K must equal the packed weight's K")
    if splits <= 0:
        splits = C.fc_gemm_splits(M, K, w_packed.shape[0], torch.cuda.get_device_properties(x.device).multi_processor_count)
    ws = torch.empty(splits * M * w_packed.shape[0], device=x.device, dtype=torch.float32)
    return conv2d(x.contiguous().view(M, 1, 1, K), w_packed, cout, 1, 1, bias=bias, relu=relu, out_f32=out_f32,
                  split_k=splits, tile=C.CONV_FC, ws=ws).view(M, cout)


def conv2d(x: torch.Tensor, w_packed: torch.Tensor, cout: int, kh: int, kw: int, stride: int = 1,
           pad: int = 0, bias: torch.Tensor | None = None, res: torch.Tensor | None = None,
           relu: bool = False, out_f32: bool = False, split_k: int = 1, tile: int = -1,
           out: torch.Tensor | None = None, stem: bool = False, out_hw: tuple | None = None,
           max_blocks: int = 0, ws: torch.Tensor | None = None) -> torch.Tensor:
    """Implicit-GEMM conv on MFMA. x: bf16 NHWC [B,H,W,Cin] (Cin % 64 == 0),
    or with ``stem`` the padded packed RGB image (``stem_image``) plus the
    output size ``out_hw`` (the padding is already in the image).
    Returns [B,Ho,Wo,cout] (bf16, or fp32 if out_f32)."""
    _need_cuda(x, w_packed, bias, res)
    C = native()
    B, H, W, Cin = x.shape
    if stem:
        Ho, Wo = out_hw
    else:
        Ho, Wo = C.conv_out_dim(H, kh, stride, pad), C.conv_out_dim(W, kw, stride, pad)
    if out is None:
        out = torch.empty(B, Ho, Wo, cout, device=x.device, dtype=torch.float32 if out_f32 else torch.bfloat16)
    if bias is not None:
        bias = bias.float().contiguous()
        if bias.numel() < w_packed.shape[0]:
            bias = torch.nn.functional.pad(bias, (0, w_packed.shape[0] - bias.numel()))
    bt_ws, bt_bytes, bt_splits = None, 0, 1
    if C.CONV_BIGTILE0 <= tile < C.CONV_BIGTILE0 + 2:  # 8-wave big-tile kernel (conv_bigtile.hip); split_k = K slices (0: engine's choice)
        bt_splits = split_k if split_k > 0 else C.conv_bigtile_splits(
            B, Ho, Wo, w_packed.shape[0], w_packed.shape[1], tile - C.CONV_BIGTILE0,
            torch.cuda.get_device_properties(x.device).multi_processor_count)
        split_k = 1
        bm, bn = 256, (256 if tile == C.CONV_BIGTILE0 else 128)
        slabs = -(-B * Ho * Wo // bm) * (w_packed.shape[0] // bn) * (bt_splits - 1)
        bt_ws = _bigtile_ws(x.device, C.conv_bigtile_ws_bytes(slabs))
        bt_bytes = bt_ws.numel()
    if ws is None and split_k > 1:
        ws = torch.empty(split_k * B * Ho * Wo * w_packed.shape[0], device=x.device, dtype=torch.float32)
    C.conv2d(x=_ptr(x.contiguous()), w=_ptr(w_packed), bias=_ptr(bias), res=_ptr(res), y=_ptr(out), B=B, H=H,
             W=W, Cin=Cin, KH=kh, KW=kw, stride=stride, pad=pad, N=cout, Npad=w_packed.shape[0],
             Kpad=w_packed.shape[1], ldo=cout, relu=relu, out_f32=out_f32, split_k=split_k, ws=_ptr(ws),
             tile=tile, zero=_ptr(_zero_page(x.device)), stem=stem, Ho=Ho, Wo=Wo, max_blocks=max_blocks,
             stream=_stream(), bt_ws=_ptr(bt_ws), bt_ws_bytes=bt_bytes, bt_splits=bt_splits)
    return out


_BT_WS: dict = {}
BT_STAMPS = None
_PHASE_STAMPS = False


def set_phase_stamps(on: bool) -> None:
    """Record per-workgroup phase stamps (start / prologue / loop / epilogue,
    100 MHz) of every following conv3x3_stream launch into BT_STAMPS (a
    measurement hook for tools/conv_bench.py; off by default)."""
    global _PHASE_STAMPS
    _PHASE_STAMPS = bool(on)


def _bigtile_ws(device: torch.device, nbytes: int) -> torch.Tensor:
    """Per-device big-tile split-K workspace (hand-off flags zeroed once, then
    fp32 slabs); grown on demand."""
    C = native()
    t = _BT_WS.get(device.index)
    if t is None or t.numel() < nbytes:
        if t is not None:
            torch.cuda.synchronize(device)
        t = torch.empty(max(nbytes, C.conv_bigtile_ws_bytes(0)), dtype=torch.uint8, device=device)
        t[:C.conv_bigtile_ws_header_bytes()].zero_()
        _BT_WS[device.index] = t
    return t


def bigtile_error(device: torch.device) -> bool:
    """True if a big-tile split-K hand-off timed out on `device` (results invalid)."""
    C = native()
    t = _BT_WS.get(device.index)
    if t is None:
        return False
    hdr = C.conv_bigtile_ws_header_bytes()
    return int(t[hdr - 256:hdr - 252].view(torch.int32).item()) != 0


def conv3x3_rows(x: torch.Tensor, w_packed: torch.Tensor, bias: torch.Tensor, res: torch.Tensor | None = None,
                 relu: bool = True, strip: int | None = None, frag: bool = False) -> torch.Tensor:
    """Direct 3x3/s1/p1 conv (conv3x3_rows.hip) on NHWC bf16 [B,56,56,64] with
    the conv2d packed weights [64, 576]; + bias (+ residual), ReLU. frag: the
    register-weight variant (weights in fragment order, 2 workgroups per CU)."""
    _need_cuda(x, w_packed, bias, res)
    C = native()
    B, H, W, Cin = x.shape
    if not C.conv3x3_rows_supported(H, W, Cin, w_packed.shape[0]):
        raise ValueError("conv3x3_rows: unsupported shape")
    if strip is None:
        cus = torch.cuda.get_device_properties(x.device).multi_processor_count
        strip = C.conv3x3_rows_pick_strip(B, H, 2 * cus if frag else cus)
    y = torch.empty_like(x)
    wf = stream_weight_frag(w_packed) if frag else None
    C.conv3x3_rows(_ptr(x.contiguous()), _ptr(w_packed.contiguous()), _ptr(bias.float().contiguous()),
                   _ptr(None if res is None else res.contiguous()), _ptr(y), _ptr(_zero_page(x.device)), B, H, W,
                   Cin, relu, strip, _stream(), _ptr(wf))
    return y


def conv3x3_block(x: torch.Tensor, w1_packed: torch.Tensor, b1: torch.Tensor, w2_packed: torch.Tensor,
                  b2: torch.Tensor) -> torch.Tensor:
    """A whole 56x56x64 basic block (conv3x3_block.hip) on NHWC bf16:
    relu(conv2(relu(conv1(x) + b1)) + b2 + x), the intermediate kept in LDS
    (rounded to bf16 like a stored activation). w*_packed: conv2d packed
    weights [64, 576]."""
    _need_cuda(x, w1_packed, b1, w2_packed, b2)
    C = native()
    B, H, W, Cin = x.shape
    if not C.conv3x3_block_supported(H, W, Cin) or w1_packed.shape[0] != Cin or w2_packed.shape[0] != Cin:
        raise ValueError("conv3x3_block: unsupported shape")
    x = x.contiguous()
    y = torch.empty_like(x)
    wf1, wf2 = stream_weight_frag(w1_packed), stream_weight_frag(w2_packed)
    C.conv3x3_block(_ptr(x), _ptr(wf1), _ptr(b1.float().contiguous()), _ptr(wf2), _ptr(b2.float().contiguous()),
                    _ptr(y), _ptr(_zero_page(x.device)), B, _stream())
    return y


def conv3x3_s2rows(x: torch.Tensor, w_packed: torch.Tensor, bias: torch.Tensor, wd_packed: torch.Tensor,
                   bd: torch.Tensor, relu: bool = True):
    """ResNet layer2.0's stride-2 3x3 conv [B,56,56,64] -> [B,28,28,128]
    and its 1x1/s2 downsample in one row-streaming kernel
    (conv3x3_s2rows.hip): returns (relu?(conv3x3(x) + bias), conv1x1_s2(x)
    + bd). w_packed: conv2d packed weights [128, 576]; wd_packed [128, 64]."""
    _need_cuda(x, w_packed, bias, wd_packed, bd)
    C = native()
    B, H, W, Cin = x.shape
    Cout = w_packed.shape[0]
    if (not C.conv3x3_s2rows_supported(H, W, Cin, Cout) or tuple(w_packed.shape) != (Cout, 9 * Cin)
            or tuple(wd_packed.shape) != (Cout, Cin)):
        raise ValueError("conv3x3_s2rows: unsupported shape")
    x = x.contiguous()
    y = torch.empty(B, H // 2, W // 2, Cout, dtype=x.dtype, device=x.device)
    yd = torch.empty_like(y)
    wf, wdf = stream_weight_frag(w_packed), stream_weight_frag(wd_packed)
    C.conv3x3_s2rows(_ptr(x), _ptr(wf), _ptr(bias.float().contiguous()), _ptr(wdf), _ptr(bd.float().contiguous()),
                     _ptr(y), _ptr(yd), _ptr(_zero_page(x.device)), B, relu, _stream())
    return y, yd


def conv3x3_s2rows128(x: torch.Tensor, w_packed: torch.Tensor, bias: torch.Tensor, relu: bool = True,
                      out_inv_scale: float = 0.0):
    """ResNet50 layer2.0.conv2, [B,56,56,128] -> [B,28,28,128] stride 2, one
    row-streaming weight-stationary workgroup per image
    (conv3x3_s2rows128.hip). Returns bf16, or e4m3 bytes (uint8) of
    relu?(conv + bias) * out_inv_scale when out_inv_scale > 0."""
    _need_cuda(x, w_packed, bias)
    C = native()
    B, H, W, Cin = x.shape
    Cout = w_packed.shape[0]
    if not C.conv3x3_s2rows128_supported(H, W, Cin, Cout) or tuple(w_packed.shape) != (Cout, 9 * Cin):
        raise ValueError("conv3x3_s2rows128: unsupported shape")
    x = x.contiguous()
    dt = torch.uint8 if out_inv_scale > 0 else x.dtype
    y = torch.empty(B, H // 2, W // 2, Cout, dtype=dt, device=x.device)
    wf = stream_weight_frag(w_packed)
    C.conv3x3_s2rows128(_ptr(x), _ptr(wf), _ptr(bias.float().contiguous()), _ptr(y), B, relu, float(out_inv_scale),
                        _stream())
    return y


def conv_small(x: torch.Tensor, w_packed: torch.Tensor, bias: torch.Tensor, res: torch.Tensor | None = None,
               relu: bool = True, stride: int = 1, wd_packed: torch.Tensor | None = None,
               bd: torch.Tensor | None = None, mf: int | None = None):
    """Query-batch 3x3/p1 conv (conv_small.hip) on NHWC bf16 [B,H,W,CI]:
    relu?(conv3x3(x) + bias (+ res)). w_packed: conv2d packed weights
    [Cout, 9 CI]. With stride 2 and wd_packed [Cout, CI] / bd also returns the
    1x1/s2 downsample conv1x1_s2(x) + bd: (y, yd)."""
    _need_cuda(x, w_packed, bias, res, wd_packed, bd)
    C = native()
    B, H, W, Cin = x.shape
    Cout = w_packed.shape[0]
    if not C.conv_small_supported(H, W, Cin, Cout, stride) or tuple(w_packed.shape) != (Cout, 9 * Cin):
        raise ValueError("conv_small: unsupported shape")
    Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
    if res is not None and tuple(res.shape) != (B, Ho, Wo, Cout):
        raise ValueError("conv_small: residual shape")
    if wd_packed is not None and (stride != 2 or bd is None or tuple(wd_packed.shape) != (Cout, Cin)):
        raise ValueError("conv_small: downsample needs stride 2, bd and [Cout, Cin] weights")
    if mf is None:
        cus = torch.cuda.get_device_properties(x.device).multi_processor_count
        mf = C.conv_small_pick_mf(B, H, W, Cin, Cout, stride, cus)
    x = x.contiguous()
    y = torch.empty(B, Ho, Wo, Cout, dtype=x.dtype, device=x.device)
    yd = torch.empty_like(y) if wd_packed is not None else None
    wdf = stream_weight_frag(wd_packed) if wd_packed is not None else None
    C.conv_small(_ptr(x), _ptr(stream_weight_frag(w_packed)), _ptr(bias.float().contiguous()),
                 _ptr(None if res is None else res.contiguous()), _ptr(y), B, H, W, Cin, Cout, stride, relu, mf,
                 _stream(), _ptr(wdf), _ptr(None if bd is None else bd.float().contiguous()), _ptr(yd))
    return (y, yd) if wd_packed is not None else y


def conv3x3_rows28(x: torch.Tensor, w_packed: torch.Tensor, bias: torch.Tensor, res: torch.Tensor | None = None,
                   relu: bool = True) -> torch.Tensor:
    """Weight-stationary row-streaming 3x3/s1/p1 conv on [B,28,28,128] ->
    128 channels (conv3x3_rows28.hip): relu?(conv(x) + bias (+ res)).
    w_packed: conv2d packed weights [128, 1152]."""
    _need_cuda(x, w_packed, bias, res)
    C = native()
    B, H, W, Cin = x.shape
    Cout = w_packed.shape[0]
    if not C.conv3x3_rows28_supported(H, W, Cin, Cout) or tuple(w_packed.shape) != (Cout, 9 * Cin):
        raise ValueError("conv3x3_rows28: unsupported shape")
    if res is not None and tuple(res.shape) != (B, H, W, Cout):
        raise ValueError("conv3x3_rows28: residual shape")
    x = x.contiguous()
    y = torch.empty_like(x)
    C.conv3x3_rows28(_ptr(x), _ptr(stream_weight_frag(w_packed)), _ptr(bias.float().contiguous()),
                     _ptr(None if res is None else res.contiguous()), _ptr(y), B, relu, _stream())
    return y


def stream_weight_frag(w_packed: torch.Tensor, cout: int | None = None) -> torch.Tensor:
    """Packed conv weights [Npad, K] -> the stream conv's fragment order
    [Cout/32][K/32][2][64 lanes][8]: lane l of fragment nf of channel group g,
    K-tile t holds channel 32g + perm32(16nf + (l & 15)), k = 32t + 8(l >> 4)
    + e, perm32(n) = 8((n & 15) >> 2) + 4(n >> 4) + (n & 3)."""
    cout = w_packed.shape[0] if cout is None else cout
    K = w_packed.shape[1]
    n = torch.arange(32)
    perm = 8 * ((n & 15) >> 2) + 4 * (n >> 4) + (n & 3)            # tile row -> channel
    lane = torch.arange(64)
    rows = perm[(torch.arange(2).view(2, 1) * 16 + (lane & 15).view(1, 64))]  # [nf, lane] -> channel in group
    w = w_packed[:cout].view(cout // 32, 32, K // 32, 4, 8)          # [g, ch, t, kq, e]
    kq = (lane >> 4).view(1, 64).expand(2, 64)
    # advanced indices separated by a slice go first: [nf, lane, g, t, e]
    out = w[:, rows.to(w.device), :, kq.to(w.device), :]
    return out.permute(2, 3, 0, 1, 4).contiguous()


def conv3x3_stream(x: torch.Tensor, w_packed: torch.Tensor, bias: torch.Tensor, res: torch.Tensor | None = None,
                   relu: bool = True, stride: int = 1, downsample: tuple | None = None,
                   frag: bool | torch.Tensor = False):
    """Direct 3x3/p1 conv (conv3x3_stream.hip) on NHWC bf16 with the conv2d
    packed weights; + bias (+ residual), ReLU. Stride 1: [B,28,28,128],
    [B,14,14,256], [B,7,7,512]; stride 2: [B,56,56,64] -> 128 channels,
    [B,28,28,128] -> 256, [B,14,14,256] -> 512.

    downsample=(wd_packed [Cout, Cin], bd[, wd_frag]): stride 2 only; also
    computes the 1x1/s2 conv + bias from the same resident input and returns
    (y, yd); wd_frag = stream_weight_frag(wd_packed), precomputed for graph
    capture."""
    _need_cuda(x, w_packed, bias, res)
    C = native()
    B, H, W, Cin = x.shape
    Cout = w_packed.shape[0]
    if not C.conv3x3_stream_supported(H, W, Cin, Cout, stride):
        raise ValueError("conv3x3_stream: unsupported shape")
    y = torch.empty(B, H // stride, W // stride, Cout, dtype=x.dtype, device=x.device)
    stamps = 0
    if _PHASE_STAMPS:  # per-workgroup phase stamps of the stream conv (tools/conv_bench.py --stamps)
        global BT_STAMPS
        if BT_STAMPS is None:
            BT_STAMPS = torch.zeros(1 << 16, dtype=torch.int64, device=x.device)
        stamps = _ptr(BT_STAMPS)
    yd = wd = bd = None
    if downsample is not None:
        wd, bd = downsample[0].contiguous(), downsample[1].float().contiguous()
        _need_cuda(wd, bd)
        if stride != 2 or tuple(wd.shape) != (Cout, Cin):
            raise ValueError("conv3x3_stream: downsample needs stride 2 and weights [Cout, Cin]")
        yd = torch.empty_like(y)
    wf = None
    if frag is not False and frag is not None:  # True, or the fragment-order weights (graph capture)
        if not C.conv3x3_stream_uses_frag(H, W, Cin, Cout, stride):
            raise ValueError("conv3x3_stream: no register-weight variant for this shape")
        wf = frag if isinstance(frag, torch.Tensor) else stream_weight_frag(w_packed)
    wdf = None
    if wf is not None and wd is not None:
        wdf = downsample[2] if len(downsample) > 2 else stream_weight_frag(wd)
    C.conv3x3_stream(_ptr(x.contiguous()), _ptr(w_packed.contiguous()), _ptr(bias.float().contiguous()),
                     _ptr(None if res is None else res.contiguous()), _ptr(y), _ptr(_zero_page(x.device)), B, H, W,
                     Cin, Cout, stride, relu, _stream(), stamps, _ptr(wd), _ptr(bd), _ptr(yd), _ptr(wf), _ptr(wdf))
    return y if downsample is None else (y, yd)


FP8 = torch.float8_e4m3fn  # OCP e4m3 (gfx950), max 448
FP8_MAX = 448.0


def quantize_fp8(t: torch.Tensor, scale: float) -> torch.Tensor:
    """e4m3(t / scale), saturating."""
    return (t.float() / scale).clamp(-FP8_MAX, FP8_MAX).to(FP8)


def pack_conv_weight_fp8(w: torch.Tensor, device=None) -> tuple[torch.Tensor, torch.Tensor]:
    """[Cout, Cin, KH, KW] -> (e4m3 [Npad, Kpad] with a per-output-channel
    scale, fp32 scales [Npad]); k = (kh*KW + kw)*Cin + c as for bf16."""
    cout, cin, kh, kw = w.shape
    kpad, npad = conv_kpad(cin, kh, kw), conv_npad(cout)
    wk = torch.zeros(npad, kpad)
    wk[:cout, : kh * kw * cin] = w.float().permute(0, 2, 3, 1).reshape(cout, -1)
    s = (wk.abs().amax(1) / FP8_MAX).clamp_min(1e-12)
    q = quantize_fp8(wk / s[:, None], 1.0)
    return (q.to(device), s.to(device)) if device is not None else (q, s)


def conv2d_fp8(x: torch.Tensor, w_q: torch.Tensor, alpha: torch.Tensor, cout: int, kh: int, kw: int,
               stride: int = 1, pad: int = 0, bias: torch.Tensor | None = None, res: torch.Tensor | None = None,
               res_scale: float = 1.0, relu: bool = False, out_scale: float | None = None,
               tile: int = -1) -> torch.Tensor:
    """fp8 implicit-GEMM conv (block-scaled e4m3 MFMA). x: e4m3 NHWC
    (Cin % 128 == 0) or bf16 (then w_q is bf16-packed and alpha unused).
    alpha = s_x * s_w[n]; residual e4m3 scaled by res_scale; output e4m3
    with scale out_scale (or bf16 when out_scale is None)."""
    _need_cuda(x, w_q, alpha, bias, res)
    C = native()
    B, H, W, Cin = x.shape
    in8 = x.dtype == FP8
    Ho, Wo = C.conv_out_dim(H, kh, stride, pad), C.conv_out_dim(W, kw, stride, pad)
    out8 = out_scale is not None
    y = torch.empty(B, Ho, Wo, cout, device=x.device, dtype=FP8 if out8 else torch.bfloat16)
    if bias is not None:
        bias = bias.float().contiguous()
        if bias.numel() < w_q.shape[0]:
            bias = torch.nn.functional.pad(bias, (0, w_q.shape[0] - bias.numel()))
    al = alpha.float().contiguous() if alpha is not None else None
    C.conv2d(x=_ptr(x.contiguous()), w=_ptr(w_q), bias=_ptr(bias), res=_ptr(res), y=_ptr(y), B=B, H=H, W=W, Cin=Cin,
             KH=kh, KW=kw, stride=stride, pad=pad, N=cout, Npad=w_q.shape[0], Kpad=w_q.shape[1], ldo=cout,
             relu=relu, out_f32=False, split_k=1, ws=0, tile=tile, zero=_ptr(_zero_page(x.device)), stem=False,
             Ho=Ho, Wo=Wo, max_blocks=0, stream=_stream(), in_fp8=in8, out_fp8=out8, alpha=_ptr(al),
             res_scale=res_scale, out_inv_scale=(1.0 / out_scale) if out8 else 1.0)
    return y


def stream8_weight_frag(w_q: torch.Tensor, cout: int) -> torch.Tensor:
    """e4m3 packed conv weights [Npad, K] (pack_conv_weight_fp8) -> the e4m3
    3x3 conv's fragment order (conv3x3_stream8.hip): [Cout/32][K/128][2 nf][2
    h][64 lanes][16 B], lane l of (group g, K-tile t, nf, h) holding
    W[32g + perm32(16nf + (l & 15))][128t + 32fq + 16(h ^ (fq & 1)) + 0..15],
    fq = l >> 4 (the odd-fq half swap matches the kernel's X reads)."""
    w = w_q[:cout].view(torch.uint8)
    K = w.shape[1]
    n = torch.arange(32)
    perm = 8 * ((n & 15) >> 2) + 4 * (n >> 4) + (n & 3)
    lane = torch.arange(64)
    fq = lane >> 4
    G, T = cout // 32, K // 128
    g = torch.arange(G).view(G, 1, 1, 1, 1, 1)
    t = torch.arange(T).view(1, T, 1, 1, 1, 1)
    nf = torch.arange(2).view(1, 1, 2, 1, 1, 1)
    h = torch.arange(2).view(1, 1, 1, 2, 1, 1)
    ln = lane.view(1, 1, 1, 1, 64, 1)
    e = torch.arange(16).view(1, 1, 1, 1, 1, 16)
    row = 32 * g + perm[16 * nf + (ln & 15)]
    col = 128 * t + 32 * (ln >> 4) + 16 * (h ^ ((ln >> 4) & 1)) + e
    del fq
    row, col = torch.broadcast_tensors(row, col)
    return w[row.to(w.device), col.to(w.device)].contiguous()


def conv3x3_stream8(x: torch.Tensor, w_q: torch.Tensor, alpha: torch.Tensor, bias: torch.Tensor, relu: bool = True,
                    out_scale: float = 1.0, frag: torch.Tensor | None = None, stride: int = 1) -> torch.Tensor:
    """e4m3 3x3/p1 conv (conv3x3_stream8.hip) on e4m3 NHWC: stride 1 on
    [B,14,14,256] / [B,7,7,512], stride 2 on [B,28,28,256] / [B,14,14,512]:
    e4m3(relu?(acc * alpha + bias) / out_scale) with acc = conv of the e4m3
    values. w_q / alpha: pack_conv_weight_fp8 (alpha = s_x * s_w)."""
    _need_cuda(x, w_q, alpha, bias)
    C = native()
    B, H, W, Cin = x.shape
    cout = Cin
    if x.dtype != FP8 or not C.conv3x3_stream8_supported(H, W, Cin, cout, stride) or w_q.shape[1] != 9 * Cin:
        raise ValueError("conv3x3_stream8: unsupported shape / dtype")
    wf = stream8_weight_frag(w_q, cout) if frag is None else frag
    y = torch.empty(B, H // stride, W // stride, cout, dtype=FP8, device=x.device)
    C.conv3x3_stream8(_ptr(x.contiguous()), _ptr(wf), _ptr(alpha.float().contiguous()), _ptr(bias.float().contiguous()),
                      _ptr(y), _ptr(_zero_page(x.device)), B, H, W, Cin, cout, stride, relu, 1.0 / out_scale,
                      _stream())
    return y


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


def preprocess_u8(images: torch.Tensor, size: int = 224, pad: int = 0, row_width: int | None = None,
                  paired: bool = False) -> torch.Tensor:
    """u8 [B,H,W,3] -> bf16 packed RGB [B, size+2p, row_width, 3] (resize,
    crop, normalise; zero border; see ``stem_image``). With ``paired`` the
    result is [B, size+2p, row_width/2, 8]: pixel pairs as [r g b r g b 0 0]
    (``paired_image``), the fused stem's input."""
    _need_cuda(images)
    if images.dtype != torch.uint8 or images.dim() != 4 or images.shape[-1] != 3:
        raise ValueError("preprocess_u8 expects uint8 [B,H,W,3]")
    B, H, W, _ = images.shape
    P = size + 2 * pad
    Wr = row_width or (P + 7) // 8 * 8
    shape = (B, P, Wr // 2, 8) if paired else (B, P, Wr, 3)
    y = torch.empty(*shape, device=images.device, dtype=torch.bfloat16)
    native().preprocess_u8(_ptr(images.contiguous()), _ptr(y), B, H, W, size, pad, Wr, _stream(), paired)
    return y


def paired_image(x_nhwc3: torch.Tensor, pad: int = 3, pairs: int | None = None) -> torch.Tensor:
    """Reference construction of the fused stem's input: the zero-padded
    image [B, H+2p, 2*pairs, 3] regrouped as [B, H+2p, pairs, 8] with
    chunk = [r g b r g b 0 0] of pixels (2q, 2q+1)."""
    B, H, W, _ = x_nhwc3.shape
    pairs = pairs or ((W + 2 * pad + 7) // 8 * 4)
    img = stem_image(x_nhwc3, pad, 2 * pairs)
    out = torch.zeros(B, H + 2 * pad, pairs, 8, dtype=x_nhwc3.dtype, device=x_nhwc3.device)
    out[..., :6] = img.reshape(B, H + 2 * pad, pairs, 6)
    return out


def pack_stem_pool_weight(w: torch.Tensor, scale: torch.Tensor | None = None, device=None) -> torch.Tensor:
    """[64, 3, 7, 7] fp32 -> bf16 [64, 224] for ``stem_conv_pool``:
    k = kh*32 + q*8 + e with kw = 2q + e//3, c = e%3 (e < 6, kw < 7)."""
    cout, cin, kh, kw = w.shape
    if (cout, cin, kh, kw) != (64, 3, 7, 7):
        raise ValueError("stem_conv_pool packs a [64, 3, 7, 7] weight")
    w = w.float()
    if scale is not None:
        w = w * scale.float().view(-1, 1, 1, 1)
    wk = torch.zeros(64, 7, 8, 3)  # [n, kh, kw (8 slots), c]
    wk[:, :, :7] = w.permute(0, 2, 3, 1)
    out = torch.zeros(64, 7, 4, 8)
    out[..., :6] = wk.reshape(64, 7, 4, 6)
    out = out.reshape(64, 224).to(torch.bfloat16)
    return out.to(device) if device is not None else out


def stem_dense_cell(j: int, fq: int) -> tuple[int, int, bool]:
    """(kernel row dy, window dword u, zero-weight pad) that lane group fq
    reads in dword slot j of the dense-K stem: kernels.h stem_dense_cell."""
    if j < 15:
        return 2 * (j // 5) + (fq & 1), 2 * (j % 5) + (fq >> 1), False
    hp, m = 2 * (j - 15) + (fq >> 1), fq & 1
    if hp < 3:
        return 2 * hp + m, 10, False
    if hp < 6:
        return (5 if m else 6), hp - 3, m == 1
    return 6, 3 + 2 * (hp - 6) + m, False


def pack_stem_dense_weight(w: torch.Tensor, scale: torch.Tensor | None = None, device=None) -> torch.Tensor:
    """[64, 3, 7, 7] fp32 -> bf16 [64, 160] in the dense-K order of the
    one-image-per-workgroup stem (stem_pool.hip V & 2): K index k = 32 s +
    8 fq + 2 i + h holds element 2 u + h of kernel row dy's 22-element window
    (kw-major rgb + 1 zero slot), (dy, u) = stem_dense_cell(4 s + i, fq);
    pad slots and element 21 are zero."""
    cout, cin, kh, kw = w.shape
    if (cout, cin, kh, kw) != (64, 3, 7, 7):
        raise ValueError("stem_conv_pool packs a [64, 3, 7, 7] weight")
    w = w.float()
    if scale is not None:
        w = w * scale.float().view(-1, 1, 1, 1)
    win = torch.zeros(64, 7, 22)
    win[:, :, :21] = w.permute(0, 2, 3, 1).reshape(64, 7, 21)  # [n, kh, kw*3 + c]
    out = torch.zeros(64, 160)
    for k in range(160):
        s, fq, i, h = k // 32, (k % 32) // 8, (k % 8) // 2, k % 2
        dy, u, pad = stem_dense_cell(4 * s + i, fq)
        if not pad:
            out[:, k] = win[:, dy, 2 * u + h]
    out = out.to(torch.bfloat16)
    return out.to(device) if device is not None else out


def stem_conv_pool(x_paired: torch.Tensor, w_packed: torch.Tensor, bias: torch.Tensor, size: int = 224,
                   strip: int | None = None) -> torch.Tensor:
    """Fused conv7x7/s2 + bias + ReLU + maxpool3x3/s2/p1 on the paired image
    (``preprocess_u8(..., pad=3, paired=True)``). Returns [B, size/4, size/4, 64]."""
    _need_cuda(x_paired, w_packed, bias)
    C = native()
    B, P, Wq, eight = x_paired.shape
    if eight != 8 or P != size + 6:
        raise ValueError("stem_conv_pool expects a paired [B, size+6, Wq, 8] image")
    ph = size // 4
    if strip is None:
        strip = C.stem_pool_pick_strip(B, ph, torch.cuda.get_device_properties(x_paired.device).multi_processor_count)
    y = torch.empty(B, ph, ph, 64, device=x_paired.device, dtype=torch.bfloat16)
    C.stem_conv_pool(_ptr(x_paired.contiguous()), _ptr(w_packed.contiguous()), _ptr(bias.float().contiguous()),
                     _ptr(y), B, size, Wq, strip, _stream())
    return y


def stem_conv_pool_u8(images: torch.Tensor, w_packed: torch.Tensor, bias: torch.Tensor,
                      strip: int | None = None, w_dense: torch.Tensor | None = None) -> torch.Tensor:
    """The fused stem with the preprocess fused too: u8 [B, S, S, 3] images
    (already at the model size) -> [B, S/4, S/4, 64]. Same values as
    ``stem_conv_pool(preprocess_u8(images, S, 3, paired=True), ...)`` (up to
    fp32 summation order with ``w_dense``: pack_stem_dense_weight of the same
    weights, which the one-image-per-workgroup kernel then uses)."""
    _need_cuda(images, w_packed, bias)
    if images.dtype != torch.uint8 or images.dim() != 4 or images.shape[-1] != 3 or images.shape[1] != images.shape[2]:
        raise ValueError("stem_conv_pool_u8 expects uint8 [B, S, S, 3]")
    C = native()
    B, S = images.shape[0], images.shape[1]
    ph = S // 4
    if strip is None:
        strip = C.stem_pool_u8_pick_strip(B, ph, torch.cuda.get_device_properties(images.device).multi_processor_count)
    y = torch.empty(B, ph, ph, 64, device=images.device, dtype=torch.bfloat16)
    if w_dense is not None:
        _need_cuda(w_dense)
        if w_dense.shape != (64, 160) or w_dense.dtype != torch.bfloat16 or not w_dense.is_contiguous():
            raise ValueError("w_dense must be pack_stem_dense_weight's contiguous bf16 [64, 160]")
    C.stem_conv_pool_u8(_ptr(images.contiguous()), _ptr(w_packed.contiguous()), _ptr(bias.float().contiguous()),
                        _ptr(y), B, S, strip, _stream(), _ptr(w_dense) if w_dense is not None else 0)
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
