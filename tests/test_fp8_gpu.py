"""fp8 (OCP e4m3) matrix-core path: pin the operand lane map of the
block-scaled MFMA with exact integer data (cdna_hip_programming.md: "check
the map with exact integer data before relying on it")."""
import pytest
import torch

import dmlc

pytestmark = pytest.mark.gpu


def _k_of(h, l, j):
    """k index held in byte j (0..31) of lane l for layout hypothesis h."""
    g = l >> 4
    if h == "contig32":
        return 32 * g + j
    if h == "halves16":
        return 16 * g + j if j < 16 else 64 + 16 * g + (j - 16)
    if h == "quarters8":
        return 8 * g + (j % 8) + 32 * (j // 8)
    if h == "quad4":
        return 4 * g + (j % 4) + 16 * (j // 4)
    raise ValueError(h)


def _pack(mat_rows_k, h):
    """[16 rows][128 k] fp8 -> per-lane raw int32 registers [64][8]."""
    bytes_ = mat_rows_k.view(torch.uint8)
    out = torch.empty(64, 32, dtype=torch.uint8)
    for l in range(64):
        for j in range(32):
            out[l, j] = bytes_[l & 15, _k_of(h, l, j)]
    return out.view(torch.int32).reshape(64, 8)


@pytest.mark.parametrize("h", ["contig32", "halves16", "quarters8", "quad4"])
def test_mfma_scale_fp8_operand_map(gpu, h):
    g = torch.Generator().manual_seed(3)
    A = torch.randint(-3, 4, (16, 128), generator=g).float()   # exact in e4m3
    B = torch.randint(-3, 4, (128, 16), generator=g).float()
    ref = A @ B
    a8 = A.to(torch.float8_e4m3fn)
    bT8 = B.t().contiguous().to(torch.float8_e4m3fn)  # [16 cols][128 k]
    ra, rb = _pack(a8, h).to(gpu), _pack(bT8, h).to(gpu)
    d = torch.empty(64, 4, device=gpu)
    dmlc.native().mfma_fp8_probe(ra.data_ptr(), rb.data_ptr(), d.data_ptr(),
                                 torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    d = d.cpu()
    got = torch.empty(16, 16)
    for l in range(64):
        for r in range(4):
            got[4 * (l >> 4) + r, l & 15] = d[l, r]
    ok = torch.equal(got, ref)
    if h == "contig32":
        assert ok, "the conv kernel's fp8 operand map (32 contiguous k per lane) is wrong"
    else:
        print(h, "matches" if ok else "differs")


from dmlc import ops  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def _nhwc(x):
    return x.permute(0, 2, 3, 1).contiguous()


def _nchw(x):
    return x.permute(0, 3, 1, 2).contiguous()


@pytest.mark.parametrize("B,H,Cin,Cout,k,s,p,res,tile", [
    (2, 14, 256, 256, 3, 1, 1, True, -1), (2, 28, 128, 128, 3, 1, 1, False, -1),
    (2, 14, 256, 512, 1, 2, 0, False, -1), (1, 7, 512, 2048, 1, 1, 0, True, -1),
    (2, 14, 256, 192, 3, 1, 1, True, 1), (3, 7, 1024, 256, 1, 1, 0, False, -1)])
def test_conv2d_fp8_in_fp8_out(gpu, B, H, Cin, Cout, k, s, p, res, tile):
    """e4m3 activations x e4m3 per-channel-scaled weights on the block-scaled
    MFMA, fp32 accumulate, bias + e4m3 residual + ReLU, e4m3 output: compared
    with torch fp32 on the same dequantised operands; the only extra error is
    the e4m3 rounding of the output (3 mantissa bits)."""
    g = torch.Generator().manual_seed(21)
    x = torch.rand(B, Cin, H, H, generator=g) * 4          # post-ReLU-like, >= 0
    w = torch.randn(Cout, Cin, k, k, generator=g) / (Cin * k * k) ** 0.5
    bias = torch.randn(Cout, generator=g) * 0.1
    sx = float(x.abs().max()) / 448
    xq = ops.quantize_fp8(_nhwc(x), sx)
    wq, sw = ops.pack_conv_weight_fp8(w)
    xd = _nchw(xq.float() * sx)
    wd = (wq.float() * sw[:, None])[:Cout, : k * k * Cin].reshape(Cout, k, k, Cin).permute(0, 3, 1, 2)
    ref = F.conv2d(xd, wd, bias, s, p)
    rq = None
    rs = 1.0
    if res:
        r = torch.randn_like(ref)
        rs = float(r.abs().max()) / 448
        rq = ops.quantize_fp8(_nhwc(r), rs)
        ref = ref + _nchw(rq.float() * rs)
    ref = F.relu(ref)
    so = float(ref.abs().max()) / 448
    y = ops.conv2d_fp8(xq.to(gpu), wq.to(gpu), (sx * sw).to(gpu), Cout, k, k, s, p, bias=bias.to(gpu),
                       res=rq.to(gpu) if res else None, res_scale=rs, relu=True, out_scale=so, tile=tile)
    torch.cuda.synchronize()
    got = _nchw(y.float().cpu() * so)
    assert got.shape == ref.shape
    rel = ((got - ref).norm() / ref.norm()).item()
    assert rel < 0.04, rel
    # elementwise: within e4m3 rounding of the reference (half ulp = 1/16 rel) plus a subnormal floor
    assert torch.all((got - ref).abs() <= ref.abs() / 14 + 4 * so * 2 ** -9)


def test_conv2d_bf16_in_fp8_out(gpu):
    """The bf16 -> e4m3 boundary conv (ResNet50 layer1 output): bf16 operands,
    e4m3 output."""
    g = torch.Generator().manual_seed(22)
    x = torch.randn(2, 64, 56, 56, generator=g).bfloat16().float()
    w = (torch.randn(256, 64, 1, 1, generator=g) / 8).bfloat16().float()
    ref = F.relu(F.conv2d(x, w))
    so = float(ref.max()) / 448
    y = ops.conv2d_fp8(_nhwc(x).bfloat16().to(gpu), ops.pack_conv_weight(w, device=gpu), None, 256, 1, 1,
                       relu=True, out_scale=so)
    torch.cuda.synchronize()
    got = _nchw(y.float().cpu() * so)
    assert ((got - ref).norm() / ref.norm()).item() < 0.04


@pytest.mark.parametrize("B,H,Cin,Cout,s,in8,out8,res", [
    (1, 56, 64, 256, 1, False, True, True),     # layer1 expand (bf16 -> e4m3 + e4m3 residual)
    (1, 56, 64, 256, 1, False, True, False),    # layer1.0 downsample
    (1, 56, 256, 64, 1, True, False, False),    # layer1 reduce (e4m3 -> bf16)
    (4, 28, 512, 128, 1, True, False, False),   # layer2 reduce
    (4, 28, 128, 512, 1, False, True, True),    # layer2 expand
    (4, 56, 256, 512, 2, True, True, False),    # layer2.0 downsample, stride 2
    (16, 14, 256, 1024, 1, False, True, True),  # layer3 expand
    (16, 28, 512, 1024, 2, True, True, False),  # layer3.0 downsample, stride 2
    (1, 56, 64, 256, 1, False, False, True),    # bf16 model: expand + bf16 residual
    (4, 56, 256, 512, 2, False, False, False),  # bf16 model: downsample
    (16, 14, 1024, 256, 1, True, False, False),  # layer3 reduce (1-KB rows, 32-pixel blocks)
    (32, 7, 512, 2048, 1, False, True, True),    # layer4 expand
    (4, 28, 512, 128, 1, False, False, False),   # bf16 model: layer2 reduce (1-KB bf16 rows)
])
def test_conv1x1_weight_stationary(gpu, B, H, Cin, Cout, s, in8, out8, res):
    """conv1x1.hip (weights in VGPRs, LDS-DMA streamed pixel blocks, counted
    asm residual loads) on the ResNet50 bottleneck shapes vs torch fp32 on the
    same (dequantised) operands, and against the implicit-GEMM kernel."""
    g = torch.Generator().manual_seed(40 + Cin + Cout + s)
    x = torch.rand(B, Cin, H, H, generator=g) * 4
    w = torch.randn(Cout, Cin, 1, 1, generator=g) / Cin ** 0.5
    bias = torch.randn(Cout, generator=g) * 0.1
    if in8:
        sx = float(x.abs().max()) / 448
        xq = ops.quantize_fp8(_nhwc(x), sx)
        wq, sw = ops.pack_conv_weight_fp8(w)
        xd = _nchw(xq.float() * sx)
        wd = (wq.float() * sw[:, None])[:Cout, :Cin].reshape(Cout, Cin, 1, 1)
        xin, wk, alpha = xq.to(gpu), wq.to(gpu), (sx * sw).to(gpu)
    else:
        xd = x.bfloat16().float()
        wd = w.bfloat16().float()
        xin, wk, alpha = _nhwc(xd).bfloat16().to(gpu), ops.pack_conv_weight(wd, device=gpu), None
    ref = F.conv2d(xd, wd, bias, s, 0)
    rq, rs = None, 1.0
    if res:
        r = torch.randn_like(ref)
        if out8:
            rs = float(r.abs().max()) / 448
            rq = ops.quantize_fp8(_nhwc(r), rs)
            ref = ref + _nchw(rq.float() * rs)
        else:
            rq = _nhwc(r).bfloat16()
            ref = ref + _nchw(rq.float())
    ref = F.relu(ref)
    C = dmlc.native()
    if out8 or in8:
        so = float(ref.abs().max()) / 448 if out8 else None
        run = lambda tile: ops.conv2d_fp8(xin, wk, alpha, Cout, 1, 1, s, 0, bias=bias.to(gpu),  # noqa: E731
                                          res=rq.to(gpu) if res else None, res_scale=rs, relu=True, out_scale=so,
                                          tile=tile)
    else:
        so = None
        run = lambda tile: ops.conv2d(xin, wk, Cout, 1, 1, s, 0, bias=bias.to(gpu),  # noqa: E731
                                      res=rq.to(gpu) if res else None, relu=True, tile=tile)
    y = run(C.CONV_1X1)
    y0 = run(-1)
    torch.cuda.synchronize()
    scale = so if out8 else 1.0
    got, got0 = _nchw(y.float().cpu() * scale), _nchw(y0.float().cpu() * scale)
    rel = ((got - ref).norm() / ref.norm()).item()
    rel0 = ((got - got0).norm() / got0.norm()).item()
    if out8:
        assert rel < 0.04, rel
        assert torch.all((got - ref).abs() <= ref.abs() / 14 + 4 * so * 2 ** -9)
        assert rel0 < 0.02, rel0
    else:
        assert rel < 8e-3, rel
        assert rel0 < 4e-3, rel0
