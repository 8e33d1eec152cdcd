"""Numerics of the hand-written gfx950 kernels vs plain PyTorch fp32 references.

Inputs are rounded to bf16 first so the reference sees exactly what the kernel
sees; the remaining difference is the bf16 output rounding plus fp32
accumulation order.
"""
import pytest
import torch
import torch.nn.functional as F

import dmlc
from dmlc import ops

pytestmark = pytest.mark.gpu


def _nhwc(x):
    return x.permute(0, 2, 3, 1).contiguous()


def _nchw(x):
    return x.permute(0, 3, 1, 2).contiguous()


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


def test_native_loaded(gpu):
    import sys
    C = dmlc.native()
    assert C.__file__.endswith(".so")
    assert any("libdmlc_gpu.so" in l for l in open("/proc/self/maps"))
    assert "dmlc._C" in sys.modules


CONV_CASES = [
    # B, H, W, Cin, Cout, k, stride, pad, relu, res, tile, split
    (2, 56, 56, 64, 64, 3, 1, 1, True, False, -1, 1),
    (2, 56, 56, 64, 128, 3, 2, 1, True, False, -1, 1),
    (2, 56, 56, 64, 128, 1, 2, 0, False, False, -1, 1),
    (3, 28, 28, 128, 128, 3, 1, 1, True, True, -1, 1),
    (1, 7, 7, 512, 512, 3, 1, 1, True, True, -1, 4),
    (2, 13, 13, 192, 384, 3, 1, 1, True, False, -1, 1),
    (2, 27, 27, 64, 192, 5, 1, 2, True, False, -1, 1),
    (2, 14, 14, 256, 256, 3, 1, 1, False, False, 1, 1),
    (2, 14, 14, 256, 256, 3, 1, 1, False, False, 2, 1),
    (2, 14, 14, 256, 512, 1, 1, 0, False, False, 0, 3),
    # multi-stage LDS rings (counted vmcnt + raw barrier)
    (3, 28, 28, 128, 128, 3, 1, 1, True, True, 3, 1),
    (2, 56, 56, 64, 64, 3, 1, 1, True, False, 4, 1),
    (2, 14, 14, 256, 256, 3, 1, 1, False, True, 5, 1),
    (3, 28, 28, 128, 128, 3, 1, 1, True, True, 6, 1),
    (1, 7, 7, 512, 512, 3, 1, 1, True, True, 6, 4),
    (1, 7, 7, 512, 512, 3, 1, 1, True, True, 3, 16),
    (2, 14, 14, 256, 256, 1, 1, 0, False, False, 3, 1),
]
# persistent grids: a tiny block cap forces every block through many tiles
PERSIST_CASES = [
    (3, 28, 28, 128, 128, 3, 1, 1, True, True, 0, 1),
    (2, 56, 56, 64, 64, 3, 1, 1, True, False, 1, 1),
    (2, 14, 14, 256, 512, 3, 2, 1, True, False, 2, 1),
    (5, 13, 13, 192, 384, 3, 1, 1, True, True, 0, 1),
]


@pytest.mark.parametrize("case", PERSIST_CASES, ids=[str(c) for c in PERSIST_CASES])
@pytest.mark.parametrize("max_blocks", [8, 24])
def test_conv2d_persistent(gpu, case, max_blocks):
    B, H, W, Cin, Cout, k, s, p, relu, use_res, tile, split = case
    g = torch.Generator().manual_seed(9)
    x = torch.randn(B, Cin, H, W, generator=g).bfloat16().float()
    w = (torch.randn(Cout, Cin, k, k, generator=g) / (Cin * k * k) ** 0.5).bfloat16().float()
    bias = torch.randn(Cout, generator=g) * 0.1
    ref = F.conv2d(x, w, bias, s, p)
    res = None
    if use_res:
        r = torch.randn_like(ref).bfloat16().float()
        ref = ref + r
        res = _nhwc(r).bfloat16().to(gpu)
    if relu:
        ref = F.relu(ref)
    wp = ops.pack_conv_weight(w, device=gpu)
    y = ops.conv2d(_nhwc(x).bfloat16().to(gpu), wp, Cout, k, k, s, p, bias=bias.to(gpu), res=res, relu=relu,
                   tile=tile, max_blocks=max_blocks)
    torch.cuda.synchronize()
    assert _rel(_nchw(y.float().cpu()), ref) < 8e-3


# 8-wave big-tile kernel (conv_bigtile.hip): tile 11 = 256x256, 12 = 256x128,
# with the K range cut into `splits` slices (split-K hand-off through slabs
# when > 1). Shapes cover M not a tile multiple, stride 2, 1x1, uneven
# slices, more units than CUs and the ResNet layer2-4 geometries.
BT_CASES = [
    # B, H, W, Cin, Cout, k, stride, pad, relu, res, tile, splits
    (4, 7, 7, 512, 512, 3, 1, 1, True, True, 11, 2),      # layer4
    (4, 7, 7, 512, 512, 3, 1, 1, True, True, 11, 3),
    (4, 7, 7, 512, 512, 3, 1, 1, False, False, 11, 4),
    (8, 14, 14, 256, 512, 3, 2, 1, True, False, 11, 2),   # layer4.0.conv1 (stride 2)
    (6, 14, 14, 256, 256, 3, 1, 1, False, True, 11, 1),   # layer3 (M not a tile multiple)
    (5, 28, 28, 128, 256, 3, 2, 1, True, False, 11, 2),
    (3, 28, 28, 128, 128, 3, 1, 1, True, True, 12, 1),    # layer2: 256x128 tiles
    (3, 56, 56, 64, 128, 3, 2, 1, True, False, 12, 1),
    (3, 28, 28, 128, 128, 3, 1, 1, True, True, 12, 2),
    (2, 14, 14, 512, 256, 1, 1, 0, False, False, 11, 1),  # 1x1, K = 512 (8 K-tiles)
    (2, 13, 13, 384, 256, 3, 1, 1, True, False, 11, 5),   # 54 K-tiles in 5 uneven slices
    (64, 14, 14, 256, 256, 3, 1, 1, True, True, 11, 2),   # 49 tiles x 2 slices: > 1 unit per XCD slot row
]


@pytest.mark.parametrize("case", BT_CASES, ids=[str(c) for c in BT_CASES])
def test_conv2d_bigtile(gpu, case):
    B, H, W, Cin, Cout, k, s, p, relu, use_res, tile, splits = case
    g = torch.Generator().manual_seed(3)
    x = torch.randn(B, Cin, H, W, generator=g).bfloat16().float()
    w = (torch.randn(Cout, Cin, k, k, generator=g) / (Cin * k * k) ** 0.5).bfloat16().float()
    bias = torch.randn(Cout, generator=g) * 0.1
    ref = F.conv2d(x, w, bias, s, p)
    res = None
    if use_res:
        r = torch.randn_like(ref).bfloat16().float()
        ref = ref + r
        res = _nhwc(r).bfloat16().to(gpu)
    if relu:
        ref = F.relu(ref)
    wp = ops.pack_conv_weight(w, device=gpu)
    xg = _nhwc(x).bfloat16().to(gpu)
    y = ops.conv2d(xg, wp, Cout, k, k, s, p, bias=bias.to(gpu), res=res, relu=relu, tile=tile, split_k=splits)
    torch.cuda.synchronize()
    assert not ops.bigtile_error(gpu), "split-K hand-off timed out"
    assert _rel(_nchw(y.float().cpu()), ref) < 8e-3
    # deterministic (fixed hand-off order) and the flags were left clean
    y2 = ops.conv2d(xg, wp, Cout, k, k, s, p, bias=bias.to(gpu), res=res, relu=relu, tile=tile, split_k=splits)
    torch.cuda.synchronize()
    assert torch.equal(y, y2)


# persistent 256x128 big tiles (tile 13): small grids force several tiles per
# workgroup, so the LDS-DMA ring streams across tile boundaries and the
# epilogue runs on the just-consumed stage while the next tile loads.
BTP_CASES = [
    # B, H, W, Cin, Cout, k, stride, pad, relu, res, grid
    (3, 28, 28, 128, 128, 3, 1, 1, True, True, 0),
    (3, 28, 28, 128, 128, 3, 1, 1, True, True, 3),
    (3, 56, 56, 64, 128, 3, 2, 1, True, False, 2),
    (4, 56, 56, 64, 128, 1, 2, 0, False, False, 5),    # 1x1 downsample, 1 K-tile per tile
    (2, 14, 14, 256, 256, 3, 1, 1, False, True, 1),    # 2 N-tiles, one workgroup walks all
    (5, 13, 13, 192, 384, 3, 1, 1, True, False, 4),    # M not a tile multiple, 3 N-tiles
]


@pytest.mark.parametrize("case", BTP_CASES, ids=[str(c) for c in BTP_CASES])
def test_conv2d_bigtile_persistent(gpu, case):
    B, H, W, Cin, Cout, k, s, p, relu, use_res, grid = case
    g = torch.Generator().manual_seed(4)
    x = torch.randn(B, Cin, H, W, generator=g).bfloat16().float()
    w = (torch.randn(Cout, Cin, k, k, generator=g) / (Cin * k * k) ** 0.5).bfloat16().float()
    bias = torch.randn(Cout, generator=g) * 0.1
    ref = F.conv2d(x, w, bias, s, p)
    res = None
    if use_res:
        r = torch.randn_like(ref).bfloat16().float()
        ref = ref + r
        res = _nhwc(r).bfloat16().to(gpu)
    if relu:
        ref = F.relu(ref)
    wp = ops.pack_conv_weight(w, device=gpu)
    y = ops.conv2d(_nhwc(x).bfloat16().to(gpu), wp, Cout, k, k, s, p, bias=bias.to(gpu), res=res, relu=relu,
                   tile=13, max_blocks=grid)
    torch.cuda.synchronize()
    assert _rel(_nchw(y.float().cpu()), ref) < 8e-3


@pytest.mark.parametrize("case", CONV_CASES, ids=[str(c) for c in CONV_CASES])
def test_conv2d_vs_torch(gpu, case):
    B, H, W, Cin, Cout, k, s, p, relu, use_res, tile, split = case
    g = torch.Generator().manual_seed(1)
    x = torch.randn(B, Cin, H, W, generator=g).bfloat16().float()
    w = (torch.randn(Cout, Cin, k, k, generator=g) / (Cin * k * k) ** 0.5).bfloat16().float()
    bias = torch.randn(Cout, generator=g) * 0.1
    ref = F.conv2d(x, w, bias, s, p)
    Ho, Wo = ref.shape[2], ref.shape[3]
    res = None
    if use_res:
        res_nchw = torch.randn(B, Cout, Ho, Wo, generator=g).bfloat16().float()
        ref = ref + res_nchw
        res = _nhwc(res_nchw).bfloat16().to(gpu)
    if relu:
        ref = F.relu(ref)
    wp = ops.pack_conv_weight(w, device=gpu)
    y = ops.conv2d(_nhwc(x).bfloat16().to(gpu), wp, Cout, k, k, s, p, bias=bias.to(gpu), res=res, relu=relu,
                   split_k=split, tile=tile)
    torch.cuda.synchronize()
    got = _nchw(y.float().cpu())
    assert got.shape == ref.shape
    assert _rel(got, ref) < 8e-3, _rel(got, ref)


@pytest.mark.parametrize("k,s,p,cout,hw", [(7, 2, 3, 64, (56, 60)), (11, 4, 2, 64, (57, 61)),
                                           (3, 2, 1, 128, (58, 62)), (4, 2, 1, 64, (57, 61)),
                                           (7, 2, 3, 64, (224, 224)), (11, 4, 2, 64, (224, 224))])
def test_conv2d_stem_packed(gpu, k, s, p, cout, hw):
    """3-channel stem on the zero-padded packed RGB image (8 (kw,c) values
    per 16-B chunk, k = kh*CPK*8 + kw*3 + c)."""
    g = torch.Generator().manual_seed(2)
    B, (H, W) = 2, hw
    x = torch.randn(B, 3, H, W, generator=g).bfloat16().float()
    w = (torch.randn(cout, 3, k, k, generator=g) / (3 * k * k) ** 0.5).bfloat16().float()
    ref = F.relu(F.conv2d(x, w, None, s, p))
    Ho, Wo = ref.shape[2:4]
    cpk = (3 * k + 7) // 8
    need = ((Wo - 1) * s * 3 + cpk * 8 + 2) // 3
    Wr = (max(W + 2 * p, need) + 7) // 8 * 8
    xp = ops.stem_image(_nhwc(x), p, Wr)
    wp = ops.pack_conv_weight(w, stem=True, device=gpu)
    y = ops.conv2d(xp.bfloat16().to(gpu), wp, cout, k, k, s, p, relu=True, stem=True, out_hw=(Ho, Wo))
    torch.cuda.synchronize()
    assert y.shape[1:3] == ref.shape[2:4]
    assert _rel(_nchw(y.float().cpu()), ref) < 8e-3


@pytest.mark.parametrize("B,S,strip", [(3, 224, None), (2, 224, 2), (2, 224, 14), (1, 224, 56),
                                       (2, 128, None), (1, 256, 8), (4, 192, 6)])
def test_stem_conv_pool(gpu, B, S, strip):
    """Fused conv7x7/s2/p3 + bias + ReLU + maxpool3x3/s2/p1 (stem_pool.hip)
    vs torch fp32 on the same bf16-rounded image and weights."""
    g = torch.Generator().manual_seed(11)
    x = torch.randn(B, 3, S, S, generator=g).bfloat16().float()
    w = (torch.randn(64, 3, 7, 7, generator=g) / 147 ** 0.5).bfloat16().float()
    bias = torch.randn(64, generator=g) * 0.1
    ref = F.max_pool2d(F.relu(F.conv2d(x, w, bias, 2, 3)), 3, 2, 1)
    xp = ops.paired_image(_nhwc(x), 3).bfloat16().to(gpu)
    wp = ops.pack_stem_pool_weight(w, device=gpu)
    y = ops.stem_conv_pool(xp, wp, bias.to(gpu), S, strip)
    torch.cuda.synchronize()
    got = _nchw(y.float().cpu())
    assert got.shape == ref.shape
    assert _rel(got, ref) < 5e-3, _rel(got, ref)
    assert (got - ref).abs().max().item() < 0.05


@pytest.mark.parametrize("B,S,strip", [(3, 224, None), (2, 224, 2), (1, 224, 56), (2, 128, None), (4, 192, 6),
                                       (1, 256, 8), (1, 224, 2), (1, 224, None)])
def test_stem_conv_pool_u8(gpu, B, S, strip):
    """Stem with the preprocess fused (u8 images in): bit-identical to the
    two-kernel path preprocess_u8(paired) -> stem_conv_pool. At 224x224 and
    query batches the strips also split the channels over 2 or 4
    workgroups (B = 1 strip 2: 4; B = 3: 2)."""
    g = torch.Generator().manual_seed(12)
    img = torch.randint(0, 256, (B, S, S, 3), dtype=torch.uint8, generator=g).to(gpu)
    w = (torch.randn(64, 3, 7, 7, generator=g) / 147 ** 0.5).bfloat16().float()
    bias = (torch.randn(64, generator=g) * 0.1).to(gpu)
    wp = ops.pack_stem_pool_weight(w, device=gpu)
    C = dmlc.native()
    pairs = C.stem_row_width(S, 3, 7, 2) // 2
    wd = ops.pack_stem_dense_weight(w, device=gpu)
    two = ops.stem_conv_pool(ops.preprocess_u8(img, S, 3, 2 * pairs, paired=True), wp, bias, S, strip)
    one = ops.stem_conv_pool_u8(img, wp, bias, strip)
    C.stem_conv_pool_set_dbg(512)  # one workgroup per image, MFMA / helper waves: same arithmetic
    try:
        roles = ops.stem_conv_pool_u8(img, wp, bias, strip)  # raw rows by 16-B LDS-DMA (aligned images)
        # dense K (5 K steps a fragment): the same products summed in another order
        dense = ops.stem_conv_pool_u8(img, wp, bias, strip, w_dense=wd)
        zeroed = ops.stem_conv_pool_u8(img, wp, bias, strip, w_dense=torch.zeros_like(wd))  # it reads w_dense
        C.stem_conv_pool_set_dbg(512 | 2048)  # ... by 4-B LDS-DMA (the paired kernel: no dense form)
        roles4 = ops.stem_conv_pool_u8(img, wp, bias, strip, w_dense=wd)
    finally:
        C.stem_conv_pool_set_dbg(0)
    torch.cuda.synchronize()
    assert torch.equal(one, two)
    assert torch.equal(roles, two)
    assert torch.equal(roles4, two)
    # fp32 sums in a different order, then one bf16 rounding: at most one
    # bf16 ulp apart, and only where a sum lands near a rounding boundary
    d, t = dense.float(), two.float()
    assert (d - t).abs().le(t.abs() * 2.0 ** -7 + 1e-6).all(), (d - t).abs().max().item()
    assert (d != t).float().mean().item() < 0.05
    assert torch.equal(zeroed, F.relu(bias).bfloat16().view(1, 1, 1, 64).expand_as(zeroed))


@pytest.mark.parametrize("HW,C,B,res,relu", [(28, 128, 1, False, True), (28, 128, 3, True, True),
                                             (28, 128, 2, True, False), (28, 128, 5, False, False),
                                             (14, 256, 1, False, True), (14, 256, 3, True, True),
                                             (14, 256, 2, True, False), (7, 512, 1, False, True),
                                             (7, 512, 3, True, True), (7, 512, 4, True, False),
                                             (56, 64, 1, True, True), (56, 64, 2, False, True)])
def test_conv3x3_stream(gpu, HW, C, B, res, relu):
    """Direct 3x3 conv with streamed weights (conv3x3_stream.hip: 28x28x128
    half images, 14x14x256 whole images, 7x7x512 image pairs x half the
    channels; odd B leaves a one-image group) vs torch fp32."""
    g = torch.Generator().manual_seed(21)
    x = torch.randn(B, C, HW, HW, generator=g).bfloat16().float()
    w = (torch.randn(C, C, 3, 3, generator=g) / (9 * C) ** 0.5).bfloat16().float()
    bias = torch.randn(C, generator=g) * 0.1
    ref = F.conv2d(x, w, bias, 1, 1)
    r = None
    if res:
        r_nchw = torch.randn_like(ref).bfloat16().float()
        ref = ref + r_nchw
        r = _nhwc(r_nchw).bfloat16().to(gpu)
    if relu:
        ref = F.relu(ref)
    wp = ops.pack_conv_weight(w, device=gpu)
    y = ops.conv3x3_stream(_nhwc(x).bfloat16().to(gpu), wp, bias.to(gpu), r, relu)
    torch.cuda.synchronize()
    assert _rel(_nchw(y.float().cpu()), ref) < 8e-3


@pytest.mark.parametrize("HW,Cin,B,relu,cmul", [(56, 64, 1, True, 2), (56, 64, 2, False, 2), (28, 128, 1, True, 2),
                                               (28, 128, 3, False, 2), (14, 256, 1, True, 2), (14, 256, 3, False, 2),
                                               (56, 128, 1, True, 1), (56, 128, 3, False, 1)])
def test_conv3x3_stream_stride2(gpu, HW, Cin, B, relu, cmul):
    """Stride-2 direct 3x3 conv (conv3x3_stream.hip: 56x56x64 -> 28x28x128 in
    quarter images, 28x28x128 -> 14x14x256 in half images, ResNet50's
    56x56x128 -> 28x28x128 in 2-row strips (LDS weight ring) and 4-row strips
    (register weights, bit-identical), even-first column layout) vs torch fp32."""
    g = torch.Generator().manual_seed(22)
    Cout = cmul * Cin
    x = torch.randn(B, Cin, HW, HW, generator=g).bfloat16().float()
    w = (torch.randn(Cout, Cin, 3, 3, generator=g) / (9 * Cin) ** 0.5).bfloat16().float()
    bias = torch.randn(Cout, generator=g) * 0.1
    ref = F.conv2d(x, w, bias, 2, 1)
    if relu:
        ref = F.relu(ref)
    wp = ops.pack_conv_weight(w, device=gpu)
    y = ops.conv3x3_stream(_nhwc(x).bfloat16().to(gpu), wp, bias.to(gpu), None, relu, stride=2)
    torch.cuda.synchronize()
    assert y.shape == (B, HW // 2, HW // 2, Cout)
    assert _rel(_nchw(y.float().cpu()), ref) < 8e-3
    if cmul == 1:  # the register-weight variant: same MFMA order per output
        yw = ops.conv3x3_stream(_nhwc(x).bfloat16().to(gpu), wp, bias.to(gpu), None, relu, stride=2, frag=True)
        torch.cuda.synchronize()
        assert torch.equal(y, yw)


@pytest.mark.parametrize("HW,C,B,res,variant", [(7, 512, 1, False, 0), (7, 512, 3, True, 0), (7, 512, 4, True, 0),
                                                (14, 256, 1, False, 0), (14, 256, 3, True, 0), (14, 256, 2, True, 1)])
def test_conv3x3_stream_register_weights(gpu, HW, C, B, res, variant):
    """Stride-1 stream convs with the weights in fragment order loaded
    straight into VGPRs (WR variants; 14x14x256 with two 32-channel groups
    per wave, ring depth 4 or 2 by variant) vs torch fp32, and bit-identical to the
    LDS-ring variants (same MFMA order per output)."""
    nat = dmlc.native()
    nat.conv3x3_stream_set_variant(variant)
    try:
        _stream_register_weights(gpu, HW, C, B, res)
    finally:
        nat.conv3x3_stream_set_variant(0)


def _stream_register_weights(gpu, HW, C, B, res):
    g = torch.Generator().manual_seed(24)
    x = torch.randn(B, C, HW, HW, generator=g).bfloat16().float()
    w = (torch.randn(C, C, 3, 3, generator=g) / (9 * C) ** 0.5).bfloat16().float()
    bias = torch.randn(C, generator=g) * 0.1
    ref = F.conv2d(x, w, bias, 1, 1)
    r = None
    if res:
        r_nchw = torch.randn_like(ref).bfloat16().float()
        ref = ref + r_nchw
        r = _nhwc(r_nchw).bfloat16().to(gpu)
    ref = F.relu(ref)
    wp = ops.pack_conv_weight(w, device=gpu)
    xg = _nhwc(x).bfloat16().to(gpu)
    y = ops.conv3x3_stream(xg, wp, bias.to(gpu), r, True, frag=True)
    y0 = ops.conv3x3_stream(xg, wp, bias.to(gpu), r, True)
    torch.cuda.synchronize()
    assert _rel(_nchw(y.float().cpu()), ref) < 8e-3
    assert torch.equal(y, y0)


@pytest.mark.parametrize("HW,Cin,B", [(56, 64, 2), (28, 128, 3), (14, 256, 2)])
def test_conv3x3_stream_fused_downsample(gpu, HW, Cin, B):
    """Stride-2 stream conv that also computes the block's 1x1/s2 downsample
    conv from its resident input (extra K-tiles on tap (1,1)) vs torch fp32;
    the 3x3 output must equal the unfused kernel's bit for bit."""
    g = torch.Generator().manual_seed(23)
    Cout = 2 * Cin
    x = torch.randn(B, Cin, HW, HW, generator=g).bfloat16().float()
    w = (torch.randn(Cout, Cin, 3, 3, generator=g) / (9 * Cin) ** 0.5).bfloat16().float()
    wd = (torch.randn(Cout, Cin, 1, 1, generator=g) / Cin ** 0.5).bfloat16().float()
    bias = torch.randn(Cout, generator=g) * 0.1
    bd = torch.randn(Cout, generator=g) * 0.1
    ref_d = F.conv2d(x, wd, bd, 2, 0)
    xg = _nhwc(x).bfloat16().to(gpu)
    wp = ops.pack_conv_weight(w, device=gpu)
    wdp = ops.pack_conv_weight(wd, device=gpu)
    y0 = ops.conv3x3_stream(xg, wp, bias.to(gpu), None, True, stride=2)
    y, yd = ops.conv3x3_stream(xg, wp, bias.to(gpu), None, True, stride=2, downsample=(wdp, bd.to(gpu)))
    torch.cuda.synchronize()
    assert torch.equal(y, y0)
    assert _rel(_nchw(yd.float().cpu()), ref_d) < 8e-3
    if dmlc.native().conv3x3_stream_uses_frag(HW, HW, Cin, Cout, 2):  # register-weight variant: same MFMA order
        y2, yd2 = ops.conv3x3_stream(xg, wp, bias.to(gpu), None, True, stride=2, downsample=(wdp, bd.to(gpu)),
                                     frag=True)
        y3 = ops.conv3x3_stream(xg, wp, bias.to(gpu), None, True, stride=2, frag=True)
        torch.cuda.synchronize()
        assert torch.equal(y2, y0) and torch.equal(yd2, yd) and torch.equal(y3, y0)
        nat = dmlc.native()
        for v in (2, 4):  # one / two channel groups per wave: same MFMA order per output
            nat.conv3x3_stream_set_variant(v)
            try:
                y4, yd4 = ops.conv3x3_stream(xg, wp, bias.to(gpu), None, True, stride=2,
                                             downsample=(wdp, bd.to(gpu)), frag=True)
                torch.cuda.synchronize()
            finally:
                nat.conv3x3_stream_set_variant(0)
            assert torch.equal(y4, y0) and torch.equal(yd4, yd)


@pytest.mark.parametrize("B,strip,res", [(2, None, False), (2, None, True), (3, 4, True), (1, 8, False),
                                         (1, 28, True)])
def test_conv3x3_rows(gpu, B, strip, res):
    """Direct row-streaming 3x3 conv (conv3x3_rows.hip) vs torch fp32."""
    g = torch.Generator().manual_seed(13)
    x = torch.randn(B, 64, 56, 56, generator=g).bfloat16().float()
    w = (torch.randn(64, 64, 3, 3, generator=g) / 24).bfloat16().float()
    bias = torch.randn(64, generator=g) * 0.1
    r = torch.randn(B, 64, 56, 56, generator=g).bfloat16().float() if res else None
    ref = F.conv2d(x, w, bias, 1, 1)
    if res:
        ref = ref + r
    ref = F.relu(ref)
    wp = ops.pack_conv_weight(w, device=gpu)
    y = ops.conv3x3_rows(_nhwc(x).bfloat16().to(gpu), wp, bias.to(gpu),
                         _nhwc(r).bfloat16().to(gpu) if res else None, True, strip)
    torch.cuda.synchronize()
    got = _nchw(y.float().cpu())
    assert _rel(got, ref) < 5e-3, _rel(got, ref)
    assert (got - ref).abs().max().item() < 0.1
    # register-weight variant (weights from L2 in fragment order): same MFMA order
    y2 = ops.conv3x3_rows(_nhwc(x).bfloat16().to(gpu), wp, bias.to(gpu),
                          _nhwc(r).bfloat16().to(gpu) if res else None, True, strip, frag=True)
    torch.cuda.synchronize()
    assert torch.equal(y2, y)


@pytest.mark.parametrize("M,K,N,relu,f32,splits", [(256, 9216, 4096, True, False, 0), (256, 4096, 4096, True, False, 0),
                                                   (256, 4096, 1000, False, True, 0), (3, 9216, 4096, True, False, 0),
                                                   (200, 1024, 256, True, False, 1), (64, 4096, 1000, False, True, 4)])
def test_fc_gemm(gpu, M, K, N, relu, f32, splits):
    """Fully connected layers on fc_gemm.hip (AlexNet's classifier shapes at
    B = 256, a query batch, a ragged M, one and several K slices) vs torch
    fp32 on the same bf16 operands; the zero-page rows past M stay out of
    the result."""
    g = torch.Generator().manual_seed(41)
    x = torch.randn(M, K, generator=g).bfloat16().float()
    w = (torch.randn(N, K, generator=g) / K ** 0.5).bfloat16().float()
    b = torch.randn(N, generator=g) * 0.1
    ref = x @ w.t() + b
    if relu:
        ref = F.relu(ref)
    wp = ops.pack_conv_weight(w.view(N, K, 1, 1), device=gpu)
    assert wp.shape[1] == K and wp.shape[0] % 128 == 0
    y = ops.fc(x.bfloat16().to(gpu), wp, N, bias=b.to(gpu), relu=relu, out_f32=f32, splits=splits)
    torch.cuda.synchronize()
    assert y.shape == (M, N) and y.dtype == (torch.float32 if f32 else torch.bfloat16)
    assert _rel(y.float().cpu(), ref) < 5e-3, _rel(y.float().cpu(), ref)


@pytest.mark.parametrize("B", [1, 3])
def test_conv3x3_block(gpu, B):
    """Fused layer1 basic block (conv3x3_block.hip: conv1 producer waves ->
    LDS -> conv2 consumer waves + residual) vs torch fp32, and vs two
    register-weight row convs: the block starts its accumulators from the
    bias and adds the residual by v_dot2c_f32_bf16, the row convs add both
    after the K loop, so the two round differently (the bf16 intermediate
    too): within a few bf16 steps of each other, equally close to fp32."""
    g = torch.Generator().manual_seed(31)
    x = torch.randn(B, 64, 56, 56, generator=g).bfloat16().float()
    w1 = (torch.randn(64, 64, 3, 3, generator=g) / 24).bfloat16().float()
    w2 = (torch.randn(64, 64, 3, 3, generator=g) / 24).bfloat16().float()
    b1 = torch.randn(64, generator=g) * 0.1
    b2 = torch.randn(64, generator=g) * 0.1
    t = F.relu(F.conv2d(x, w1, b1, 1, 1)).bfloat16().float()
    ref = F.relu(F.conv2d(t, w2, b2, 1, 1) + x)
    xg = _nhwc(x).bfloat16().to(gpu)
    wp1, wp2 = ops.pack_conv_weight(w1, device=gpu), ops.pack_conv_weight(w2, device=gpu)
    y = ops.conv3x3_block(xg, wp1, b1.to(gpu), wp2, b2.to(gpu))
    tg = ops.conv3x3_rows(xg, wp1, b1.to(gpu), None, True, frag=True)
    y2 = ops.conv3x3_rows(tg, wp2, b2.to(gpu), xg, True, frag=True)
    torch.cuda.synchronize()
    got = _nchw(y.float().cpu())
    assert _rel(got, ref) < 5e-3, _rel(got, ref)
    assert abs(_rel(got, ref) - _rel(_nchw(y2.float().cpu()), ref)) < 1e-3
    d = (y.float() - y2.float()).abs()
    tol = y2.float().abs() * 2.0 ** -5 + 2e-3 * y2.float().abs().max()
    assert (d <= tol).all(), (d - tol).max()
    assert (d > 0).float().mean() < 5e-2


@pytest.mark.parametrize("B", [1, 5])
def test_conv3x3_s2rows(gpu, B):
    """Row-streaming weight-stationary layer2.0 conv1 + downsample
    (conv3x3_s2rows.hip) vs torch fp32 and vs the stream conv's fused
    downsample variant."""
    g = torch.Generator().manual_seed(37)
    x = torch.randn(B, 64, 56, 56, generator=g).bfloat16().float()
    w = (torch.randn(128, 64, 3, 3, generator=g) / 24).bfloat16().float()
    wd = (torch.randn(128, 64, 1, 1, generator=g) / 8).bfloat16().float()
    bias = torch.randn(128, generator=g) * 0.1
    bd = torch.randn(128, generator=g) * 0.1
    ref = F.relu(F.conv2d(x, w, bias, 2, 1))
    ref_d = F.conv2d(x, wd, bd, 2, 0)
    xg = _nhwc(x).bfloat16().to(gpu)
    wp, wdp = ops.pack_conv_weight(w, device=gpu), ops.pack_conv_weight(wd, device=gpu)
    y, yd = ops.conv3x3_s2rows(xg, wp, bias.to(gpu), wdp, bd.to(gpu))
    y0, yd0 = ops.conv3x3_stream(xg, wp, bias.to(gpu), None, True, stride=2, downsample=(wdp, bd.to(gpu)))
    torch.cuda.synchronize()
    assert _rel(_nchw(y.float().cpu()), ref) < 5e-3, _rel(_nchw(y.float().cpu()), ref)
    assert _rel(_nchw(yd.float().cpu()), ref_d) < 5e-3, _rel(_nchw(yd.float().cpu()), ref_d)
    assert (y.float() - y0.float()).abs().max().item() < 0.05
    assert (yd.float() - yd0.float()).abs().max().item() < 0.05


@pytest.mark.parametrize("B,out8", [(1, False), (3, False), (2, True)])
def test_conv3x3_s2rows128(gpu, B, out8):
    """ResNet50 layer2.0.conv2 row-streaming kernel (conv3x3_s2rows128.hip)
    vs torch fp32: bf16 output, and e4m3 output (relu(v) * inv_scale,
    dequantised) against the same reference at e4m3 resolution."""
    g = torch.Generator().manual_seed(41 + B)
    x = torch.randn(B, 128, 56, 56, generator=g).bfloat16().float()
    w = (torch.randn(128, 128, 3, 3, generator=g) / 34).bfloat16().float()
    bias = torch.randn(128, generator=g) * 0.1
    ref = F.relu(F.conv2d(x, w, bias, 2, 1))
    xg = _nhwc(x).bfloat16().to(gpu)
    wp = ops.pack_conv_weight(w, device=gpu)
    if not out8:
        y = ops.conv3x3_s2rows128(xg, wp, bias.to(gpu))
        torch.cuda.synchronize()
        assert _rel(_nchw(y.float().cpu()), ref) < 5e-3, _rel(_nchw(y.float().cpu()), ref)
    else:
        scale = ref.abs().max().item() / 448.0
        y8 = ops.conv3x3_s2rows128(xg, wp, bias.to(gpu), out_inv_scale=1.0 / scale)
        torch.cuda.synchronize()
        deq = y8.view(torch.float8_e4m3fn).float().cpu() * scale
        assert _rel(_nchw(deq), ref) < 4e-2, _rel(_nchw(deq), ref)


# every ResNet18/34 3x3 shape at query batches; mf None = the engine's pick
@pytest.mark.parametrize("HW,Cin,Cout,stride", [(56, 64, 64, 1), (56, 64, 128, 2), (28, 128, 128, 1),
                                                (28, 128, 256, 2), (14, 256, 256, 1), (14, 256, 512, 2),
                                                (7, 512, 512, 1)])
@pytest.mark.parametrize("B,mf", [(1, None), (1, 1), (1, 2), (1, 4), (3, None)])
def test_conv_small(gpu, HW, Cin, Cout, stride, B, mf):
    """Query-batch conv (conv_small.hip) vs torch fp32: stride 1 with a
    residual, stride 2 with the fused 1x1/s2 downsample."""
    g = torch.Generator().manual_seed(53 + HW + Cin)
    x = torch.randn(B, Cin, HW, HW, generator=g).bfloat16().float()
    w = (torch.randn(Cout, Cin, 3, 3, generator=g) / (3 * Cin ** 0.5)).bfloat16().float()
    bias = torch.randn(Cout, generator=g) * 0.1
    wp = ops.pack_conv_weight(w, device=gpu)
    xg = _nhwc(x).bfloat16().to(gpu)
    if stride == 1:
        r = torch.randn(B, Cout, HW, HW, generator=g).bfloat16().float()
        ref = F.relu(F.conv2d(x, w, bias, 1, 1) + r)
        y = ops.conv_small(xg, wp, bias.to(gpu), _nhwc(r).bfloat16().to(gpu), True, mf=mf)
        torch.cuda.synchronize()
        assert _rel(_nchw(y.float().cpu()), ref) < 5e-3, _rel(_nchw(y.float().cpu()), ref)
    else:
        wd = (torch.randn(Cout, Cin, 1, 1, generator=g) / Cin ** 0.5).bfloat16().float()
        bd = torch.randn(Cout, generator=g) * 0.1
        ref = F.relu(F.conv2d(x, w, bias, 2, 1))
        ref_d = F.conv2d(x, wd, bd, 2, 0)
        y, yd = ops.conv_small(xg, wp, bias.to(gpu), None, True, stride=2,
                               wd_packed=ops.pack_conv_weight(wd, device=gpu), bd=bd.to(gpu), mf=mf)
        torch.cuda.synchronize()
        assert _rel(_nchw(y.float().cpu()), ref) < 5e-3, _rel(_nchw(y.float().cpu()), ref)
        assert _rel(_nchw(yd.float().cpu()), ref_d) < 5e-3, _rel(_nchw(yd.float().cpu()), ref_d)


@pytest.mark.parametrize("B,res", [(1, False), (3, True), (2, False)])
def test_conv3x3_rows28(gpu, B, res):
    """Weight-stationary row-streaming layer2 conv (conv3x3_rows28.hip) vs
    torch fp32, and vs the stream conv on the same operands."""
    g = torch.Generator().manual_seed(41)
    x = torch.randn(B, 128, 28, 28, generator=g).bfloat16().float()
    w = (torch.randn(128, 128, 3, 3, generator=g) / 34).bfloat16().float()
    bias = torch.randn(128, generator=g) * 0.1
    r = torch.randn(B, 128, 28, 28, generator=g).bfloat16().float() if res else None
    ref = F.conv2d(x, w, bias, 1, 1)
    if res:
        ref = ref + r
    ref = F.relu(ref)
    xg = _nhwc(x).bfloat16().to(gpu)
    rg = _nhwc(r).bfloat16().to(gpu) if res else None
    wp = ops.pack_conv_weight(w, device=gpu)
    y = ops.conv3x3_rows28(xg, wp, bias.to(gpu), rg, True)
    y0 = ops.conv3x3_stream(xg, wp, bias.to(gpu), rg, True)
    torch.cuda.synchronize()
    got = _nchw(y.float().cpu())
    assert _rel(got, ref) < 5e-3, _rel(got, ref)
    assert (y.float() - y0.float()).abs().max().item() < 0.05


def test_preprocess_paired(gpu):
    g = torch.Generator().manual_seed(12)
    img = torch.randint(0, 256, (2, 224, 224, 3), generator=g, dtype=torch.uint8)
    ref = _nhwc((_nchw(img.float()) / 255 - MEAN) / STD)
    y = ops.preprocess_u8(img.to(gpu), 224, 3, 232, paired=True)
    torch.cuda.synchronize()
    assert y.shape == (2, 230, 116, 8)
    exp = ops.paired_image(ref, 3, 116)
    y = y.float().cpu()
    assert _rel(y, exp) < 4e-3
    assert torch.all(y[..., 6:] == 0)


def test_linear_fp32_out(gpu):
    """FC = 1x1 conv on [B,1,1,K]; N=1000 padded to 1024, fp32 logits."""
    g = torch.Generator().manual_seed(3)
    B, K, N = 5, 512, 1000
    x = torch.randn(B, K, generator=g).bfloat16().float()
    w = (torch.randn(N, K, generator=g) / K ** 0.5).bfloat16().float()
    b = torch.randn(N, generator=g)
    ref = x @ w.t() + b
    wp = ops.pack_conv_weight(w.view(N, K, 1, 1), device=gpu)
    for split in (1, 4):
        y = ops.conv2d(x.view(B, 1, 1, K).bfloat16().to(gpu), wp, N, 1, 1, bias=b.to(gpu), out_f32=True,
                       split_k=split)
        torch.cuda.synchronize()
        assert y.dtype == torch.float32
        assert _rel(y.view(B, N).cpu(), ref) < 5e-3


def test_maxpool(gpu):
    g = torch.Generator().manual_seed(4)
    x = torch.randn(2, 64, 112, 112, generator=g).bfloat16().float()
    for k, s, p in [(3, 2, 1), (3, 2, 0)]:
        ref = F.max_pool2d(x, k, s, p)
        y = ops.maxpool2d(_nhwc(x).bfloat16().to(gpu), k, s, p)
        torch.cuda.synchronize()
        assert torch.equal(_nchw(y.float().cpu()), ref)


def test_avgpool(gpu):
    g = torch.Generator().manual_seed(5)
    x = torch.randn(3, 512, 7, 7, generator=g).bfloat16().float()
    ref = F.adaptive_avg_pool2d(x, 1).view(3, 512)
    y = ops.avgpool_global(_nhwc(x).bfloat16().to(gpu))
    torch.cuda.synchronize()
    assert _rel(y.float().cpu(), ref) < 5e-3
    x2 = torch.randn(2, 256, 13, 13, generator=g).bfloat16().float()
    ref2 = F.adaptive_avg_pool2d(x2, (6, 6))
    y2 = ops.avgpool_adaptive(_nhwc(x2).bfloat16().to(gpu), 6, 6)
    torch.cuda.synchronize()
    assert _rel(_nchw(y2.float().cpu()), ref2) < 5e-3


MEAN = torch.tensor([0.485, 0.456, 0.406]).view(1, 3, 1, 1)
STD = torch.tensor([0.229, 0.224, 0.225]).view(1, 3, 1, 1)


def test_preprocess_identity(gpu):
    g = torch.Generator().manual_seed(6)
    img = torch.randint(0, 256, (3, 224, 224, 3), generator=g, dtype=torch.uint8)
    ref = (_nchw(img.float()) / 255 - MEAN) / STD
    for pad, wr in ((0, 224), (3, 232), (2, 240)):
        y = ops.preprocess_u8(img.to(gpu), 224, pad, wr)
        torch.cuda.synchronize()
        y = y.float().cpu()
        assert y.shape == (3, 224 + 2 * pad, wr, 3)
        exp = ops.stem_image(_nhwc(ref), pad, wr)
        assert _rel(y, exp) < 4e-3
        assert torch.all(y[:, :pad] == 0) and torch.all(y[:, :, 224 + pad:] == 0)


def test_preprocess_resize(gpu):
    """Short side -> 224 (long = floor(224*long/short)), centre crop at
    integer offsets, bilinear align_corners=False == torch interpolate."""
    g = torch.Generator().manual_seed(7)
    for (H, W) in [(300, 400), (500, 333), (224, 224), (180, 240)]:
        img = torch.randint(0, 256, (2, H, W, 3), generator=g, dtype=torch.uint8)
        if H <= W:
            rh, rw = 224, (224 * W) // H
        else:
            rh, rw = (224 * H) // W, 224
        rs = F.interpolate(_nchw(img.float()), size=(rh, rw), mode="bilinear", align_corners=False)
        oy, ox = (rh - 224) // 2, (rw - 224) // 2
        ref = (rs[:, :, oy:oy + 224, ox:ox + 224] / 255 - MEAN) / STD
        y = ops.preprocess_u8(img.to(gpu), 224, 0)
        torch.cuda.synchronize()
        got = _nchw(y.float().cpu()[..., :3].contiguous())
        assert _rel(got, ref) < 5e-3, (H, W, _rel(got, ref))


def test_softmax_top1(gpu):
    g = torch.Generator().manual_seed(8)
    logits = torch.randn(37, 1000, generator=g) * 3
    logits[5, 17] = 100.0
    p = torch.softmax(logits, -1)
    pv, pi = p.max(-1)
    idx, prob = ops.softmax_top1(logits.to(gpu))
    torch.cuda.synchronize()
    assert torch.equal(idx.cpu().long(), pi)
    assert torch.allclose(prob.cpu(), pv, rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("B,H,C,S", [(3, 14, 256, 1), (2, 7, 512, 1), (3, 7, 512, 1), (40, 14, 256, 1),
                                     (3, 28, 256, 2), (2, 14, 512, 2), (3, 28, 128, 1), (1, 28, 128, 1),
                                     (2, 56, 128, 2)])
def test_conv3x3_stream8(gpu, B, H, C, S):
    """The e4m3 3x3/s1 conv (conv3x3_stream8.hip, block-scaled e4m3 MFMA) vs
    fp32 torch on the same e4m3 operands (dequantised): the only difference is
    the output's e4m3 rounding (3 mantissa bits, <= 1/16 relative), so the
    dequantised output is within 0.04 relative L2 and no element is more than
    one e4m3 step off the exactly rounded fp32 result. Odd batches leave the
    7x7 kernel's last workgroup one image short; stride 2 (ResNet50 layer3.0 /
    layer4.0 conv2) runs half-image strips on 28x28x256 (layer2.0 conv2:
    quarter-image strips of 56x56x128); layer2 (28x28x128) half images with a
    halo row and 128-B pixels."""
    g = torch.Generator().manual_seed(100 + B + C)
    x = torch.randn(B, H, H, C, generator=g).clamp_min(0)  # post-ReLU t1
    sx = x.abs().max().item() / ops.FP8_MAX
    xq = ops.quantize_fp8(x, sx)
    w = torch.randn(C, C, 3, 3, generator=g) / (9 * C) ** 0.5
    wq, sw = ops.pack_conv_weight_fp8(w)
    bias = torch.randn(C, generator=g) * 0.05
    alpha = sx * sw
    wd = (wq.float()[:C, :9 * C] * sw[:C, None]).view(C, 3, 3, C).permute(0, 3, 1, 2)
    ref = F.relu(F.conv2d(xq.float().permute(0, 3, 1, 2) * sx, wd, bias, stride=S, padding=1)).permute(0, 2, 3, 1)
    out_scale = ref.abs().max().item() / ops.FP8_MAX
    y = ops.conv3x3_stream8(xq.to(gpu), wq.to(gpu), alpha.to(gpu), bias.to(gpu), relu=True, out_scale=out_scale,
                            stride=S)
    if C == 128 and S == 2:  # layer2.0's other strip height (variant 4): same sums, same bits
        Cn = dmlc.native()
        Cn.conv3x3_stream8_set_variant(4)
        try:
            y2 = ops.conv3x3_stream8(xq.to(gpu), wq.to(gpu), alpha.to(gpu), bias.to(gpu), relu=True,
                                     out_scale=out_scale, stride=S)
        finally:
            Cn.conv3x3_stream8_set_variant(0)
        torch.cuda.synchronize()
        assert torch.equal(y.view(torch.uint8), y2.view(torch.uint8))
    torch.cuda.synchronize()
    got = y.float().cpu() * out_scale
    assert _rel(got, ref) < 0.04, _rel(got, ref)
    exact = ops.quantize_fp8(ref, out_scale).float() * out_scale
    # about one e4m3 step (accumulation order moves values across a rounding
    # boundary): all but 1e-4 of the elements within one, none beyond two
    step = (exact.abs() / 8).clamp_min(out_scale * 2 ** -9)
    err = (got - exact).abs()
    assert (err <= step * 1.01).float().mean().item() >= 0.9999
    assert (err <= 2 * step * 1.01).all()
