"""CPU checks of the operand layouts the HIP kernels assume (no GPU needed).

Each test rebuilds, in plain PyTorch, the exact reads a kernel performs on a
packed layout and checks that they reproduce the fp32 torch op. A layout bug
then fails here, on the CPU, before any kernel runs.
"""
import torch
import torch.nn.functional as F

from dmlc import ops


def test_stem_pool_paired_layout_reproduces_conv():
    """stem_pool.hip: output column ow at kernel row kh reads the 4 chunks
    ow..ow+3 of padded input row 2*oh + kh; chunk q = pixels (2q, 2q+1) as
    [r g b r g b 0 0]; K = kh*32 + q*8 + e against pack_stem_pool_weight."""
    g = torch.Generator().manual_seed(0)
    B, S = 2, 64
    x = torch.randn(B, 3, S, S, generator=g)
    w = torch.randn(64, 3, 7, 7, generator=g).bfloat16().float()  # exact after packing
    ref = F.conv2d(x, w, None, 2, 3)  # [B, 64, S/2, S/2]
    xp = ops.paired_image(x.permute(0, 2, 3, 1), 3)  # [B, S+6, Wq, 8]
    wp = ops.pack_stem_pool_weight(w).float()  # [64, 224]
    Ho = S // 2
    assert xp.shape[2] >= Ho + 3
    rows = torch.arange(Ho).view(Ho, 1) * 2 + torch.arange(7).view(1, 7)  # [Ho, 7] input rows
    cols = torch.arange(Ho).view(Ho, 1) + torch.arange(4).view(1, 4)  # [Ho, 4] chunks
    # A[b, oh, ow, kh, q, e]
    A = xp[:, rows][:, :, :, cols]  # [B, Ho, 7, Ho, 4, 8]
    A = A.permute(0, 1, 3, 2, 4, 5).reshape(B, Ho, Ho, 224)
    got = torch.einsum("bhwk,nk->bnhw", A, wp)
    assert torch.allclose(got, ref, atol=1e-4, rtol=1e-4), (got - ref).abs().max()


def test_stem_pool_pooling_identity():
    """The fused epilogue computes relu(max(window) + bias) per channel and
    treats out-of-image taps as absent; for post-ReLU values that equals
    maxpool(relu(conv + bias)) with -inf padding (what torch does)."""
    g = torch.Generator().manual_seed(1)
    c = torch.randn(2, 64, 16, 16, generator=g)
    b = torch.randn(64, generator=g)
    ref = F.max_pool2d(F.relu(c + b.view(1, -1, 1, 1)), 3, 2, 1)
    # horizontal: max over (2pw-1, 2pw, 2pw+1) with the left pad excluded
    padded = F.pad(c, (1, 0), value=float("-inf"))
    h = torch.stack([padded[..., 0:-1:2], padded[..., 1::2], padded[..., 2::2]], 0).amax(0)
    h = F.relu(h + b.view(1, -1, 1, 1))
    # vertical with a zero row above (neutral for values >= 0)
    hv = F.pad(h, (0, 0, 1, 0), value=0.0)
    got = torch.stack([hv[:, :, 0:-1:2], hv[:, :, 1::2], hv[:, :, 2::2]], 0).amax(0)
    assert torch.equal(got, ref)
