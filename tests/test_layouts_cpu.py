"""CPU checks of the operand layouts the HIP kernels assume (no GPU needed).

Each test rebuilds, in plain PyTorch, the exact reads a kernel performs on a
packed layout and checks that they reproduce the fp32 torch op. A layout bug
then fails here, on the CPU, before any kernel runs.
"""
import pytest
import torch
import torch.nn.functional as F

import dmlc
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


# ds_read_b128 is serviced in four 16-lane groups (MI355X_MICROARCH.md §LDS);
# a group is conflict-free when its distinct 16-B addresses hit distinct banks.
_B128_GROUPS = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
                list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
_B128_GROUPS += [[l + 32 for l in g] for g in _B128_GROUPS]


def _b128_ways(addr):
    worst = 1
    for grp in _B128_GROUPS:
        banks = {}
        for l in grp:
            for b in range(addr[l] // 4, addr[l] // 4 + 4):
                banks.setdefault(b % 64, set()).add(addr[l])
        worst = max(worst, max(len(v) for v in banks.values()))
    return worst


def test_row_conv_lds_reads_conflict_free():
    """conv3x3_rows.hip: input fragment (16 pixels x 8 channels, chunk
    swizzle q & 7) and weight fragment (16 channels x 8 k, swizzle
    2*((n>>3)&1)) reads are bank-conflict free for every fragment, tap and
    channel half the kernel issues."""
    W, C, R = 56, 64, 4
    for wm in range(2):
        for f in range(R * W // 32):
            for kw in range(3):
                for h in range(2):
                    addr = []
                    for l in range(64):
                        fr, g = l & 15, l >> 4
                        p = wm * (R * W // 2) + 16 * f + fr
                        q = p % W + kw
                        addr.append((p // W) * (W + 2) * C * 2 + q * C * 2 + (((4 * h + g) ^ (q & 7)) << 4))
                    assert _b128_ways(addr) == 1, (wm, f, kw, h)
    for wn in range(2):
        for nf in range(2):
            addr = []
            for l in range(64):
                fr, g = l & 15, l >> 4
                n = wn * 32 + nf * 16 + fr
                addr.append(n * 64 + ((g ^ (((n >> 3) & 1) << 1)) << 4))
            assert _b128_ways(addr) == 1, (wn, nf)


def test_block_conv_lds_layout_conflict_free():
    """conv3x3_block.hip: staged rows split by K half ([h][q][4 chunks],
    chunk c of column q holding channels 8*(4h + (c ^ ((q >> 1) & 3)))):
    the input-fragment reads of both halves (h = 1 at a fixed +3712 B) and
    the producers' ds_write_b128 of the intermediate are conflict free; the
    DMA staging order covers every in-image (h, q, chunk) exactly once."""
    W, R, Q = 56, 4, 58
    half = Q * 64
    slot = 2 * half
    assert slot % 256 == 0
    for wm in range(2):
        for f in range(R * W // 32):
            for kw in range(3):
                for h in range(2):
                    addr = []
                    for l in range(64):
                        fr, g = l & 15, l >> 4
                        p = wm * (R * W // 2) + 16 * f + fr
                        q = p % W + kw
                        addr.append((p // W) * slot + h * half + q * 64 + ((g ^ ((q >> 1) & 3)) << 4))
                    assert _b128_ways(addr) == 1, (wm, f, kw, h)
            for wn in range(2):  # epilogue store of t: channels wn*32 + 8g .. +7 of pixel p
                addr = []
                for l in range(64):
                    fr, g = l & 15, l >> 4
                    p = wm * (R * W // 2) + 16 * f + fr
                    q = p % W + 1
                    addr.append((p // W) * slot + wn * half + q * 64 + ((g ^ ((q >> 1) & 3)) << 4))
                assert _b128_ways(addr) == 1, (wm, f, wn)
    seen, dst = set(), set()
    for h in range(2):  # load_row: chunk k of K half h's run (q = 1..56) -> LDS chunk, source channel group
        for k in range(4 * W):
            q, c = 1 + k // 4, k % 4
            dst.add(h * half // 16 + 4 + k)
            seen.add((q, 4 * h + (c ^ ((q >> 1) & 3))))
    assert seen == {(q, cg) for q in range(1, W + 1) for cg in range(8)}
    # never DMA'd (zeroed at kernel start): the pad columns q = 0, 57 of both halves
    assert {i for i in range(slot // 16) if i not in dst} == {h * half // 16 + j for h in range(2)
                                                               for j in (0, 1, 2, 3, 228, 229, 230, 231)}


def test_stem_pool_lds_reads_conflict_free():
    """stem_pool.hip: lane (fr, g) of fragment f reads pair chunk
    16f + fr + g of a staged row; overlapping windows broadcast."""
    for f in range(8):
        addr = [(16 * f + (l & 15) + (l >> 4)) * 16 for l in range(64)]
        assert _b128_ways(addr) == 1


def test_stream_weight_frag_layout_matches_native_index():
    """ops.stream_weight_frag (used by the kernel tests) and the engine's
    stream_frag_index (C++, kernels.h) describe the same permutation: every
    (channel, k) lands in the lane / element the WR stream conv reads."""
    import torch
    from dmlc import ops
    cout, K = 64, 96
    w = torch.arange(cout * K, dtype=torch.float32).view(cout, K)
    f = ops.stream_weight_frag(w).reshape(-1)

    def perm32(n):
        return 8 * ((n & 15) >> 2) + 4 * (n >> 4) + (n & 3)

    for g in range(cout // 32):
        for t in range(K // 32):
            for nf in range(2):
                for lane in range(64):
                    for e in range(8):
                        idx = ((((g * (K // 32) + t) * 2 + nf) * 64 + lane) * 8) + e
                        n = 32 * g + perm32(16 * nf + (lane & 15))
                        k = 32 * t + 8 * (lane >> 4) + e
                        assert f[idx] == w[n, k]


@pytest.mark.parametrize("rb,fp8", [(128, False), (128, True), (256, False), (256, True), (512, False),
                                    (512, True), (1024, False), (1024, True)])
def test_conv1x1_lds_conflict_free(rb, fp8):
    """conv1x1.hip: staged pixel rows of rb bytes, 16-B chunk c of pixel p at
    physical chunk c ^ swz(p); the B-fragment reads (bf16: chunk 4ks + g of
    pixel 16pf + fr; e4m3: chunks 8ks + 2g and 8ks + 2g + 1) are conflict free
    for every pixel fragment and K step, and the DMA staging order covers
    every (pixel, chunk) once."""
    cpr = rb // 16
    bm = 64 if rb <= 512 else 32

    def swz(p):
        if rb == 128:
            return ((((p & 7) << 1) | ((p >> 3) & 1)) & 7) if fp8 else (p & 7)
        return p & 15

    ks_n = cpr // 8 if fp8 else cpr // 4
    for pf in range(bm // 16):
        for ks in range(ks_n):
            for half in ((0, 1) if fp8 else (0,)):
                addr = []
                for l in range(64):
                    fr, g = l & 15, l >> 4
                    p = 16 * pf + fr
                    c = 8 * ks + 2 * g + half if fp8 else 4 * ks + g
                    addr.append(p * rb + ((c ^ swz(p)) << 4))
                assert _b128_ways(addr) == 1, (pf, ks, half)
    seen = set()
    for i in range(bm * cpr):
        p, pc = i // cpr, i % cpr
        seen.add((p, pc ^ swz(p)))
    assert seen == {(p, c) for p in range(bm) for c in range(cpr)}


def _s2rows_pos(x):
    """conv3x3_s2rows.hip staged-row slot of input column x (-1: the pad)."""
    return 0 if x == -1 else ((x + 1) // 2 if x & 1 else 29 + x // 2)


def _s2rows_swz(y, x):
    return ((((y + 1) >> 1) * 28 + ((x + 1) >> 1)) >> 1) & 3


def test_s2rows_lds_layout():
    """conv3x3_s2rows.hip: every ds_read_b128 of a 112-pixel step (7
    fragments x 9 taps x 2 K halves, all 7 steps, through the 17-row ring
    with its 2 guard slots) is conflict free and reads the channels the
    weight fragment expects; the DMA staging order of a row covers every
    (column, channel chunk) once."""
    RB, HALF, RING = 7424, 3712, 17
    # ring contents as (row) per slot, guard slots 17/18 mirroring 0/1
    for r0 in range(0, 28, 4):
        sb = (2 * r0) % RING
        for f in range(7):
            for kh in range(3):
                for kw in range(3):
                    for h in range(2):
                        addr = []
                        for l in range(64):
                            fr, g = l & 15, l >> 4
                            p = 16 * f + fr
                            r, c = r0 + p // 28, p % 28
                            y, x = 2 * r + kh - 1, 2 * c + kw - 1
                            sl = sb + 2 * (p // 28)
                            sl = sl - RING if sl >= RING else sl
                            # kernel: rowoff + col[v] + immediate
                            v = (kw == 2) + 2 * (kh == 2)
                            s = ((p + (v & 1) + 28 * (v >> 1)) >> 1) & 3
                            col = (c + (v & 1)) * 64 + ((g ^ s) << 4)
                            a = sl * RB + col + kh * RB + (29 * 64 if kw == 1 else 0) + h * HALF
                            addr.append(a)
                            # the slot holds row y (mod the ring, guards mirror slots 0/1)
                            slot = a // RB
                            assert (slot % RING) == (y + 1) % RING and slot < RING + 2
                            off = a % RB
                            hh, j = off // HALF, off % HALF
                            assert hh == h and j // 64 == _s2rows_pos(x)
                            # stored chunk holds logical chunk 4h + (phys ^ swz(y, x)) == 4h + g
                            assert ((j % 64) // 16) ^ _s2rows_swz(y, x) == g
                        assert _b128_ways(addr) == 1, (r0, f, kh, kw, h)
    seen, dst = set(), set()
    for h in range(2):  # load_row: chunk k of K-half h's run -> LDS chunk, source column / channel chunk
        for k in range(224):
            pos, c = 1 + k // 4, k % 4
            x = 2 * pos - 1 if pos < 29 else 2 * (pos - 29)
            assert _s2rows_pos(x) == pos
            dst.add(h * HALF // 16 + 4 + k)
            seen.add((x, 4 * h + (c ^ _s2rows_swz(0, x))))
    assert seen == {(x, cc) for x in range(56) for cc in range(8)}
    # the chunks never DMA'd (pad slot 0 and spare slot 57 of each plane) stay zero
    assert {i for i in range(RB // 16) if i not in dst} == {h * HALF // 16 + j for h in range(2) for j in (0, 1, 2, 3, 228, 229, 230, 231)}


def test_s2rows128_lds_layout():
    """conv3x3_s2rows128.hip (ResNet50 layer2.0.conv2): every ds_read_b128 of
    a 2-row step (4 fragments, the last 8 lanes clamped to pixel 55; 9 taps x
    4 channel quarters; all 14 steps through the 9-row ring and its 2 guard
    slots) is conflict free and reads the channels the weight fragment
    expects; the DMA order of a row covers every (column, channel chunk) once;
    the ring fits the LDS."""
    PLANE, RING = 57 * 64, 9
    RB = 4 * PLANE
    assert RB % 256 == 0 and (RING + 2) * RB <= 160 * 1024
    for r0 in range(0, 28, 2):
        sb = (2 * r0) % RING
        for f in range(4):
            for kh in range(3):
                for kw in range(3):
                    for q in range(4):
                        addr = []
                        for l in range(64):
                            fr, g = l & 15, l >> 4
                            p = min(16 * f + fr, 55)
                            r, c = r0 + p // 28, p % 28
                            y, x = 2 * r + kh - 1, 2 * c + kw - 1
                            sl = sb + 2 * (p // 28)
                            sl = sl - RING if sl >= RING else sl
                            v = (kw == 2) + 2 * (kh == 2)
                            s = ((p + (v & 1) + 28 * (v >> 1)) >> 1) & 3
                            col = (c + (v & 1)) * 64 + ((g ^ s) << 4)
                            a = sl * RB + col + kh * RB + (29 * 64 if kw == 1 else 0) + q * PLANE
                            addr.append(a)
                            slot = a // RB
                            assert slot < RING + 2
                            if y >= 0:
                                assert (slot % RING) == (y + 1) % RING
                            else:
                                assert slot == 0  # the zero row (step 0 only)
                            off = a % RB
                            qq, j = off // PLANE, off % PLANE
                            assert qq == q and j // 64 == _s2rows_pos(x)
                            assert ((j % 64) // 16) ^ _s2rows_swz(y, x) == g
                        assert _b128_ways(addr) == 1, (r0, f, kh, kw, q)
    # rows in use at a step (2 r0 - 1 .. 2 r0 + 3) and those DMA'd during it
    # (2 r0 + 4 .. 2 r0 + 7) occupy 9 distinct slots
    for r0 in range(0, 26, 2):
        assert len({(yy + 1) % RING for yy in range(2 * r0 - 1, 2 * r0 + 8)}) == 9
    seen = set()
    for q in range(4):
        for k in range(224):
            pos, c = 1 + k // 4, k % 4
            x = 2 * pos - 1 if pos < 29 else 2 * (pos - 29)
            seen.add((x, 4 * q + (c ^ _s2rows_swz(0, x))))
    assert seen == {(x, cc) for x in range(56) for cc in range(16)}


def test_rows28_lds_layout():
    """conv3x3_rows28.hip: every ds_read_b128 of a 112-pixel step (7
    fragments x 9 taps x 4 channel quarters, all 7 steps, through the
    10-row ring with its 2 guard slots) is conflict free and reads the
    channels its weight fragment expects; the per-wave DMA runs cover every
    (column, channel chunk) once and leave the pad slots alone."""
    RB, PLANE, RING = 7680, 1920, 10

    def swz(y, x):
        return ((28 * y + x) >> 1) & 3

    for r0 in range(0, 28, 4):
        for f in range(7):
            for kh in range(3):
                for kw in range(3):
                    for q in range(4):
                        addr = []
                        for l in range(64):
                            fr, g = l & 15, l >> 4
                            p = 16 * f + fr
                            y, x = r0 + p // 28 + kh - 1, p % 28 + kw - 1
                            sl = r0 % RING + p // 28
                            sl = sl - RING if sl >= RING else sl
                            s = ((p + kw - 1) >> 1) & 3
                            col = (p % 28 + kw) * 64 + ((g ^ s) << 4)
                            a = sl * RB + (col ^ (0 if kh == 1 else 32)) + kh * RB + q * PLANE
                            addr.append(a)
                            assert a // RB % RING == (y + 1) % RING and a // RB < RING + 2
                            off = a % RB
                            assert off // PLANE == q and (off % PLANE) // 64 == x + 1
                            if 0 <= x < 28:
                                assert ((off % 64) // 16) ^ swz(y, x) == g
                        assert _b128_ways(addr) == 1, (r0, f, kh, kw, q)
    seen, dst = set(), set()
    for wave in range(4):
        for k in range(112):
            x, c = k >> 2, k & 3
            dst.add(wave * PLANE // 16 + 4 + k)
            seen.add((x, 4 * wave + (c ^ swz(3, x))))
    assert seen == {(x, cc) for x in range(28) for cc in range(16)}
    assert {i for i in range(RB // 16) if i not in dst} == {w * PLANE // 16 + j for w in range(4)
                                                             for j in (0, 1, 2, 3, 116, 117, 118, 119)}
    # epilogue residual reads: chunk (4 wave + g) ^ fr of pixel 16 f + fr
    for f in range(7):
        for wave in range(4):
            addr = [(16 * f + (l & 15)) * 256 + (((4 * wave + (l >> 4)) ^ (l & 15)) << 4) for l in range(64)]
            assert _b128_ways(addr) == 1


def _permlane32_swap(a, b):
    """gfx950 v_permlane32_swap_b32 as measured on the GPU
    (tools/probes/permlane_probe.hip, profiles/r2_stem_permlane_ab.txt):
    [0] = rows (a0, a1, b0, b1), [1] = rows (a2, a3, b2, b3), 16-lane rows."""
    r = lambda v, i: v[16 * i:16 * i + 16]  # noqa: E731
    return r(a, 0) + r(a, 1) + r(b, 0) + r(b, 1), r(a, 2) + r(a, 3) + r(b, 2) + r(b, 3)


def _permlane16_swap(a, b):
    """v_permlane16_swap_b32, measured: [0] = rows (a0, b0, a2, b2), [1] = rows (a1, b1, a3, b3)."""
    r = lambda v, i: v[16 * i:16 * i + 16]  # noqa: E731
    return r(a, 0) + r(b, 0) + r(a, 2) + r(b, 2), r(a, 1) + r(b, 1) + r(a, 3) + r(b, 3)


def test_stem_row_rotation_from_permlane_swaps():
    """stem_pool.hip rot_rows_down1: lane l must receive lane (l - 16) mod 64's
    value (the pooling window's left neighbour column lives in the row group
    below). Emulates the two swaps with their measured semantics and the
    kernel's two lane selects."""
    x = list(range(64))
    p32 = _permlane32_swap(x, x)
    z = [p32[1][l] if l < 32 else p32[0][l] for l in range(64)]
    p16 = _permlane16_swap(z, x)
    y = [p16[0][l] if (l & 16) else p16[1][l] for l in range(64)]
    assert y == [(l - 16) % 64 for l in range(64)]


def _small_swz(q, ch):
    return (q & 15) if ch >= 16 else ((q >> 1) & 7)


@pytest.mark.parametrize("H,CI,S", [(56, 64, 1), (56, 64, 2), (28, 128, 1), (28, 128, 2), (14, 256, 1),
                                    (14, 256, 2), (7, 512, 1)])
@pytest.mark.parametrize("mf", [1, 2, 4])
def test_conv_small_lds_addressing(H, CI, S, mf):
    """conv_small.hip: every (pixel, tap, channel chunk) the K loop reads from
    the staged rows is the input chunk it needs (zero chunk for padding taps,
    the DMA's source permutation inverted). The ds_read_b128 fragment reads
    are at most 4-way bank conflicted (stride 2 puts the 16 pixels of a
    fragment 2 apart; a fragment that wraps an output row jumps): tolerated
    on this latency-bound query-batch path, where LDS is far from busy."""
    W = H
    CH, KPT = CI // 8, CI // 32
    Ho = (H - 1) // S + 1
    P = Ho * Ho
    tp = mf * 16
    worst = 1
    tiles = list(range(0, P, tp))
    for p0 in {tiles[0], tiles[len(tiles) // 2], tiles[-1]}:
        p1 = min(p0 + tp, P)
        oh_lo, oh_hi = p0 // Ho, (p1 - 1) // Ho
        ih_lo, ih_hi = max(0, oh_lo * S - 1), min(H - 1, oh_hi * S + 1)
        total = (ih_hi - ih_lo + 1) * W * CH
        # DMA: LDS slot s <- input chunk (row, col, c)
        staged = {}
        for s in range(total):
            q, cp = divmod(s, CH)
            staged[s] = (ih_lo + q // W, q % W, cp ^ _small_swz(q, CH))
        assert len(set(staged.values())) == total
        for t in range(9 * KPT):
            tap = t // KPT
            kh, kw = divmod(tap, 3)
            for f in range(mf):
                addr = []
                for l in range(64):
                    fr, fq = l & 15, l >> 4
                    c = (t % KPT) * 4 + fq
                    p = p0 + 16 * f + fr
                    oh, ow = divmod(p, Ho)
                    ih, iw = oh * S - 1 + kh, ow * S - 1 + kw
                    ok = p < p1 and 0 <= ih < H and 0 <= iw < W
                    if not ok:
                        addr.append(-16)  # the zero chunk
                        continue
                    q = (oh * S - 1 - ih_lo) * W + (ow * S - 1) + kh * W + kw
                    slot = q * CH + (c ^ _small_swz(q, CH))
                    assert staged[slot] == (ih, iw, c), (p0, t, f, l)
                    addr.append(slot * 16)
                real = [a for a in addr if a >= 0]
                if real:
                    worst = max(worst, _b128_ways([a if a >= 0 else real[0] for a in addr]))
    assert worst <= 4, worst


@pytest.mark.parametrize("H,CI,IMG", [(14, 256, 1), (7, 512, 2)])
def test_stream8_lds_layout(H, CI, IMG):
    """conv3x3_stream8.hip (e4m3 3x3): the staged image (logical chunk pair m
    of staged pixel q at physical pair m ^ (q & 7)) read back through the
    kernel's per-lane offsets reproduces every lane's 32 input channels in the
    weight packing's order (odd fq: second 16 first), and both 16-B reads of
    every X fragment are bank-conflict free for every tap and K-tile."""
    W, CPX = H, CI // 16
    npx = IMG * H * W
    torch.manual_seed(0)
    img = torch.randint(0, 256, (npx, CI), dtype=torch.uint8)
    lds = torch.zeros(npx * CI + CI, dtype=torch.uint8)  # + the zero pixel
    for q in range(npx):  # staging: physical chunk pc holds logical ((pc>>1) ^ (q&7)) << 1 | (pc&1)
        for pc in range(CPX):
            lc = (((pc >> 1) ^ (q & 7)) << 1) | (pc & 1)
            lds[q * CI + 16 * pc: q * CI + 16 * pc + 16] = img[q, 16 * lc: 16 * lc + 16]
    ZB = npx * CI
    nfrag = (npx + 15) // 16
    for tap in range(9):
        kh, kw = divmod(tap, 3)
        ktap = (kh - 1) * W + (kw - 1)
        for cc in range(CI // 128):
            for f in range(nfrag):
                a0, a1, want = [], [], []
                for lane in range(64):
                    fr, fq = lane & 15, lane >> 4
                    p = min(16 * f + fr, npx - 1)
                    ii, pi = divmod(p, H * W)
                    r, c = divmod(pi, W)
                    inside = 0 <= r + kh - 1 < H and 0 <= c + kw - 1 < W
                    xa = ((ii * H + r) * W + c) * CI + ktap * CI if inside else ZB
                    u = fq ^ ((fr + ktap) & 7)
                    tsw0 = (u << 5) | ((fq & 1) << 4)
                    a0.append(xa + (tsw0 ^ (cc << 7)))
                    a1.append(xa + ((tsw0 ^ 16) ^ (cc << 7)))
                    got = torch.cat([lds[a0[-1]:a0[-1] + 16], lds[a1[-1]:a1[-1] + 16]])
                    if inside and 16 * f + fr < npx:
                        q = p + ktap
                        ch = 128 * cc + 32 * fq
                        exp = img[q, ch:ch + 32]
                        if fq & 1:
                            exp = torch.cat([exp[16:], exp[:16]])
                        assert torch.equal(got, exp), (tap, cc, f, lane)
                    elif not inside:
                        assert not got.any()
                # conflicts among every real pixel's lanes, border lanes (zero
                # pixel, their own chunk offsets) included
                live = [l for l in range(64) if 16 * f + (l & 15) < npx]
                for addr in (a0, a1):
                    for grp in _B128_GROUPS:
                        slots = {}
                        for l in grp:
                            if l in live:
                                slots.setdefault((addr[l] // 16) % 16, set()).add(addr[l])
                        assert all(len(v) == 1 for v in slots.values()), (tap, cc, f)


@pytest.mark.parametrize("HS", [14])
def test_stream8_half_image_lds_layout(HS):
    """conv3x3_stream8.hip on ResNet50 layer2 (28x28x128, stride 1): a
    workgroup stages a strip of HS output rows plus its halo rows inside the
    image (rows rs = max(r0 - 1, 0) .. min(r0 + HS, 27)); 128-B pixels key chunk pair m of
    staged pixel K = i * W + x at m ^ ((K >> 1) & 3). The kernel's tap
    offsets (K = p + (r0 - rs) * W + ktap) read every lane's 32 channels
    (odd fq: second 16 first), zero-pixel taps read zeros, and both 16-B reads
    of every X fragment are bank-conflict free."""
    H = W = 28
    CI = 128
    CPX = CI // 16
    torch.manual_seed(2)
    img = torch.randint(1, 256, (H, W, CI), dtype=torch.uint8)
    for part in range(H // HS):
        r0 = part * HS
        rs = max(r0 - 1, 0)
        nrows = min(r0 + HS, H - 1) - rs + 1
        assert nrows <= HS + (2 if H // HS > 2 else 1)
        lds = torch.zeros(nrows * W * CI + 256, dtype=torch.uint8)  # + two zero pixels
        ZB = nrows * W * CI
        for i in range(nrows):
            for x in range(W):
                K = i * W + x
                for pc in range(CPX):
                    lc = (((pc >> 1) ^ ((K >> 1) & 3)) << 1) | (pc & 1)
                    o = (i * W + x) * CI + 16 * pc
                    lds[o:o + 16] = img[rs + i, x, 16 * lc:16 * lc + 16]
        npix = HS * W
        kb = (r0 - rs) * W
        for tap in range(9):
            kh, kw = divmod(tap, 3)
            ktap = (kh - 1) * W + (kw - 1)
            for f in range((npix + 15) // 16):
                a0, a1 = [], []
                for lane in range(64):
                    fr, fq = lane & 15, lane >> 4
                    p = min(16 * f + fr, npix - 1)
                    prow, pcol = divmod(p, W)
                    r = r0 + prow
                    inside = 0 <= r + kh - 1 < H and 0 <= pcol + kw - 1 < W
                    zh = (fr + kb + ktap) & 1  # the zero pixel in the window half of the lane's K parity
                    xa = ((r - rs) * W + pcol) * CI + ktap * CI if inside else ZB + 128 * zh
                    u = fq ^ (((fr + kb + ktap) >> 1) & 3)
                    t0 = (u << 5) | ((fq & 1) << 4)
                    a0.append(xa + t0)
                    a1.append(xa + (t0 ^ 16))
                    got = torch.cat([lds[a0[-1]:a0[-1] + 16], lds[a1[-1]:a1[-1] + 16]])
                    if inside and 16 * f + fr < npix:
                        exp = img[r + kh - 1, pcol + kw - 1, 32 * fq:32 * fq + 32]
                        if fq & 1:
                            exp = torch.cat([exp[16:], exp[:16]])
                        assert torch.equal(got, exp), (part, tap, f, lane)
                    elif not inside:
                        assert not got.any()
                live = [l for l in range(64) if 16 * f + (l & 15) < npix]  # border lanes included
                for addr in (a0, a1):
                    for grp in _B128_GROUPS:
                        slots = {}
                        for l in grp:
                            if l in live:
                                slots.setdefault((addr[l] // 16) % 16, set()).add(addr[l])
                        assert all(len(v) == 1 for v in slots.values()), (part, tap, f)


@pytest.mark.parametrize("H,CI,HS", [(14, 256, 7), (7, 512, 7), (28, 128, 4), (28, 128, 7)])
def test_stream8_stride2_lds_layout(H, CI, HS):
    """conv3x3_stream8.hip at stride 2 (ResNet50 layer2.0 / layer3.0 / layer4.0
    conv2): staged input rows with each row's even columns first, chunk pairs
    keyed by K = (((y + 1) >> 1) - r0) * W + ((x + 1) >> 1) (pair m at m ^ (K
    & 7), 128-B pixels m ^ ((K >> 1) & 3)); the kernel's tap offsets read
    every lane's 32 channels of input pixel (2r + kh - 1, 2c + kw - 1) (odd fq:
    second 16 first) and both reads are conflict free."""
    W = H
    HI, WI, CPX = 2 * H, 2 * W, CI // 16

    def pswz(k):
        return k & 7 if CPX >= 16 else (k >> 1) & 3
    torch.manual_seed(1)
    img = torch.randint(0, 256, (HI, WI, CI), dtype=torch.uint8)
    for part in range(H // HS):
        r0 = part * HS
        rs = max(2 * r0 - 1, 0)
        nrows = min(2 * (r0 + HS - 1) + 1, HI - 1) - rs + 1
        lds = torch.zeros(nrows * WI * CI + max(CI, 256), dtype=torch.uint8)  # + the zero pixel(s)
        ZB = nrows * WI * CI
        for i in range(nrows):
            y = rs + i
            for q in range(WI):
                x = 2 * q if q < WI // 2 else 2 * (q - WI // 2) + 1
                K = (((y + 1) >> 1) - r0) * W + ((x + 1) >> 1)
                for pc in range(CPX):
                    lc = (((pc >> 1) ^ pswz(K)) << 1) | (pc & 1)
                    o = (i * WI + q) * CI + 16 * pc
                    lds[o:o + 16] = img[y, x, 16 * lc:16 * lc + 16]
        npix = HS * W
        for tap in range(9):
            kh, kw = divmod(tap, 3)
            dq = WI // 2 - 1 if kw == 0 else (0 if kw == 1 else WI // 2)
            toff = ((kh - 1) * WI + dq) * CI
            ktap = (W if kh == 2 else 0) + (1 if kw == 2 else 0)
            for cc in range(CI // 128):
                for f in range((npix + 15) // 16):
                    a0, a1 = [], []
                    for lane in range(64):
                        fr, fq = lane & 15, lane >> 4
                        p = min(16 * f + fr, npix - 1)
                        prow, pcol = divmod(p, W)
                        r = r0 + prow
                        inside = not ((r == 0 and kh == 0) or (pcol == 0 and kw == 0))
                        # (128-B pixels: the zero pixel in the window half a real pixel of this
                        # K would use: K's parity, flipped for kw != 1)
                        zh = ((fr + ktap) & 1) ^ (1 if kw != 1 else 0) if CPX < 16 else 0
                        xa = ((2 * r - rs) * WI + pcol) * CI + toff if inside else ZB + 128 * zh
                        u = fq ^ pswz(fr + ktap)
                        t0 = (u << 5) | ((fq & 1) << 4)
                        a0.append(xa + (t0 ^ (cc << 7)))
                        a1.append(xa + ((t0 ^ 16) ^ (cc << 7)))
                        got = torch.cat([lds[a0[-1]:a0[-1] + 16], lds[a1[-1]:a1[-1] + 16]])
                        if inside and 16 * f + fr < npix:
                            ch = 128 * cc + 32 * fq
                            exp = img[2 * r + kh - 1, 2 * pcol + kw - 1, ch:ch + 32]
                            if fq & 1:
                                exp = torch.cat([exp[16:], exp[:16]])
                            assert torch.equal(got, exp), (part, tap, cc, f, lane)
                        elif not inside:
                            assert not got.any()
                    live = [l for l in range(64) if 16 * f + (l & 15) < npix]  # border lanes included
                    for addr in (a0, a1):
                        for grp in _B128_GROUPS:
                            slots = {}
                            for l in grp:
                                if l in live:
                                    slots.setdefault((addr[l] // 16) % 16, set()).add(addr[l])
                            assert all(len(v) == 1 for v in slots.values()), (part, tap, cc, f)


def _b32_store_ways(addr, groups=((0, 32), (32, 64))):
    """ds_write_b16/b32: two 32-lane groups, bank (a/4) mod 32; lanes on one
    dword (the two halves of a b16 pair) are one access."""
    worst = 1
    for lo, hi in groups:
        banks = {}
        for l in range(lo, hi):
            banks.setdefault((addr[l] // 4) % 32, set()).add(addr[l] // 4)
        worst = max(worst, max(len(v) for v in banks.values()))
    return worst


def test_stem_hpool_store_layout():
    """stem_pool.hip hpool_packed: lane (fr, g) of column fragment f stores
    channel 16n + fr of pooled columns 8f + 2g (low half) and 8f + 2g + 1
    (high half, +kHpCol) at hbase = g*2*kHpCol + (fr>>3)*16 + (fr&7)*2 plus
    the immediates f*8*kHpCol + n*32. Every (pooled column, channel) of a
    pooled conv row is written exactly once, at pw*kHpCol + 2c, which is
    where the vertical max reads 16-B channel chunks; no ds_write_b16 of the
    epilogue has two distinct dwords on one bank (4 row groups 288 B = 8
    banks apart)."""
    kHpCol, PW, NF, NB = 144, 56, 7, 4
    seen = {}
    for f in range(NF):
        for n in range(NB):
            for hi in range(2):
                addr = []
                for l in range(64):
                    fr, g = l & 15, l >> 4
                    a = g * 2 * kHpCol + (fr >> 3) * 16 + (fr & 7) * 2 + f * 8 * kHpCol + n * 32 + hi * kHpCol
                    pw, c = 8 * f + 2 * g + hi, 16 * n + fr
                    assert a == pw * kHpCol + 2 * c
                    assert (pw, c) not in seen
                    seen[(pw, c)] = a
                    addr.append(a)
                assert _b32_store_ways(addr) == 1, (f, n, hi)
    assert set(seen) == {(pw, c) for pw in range(PW) for c in range(64)}
    assert max(seen.values()) + 2 <= PW * kHpCol  # inside one pooled row


def test_stem_vertical_max_reads():
    """stem_pool.hip vertical 3-max (helper waves, 256 threads): item it ->
    pooled row pr = it >= per_row, column pw, channel chunk cg, 16-B reads at
    pw*kHpCol + cg*16 of three conv rows; the items of the two pooled rows
    cover every (pw, cg) once each, a wave never straddles the two rows, and
    the reads are 2-way bank conflicted (8 columns of 144 B per 16-lane
    group), pinned here: on the helper waves, off the MFMA waves' path
    (profiles/r4_stem_roles.txt: the helpers finish inside the MFMA phase)."""
    kHpCol, PW = 144, 56
    per_row = PW * 8
    assert per_row % 64 == 0
    items = set()
    worst = 1
    for j in range(4):
        for w in range(4):
            addr = []
            for l in range(64):
                it = w * 64 + l + j * 256
                if it >= 2 * per_row:
                    addr.append(None)
                    continue
                pr = it >= per_row
                rem = it - pr * per_row
                pw, cg = rem >> 3, rem & 7
                items.add((pr, pw, cg))
                addr.append(pw * kHpCol + cg * 16)
            live = [a for a in addr if a is not None]
            if live:
                worst = max(worst, _b128_ways([a if a is not None else live[0] for a in addr]))
    assert items == {(pr, pw, cg) for pr in range(2) for pw in range(PW) for cg in range(8)}
    assert worst == 2


def test_stem_convert_store_layout():
    """stem_pool.hip convert_rows (helpers): item it = (row, k) writes paired
    chunks 4k .. 4k+3 of its row (16 B each: pixels 8k-3+2q, 8k-2+2q as
    [r g b r g b 0 0]); every chunk of the rows converted is written exactly
    once and holds the pixel pair the MFMA waves' window reads (chunk p =
    padded pixels 2p, 2p+1, padded column = image column + 3). The
    ds_write_b128 stores are 4-way bank conflicted (64-B per-lane stride),
    pinned here: helper waves, 8 stores per item."""
    S = 224
    need = ((112 - 1) * 6 + 26) // 3
    Wr = ((max(S + 6, need)) + 7) // 8 * 8
    Wq = Wr // 2
    G4 = (Wq + 3) // 4
    RB = Wq * 16
    rows = 8
    written = {}
    for it in range(rows * G4):
        r, k = divmod(it, G4)
        for q in range(4):
            chunk = 4 * k + q
            if chunk >= Wq:
                continue
            assert (r, chunk) not in written
            # pixels of the chunk: ix = 8k - 3 + i for i = 2q, 2q + 1
            written[(r, chunk)] = (8 * k - 3 + 2 * q, 8 * k - 3 + 2 * q + 1)
    assert set(written) == {(r, c) for r in range(rows) for c in range(Wq)}
    for (r, c), (p0, p1) in written.items():
        assert (p0 + 3, p1 + 3) == (2 * c, 2 * c + 1)  # padded columns of pair chunk c
    worst = 1
    for t0 in range(0, rows * G4, 64):
        for q in range(4):
            addr = []
            for l in range(64):
                it = min(t0 + l, rows * G4 - 1)
                r, k = divmod(it, G4)
                addr.append((r % 13) * RB + (4 * k + q) * 16)
            banks = {}
            for grp in [list(range(i, i + 8)) for i in range(0, 64, 8)]:  # ds_write_b128: 8 x 8 contiguous
                for l in grp:
                    banks.setdefault((grp[0], (addr[l] // 4) % 32), set()).add(addr[l])
            worst = max(worst, max(len(v) for v in banks.values()))
    assert worst <= 4, worst


def _dense_rbs(RB):
    """stem_pool.hip dense ring slot stride: a multiple of 128 B with room for
    the odd rows' 64-B offset."""
    return (RB + 64 + 127) // 128 * 128


def _dense_stem_addr(fr, fq, j, RB=1392):
    """stem_pool.hip dense-K operand address of lane (fr, fq), dword slot j
    (= 4 s + i), fragment 0, with kernel row dy in ring slot dy (the ring only
    moves the slot bases by multiples of 128 B; conv row 0, so the absolute
    row's parity is dy's): slot dy * RBS, odd rows 64 B further, window dword
    u of output column fr at 12 fr + 4 u (kernels.h stem_dense_cell)."""
    dy, u, _ = ops.stem_dense_cell(j, fq)
    return dy * _dense_rbs(RB) + 64 * (dy & 1) + 12 * fr + 4 * u


@pytest.mark.parametrize("S", [128, 224, 256])
def test_stem_dense_layout(S):
    """Dense-K stem (stem_pool.hip stem_roles_kernel V & 2): the dense row
    holds padded pixel p (image column p - 3) channel c at element 3p + c;
    stem_dense_cell covers every (kernel row, window dword) exactly once plus
    3 zero-weight pads, every operand dword a lane reads is the pair of window
    elements its K slots name (elements 2u, 2u + 1 of output column ox's
    window starting at element 6 ox), inside the row, and the weight order
    (pack_stem_dense_weight, the engine's stem_dense_k_index) puts tap
    (dy, dx, c) at that K."""
    NF = S // 32
    NG = 4 * NF + 1
    RB = NG * 48
    RBS = _dense_rbs(RB)
    Wq = (((max(S + 6, ((S // 2 - 1) * 6 + 26) // 3)) + 7) // 8 * 8) // 2
    assert RBS <= Wq * 16  # the launcher's LDS budget (paired rows)
    Ho = S // 2
    assert NG * 8 >= S + 6
    cells = [ops.stem_dense_cell(j, fq) for j in range(20) for fq in range(4)]
    real = [(dy, u) for dy, u, pad in cells if not pad]
    assert sorted(real) == [(dy, u) for dy in range(7) for u in range(11)]
    assert sum(pad for _, _, pad in cells) == 3
    g = torch.Generator().manual_seed(3)
    w = torch.randn(64, 3, 7, 7, generator=g)
    wd = ops.pack_stem_dense_weight(w).float()
    wb = w.bfloat16().float()
    C = dmlc.native()
    seen = set()
    for k in range(160):
        s, fq, i, h = k // 32, (k % 32) // 8, (k % 8) // 2, k % 2
        dy, u, pad = ops.stem_dense_cell(4 * s + i, fq)
        e = 2 * u + h
        if pad or e == 21:
            assert wd[:, k].abs().max() == 0
            continue
        dx, c = e // 3, e % 3
        assert C.stem_dense_k_index(dy, dx, c) == k
        assert torch.equal(wd[:, k], wb[:, c, dy, dx])
        seen.add((dy, dx, c))
    assert len(seen) == 147
    for f in range(NF):
        for fr in range(16):
            ox = 16 * f + fr
            for fq in range(4):
                for j in range(20):
                    a = _dense_stem_addr(fr, fq, j, RB) + 192 * f
                    row, off = divmod(a, RBS)
                    off -= 64 * (row & 1)
                    dy, u, _ = ops.stem_dense_cell(j, fq)
                    assert 0 <= off and off + 4 <= RB and a % 4 == 0
                    assert row == dy and off // 2 == 6 * ox + 2 * u
    assert 6 * (Ho - 1) + 21 < 3 * (S + 6) <= NG * 24


def test_stem_dense_lds_conflicts():
    """Dense-K stem LDS traffic. The helpers' conversion stores (lane =
    8-pixel group g: three 16-B stores at 48 g + 16 q of its row; ds_write_b128,
    8-lane groups over 32 banks) are conflict free within a row and at most
    2-way in the groups that cross into an odd row (8 + 1 LDS-array cycles
    under the store's ~13-cycle data transfer: no cost). The MFMA waves' operand
    reads (ds_read_b32: lanes 0-31 and 32-63 each one LDS cycle over 32 banks,
    bank (a/4) mod 32) are conflict free in 18 of the 20 dword slots: each half
    pairs dword u of an even and an odd kernel row, 16 banks apart, against
    the 3 fr + u lane pattern; slots 18, 19 (row 6 against itself) are 2-way.
    The pooling epilogue (hpool_edge) stores, per lane (channel fr of block
    n, 4-column group G = 4 f + fq), pooled columns 2G, 2G + 1 into the hp
    row and relu(v3) into the edge row: together they cover every (pooled
    column, channel) and (group, channel) of a fragment once, at most 2-way
    per 32-lane half."""
    RB, RBS = 1392, _dense_rbs(1392)
    worst = 1
    for t0 in range(0, 8 * 29, 64):
        for q in range(3):
            addr = []
            for l in range(64):
                r, g = divmod(t0 + l, 29)
                addr.append((r % 21) * RBS + 64 * (r & 1) + 48 * g + 16 * q)
            worst = max(worst, _b128_ways(addr))
            for grp in [list(range(i, i + 8)) for i in range(0, 64, 8)]:  # 8-lane write groups, 32 banks
                banks = {}
                for l in grp:
                    for b in range(addr[l] // 4, addr[l] // 4 + 4):
                        banks.setdefault(b % 32, set()).add(addr[l])
                worst = max(worst, max(len(v) for v in banks.values()))
    assert worst <= 2
    ways = []
    for j in range(20):
        w = 1
        for half in (range(0, 32), range(32, 64)):
            banks = {}
            for l in half:
                a = _dense_stem_addr(l & 15, l >> 4, j, RB) + 192 * 3
                banks.setdefault((a // 4) % 32, set()).add(a)
            w = max(w, max(len(v) for v in banks.values()))
        ways.append(w)
    assert ways[:18] == [1] * 18, ways
    assert ways[18:] == [2, 2], ways
    kHpCol = 144
    hcov, ecov = set(), set()
    for half in (range(0, 32), range(32, 64)):
        hb, eb = {}, {}
        for l in half:
            fr, fq = l & 15, l >> 4
            h = fq * 2 * kHpCol + (fr >> 3) * 16 + (fr & 7) * 2  # lo16 at h, hi16 at h + kHpCol
            e = fq * kHpCol + (fr >> 3) * 16 + (fr & 7) * 2
            for a in (h, h + kHpCol):
                hcov.add(divmod(a, kHpCol))
                hb.setdefault((a // 4) % 32, set()).add(a // 4)
            ecov.add(divmod(e, kHpCol))
            eb.setdefault((e // 4) % 32, set()).add(e // 4)
        assert max(len(v) for v in hb.values()) <= 2 and max(len(v) for v in eb.values()) <= 2
    assert hcov == {(col, 2 * c) for col in range(8) for c in range(16)}
    assert ecov == {(g, 2 * c) for g in range(4) for c in range(16)}


@pytest.mark.parametrize("C,ipw", [(512, 4), (512, 16), (2048, 16), (2048, 4)])
def test_head_lds_layout(C, ipw):
    """head.hip: pooled rows at a (C + 16)-element stride; the fc's B-operand
    read (lane: image col = lane & 15, 16-B chunk kq = lane >> 4, K offset k)
    is conflict free for every K step with 4 live images (head_fused) and 16
    (head_pooled); the logits store (one 16-B chunk per lane at col*lgs +
    16tt + 4kq, lgs = nsplit + 4) is conflict free in its 8-lane groups and
    the per-image softmax reads (consecutive classes) cover each image's
    split exactly."""
    ldp = C + 16
    for k in range(0, C, 32):
        addr = []
        for l in range(64):
            col, kq = l & 15, l >> 4
            addr.append(col * ldp * 2 + kq * 16 + 2 * k if col < ipw else None)
        live = [a for a in addr if a is not None]
        assert _b128_ways([a if a is not None else live[0] for a in addr]) == 1, k
    for nsplit in (64, 128, 256, 1008):
        lgs = nsplit + 4
        for tt in range(0, nsplit // 16):
            addr = [(l & 15) * lgs * 4 + (tt * 16 + (l >> 4) * 4) * 4 for l in range(64)]
            for g0 in range(0, 64, 8):  # ds_write_b128: 8 x 8 contiguous, bank (a/4) mod 32
                banks = {}
                for l in range(g0, g0 + 8):
                    if (l & 15) >= ipw:
                        continue
                    for d in range(4):
                        banks.setdefault((addr[l] // 4 + d) % 32, set()).add(addr[l])
                assert max((len(v) for v in banks.values()), default=1) == 1, (nsplit, tt, g0)
        slots = {(l & 15, tt * 16 + (l >> 4) * 4 + r) for tt in range(nsplit // 16) for l in range(64) for r in range(4)}
        assert slots == {(c, n) for c in range(16) for n in range(nsplit)}


@pytest.mark.parametrize("in8", [False, True])
def test_igemm_fragment_reads_conflict_free(in8):
    """conv_igemm.hip: 128-B LDS rows, physical chunk = logical ^ h(row) with
    h = (row >> 1) & 7 (bf16: lane (fr, fq) reads chunk 4 ks + fq of row fr)
    or (row >> 1) & 5 (e4m3: chunks 2 fq and 2 fq + 1, two reads); every
    ds_read_b128 of a 16-row fragment is bank-conflict free (the e4m3 tiles
    with the bf16 swizzle were 2-way: 45.7% conflict cycles measured)."""
    h = (lambda r: (r >> 1) & 5) if in8 else (lambda r: (r >> 1) & 7)
    reads = [(lambda fq, s=s: 2 * fq + s) for s in range(2)] if in8 else \
        [(lambda fq, ks=ks: 4 * ks + fq) for ks in range(2)]
    for base in (0, 16, 32, 48):  # fragments start at 16-row multiples
        for rd in reads:
            addr = []
            for l in range(64):
                fr, fq = l & 15, l >> 4
                r = base + fr
                addr.append(r * 128 + ((rd(fq) ^ h(r)) << 4))
            assert _b128_ways(addr) == 1, (base, in8)
