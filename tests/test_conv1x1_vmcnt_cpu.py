"""conv1x1.hip's explicit vmcnt waits, checked against a model of the kernel's
issue order (CPU).

The weight-stationary 1x1 conv issues its LDS-DMA, residual loads and stores
as operations the compiler does not track, and waits for them with counted
`s_waitcnt vmcnt(N)`: vmcnt retires in issue order, so an operation has
completed once at least N operations were issued after it. The thresholds come
from one constexpr plan (`c1_plan`, exported as `conv1x1_plan`) that the kernel
instantiates as template constants. This test replays one wave's issue order
(prologue, then per block: residual loads, DMA, [the chained reduce's stores of
the previous block], wait, MFMAs, residual wait, stores) for every kernel form
and checks that each wait covers what the code after it reads (safety) and, in
the steady state, no more (tightness: a wait that drains extra operations
stalls the pipeline it exists to keep full).
"""
import pytest

import dmlc

C = dmlc.native()


def forms():
    """(in8, out8, rb, nw, res, wv, ch) of every launchable conv1x1 form."""
    out = []
    for in8, out8, res in [(False, False, False), (False, False, True), (True, False, False), (False, True, False),
                           (False, True, True), (True, True, False), (True, True, True)]:
        for rb in (128, 256, 512, 1024):
            for wv in (4, 8):
                for nw in (64, 32, 16):
                    fits = nw * rb <= 16384 or (wv == 8 and not in8 and rb == 1024 and nw == 32)
                    if fits:
                        out.append((in8, out8, rb, nw, res, wv, False))
    out.append((True, True, 128, 64, True, 8, True))  # conv1x1_chain
    return out


def replay(p, res, ch, nblocks):
    """One wave's vector-memory operations in issue order: a list of tags, and
    the wait points as (threshold, [tags that must have completed], steady,
    number of operations issued before the wait)."""
    S, dt, rt, st, st2, pre = p["s"], p["dt"], p["rt"], p["st"], p["st2"], p["pre"]
    ops, waits = [], []

    def issue(tag, n):
        ops.extend([tag] * n)

    if pre:
        issue(("res", 0), rt)
    for s in range(S - 1):
        issue(("dma", s), dt)
    for it in range(nblocks):
        if pre:
            issue(("res", it + 1), rt)
        elif res:
            issue(("res", it), rt)
        issue(("dma", it + S - 1), dt)
        if ch and it > 0:
            issue(("st2", it - 1), st2)
        # the block's rows (prologue blocks: and, PRE, the residual loaded before them)
        if it < S - 1:
            n = p["pro_wait_ch"] if ch and it > 0 else p["pro_wait"]
            need = [("dma", it)] + ([("res", it)] if pre else [])
            waits.append((n, need, False, len(ops)))
        elif ch and it == S - 1:
            waits.append((p["n1_first"], [("dma", it)], True, len(ops)))
        else:
            waits.append((p["n1"], [("dma", it)], True, len(ops)))
        if res and (not pre or it >= S - 1):
            waits.append((p["res_wait"], [("res", it)], True, len(ops)))
        issue(("st", it), st - st2)
    return ops, waits


@pytest.mark.parametrize("form", forms())
def test_conv1x1_vmcnt_plan(form):
    in8, out8, rb, nw, res, wv, ch = form
    S = 3 if rb <= 256 else 2
    p = C.conv1x1_plan(in8, out8, rb, nw, res, S, wv, ch)
    assert p["s"] == S and p["dt"] >= 1
    nf = nw // 16
    ng = nf // 4 if (out8 and nf >= 4) else nf // 2 if nf >= 2 else 1  # channel groups per lane
    assert p["st"] == (64 if rb <= 512 else 32) // 16 * ng + p["st2"]  # one store per pixel fragment and group
    for k in ("n1", "n1_first", "pro_wait", "pro_wait_ch", "res_wait"):
        assert 0 <= p[k] < 64, (k, p)  # s_waitcnt vmcnt range
    ops, waits = replay(p, res, ch, nblocks=9)
    for n, need, steady, at in waits:
        issued = ops[:at]
        for tag in need:
            last = max(i for i, t in enumerate(issued) if t == tag)
            after = len(issued) - 1 - last
            assert after >= n, (form, tag, n, after)  # the wait covers it
            if steady:
                assert after == n, (form, tag, n, after)  # and drains nothing newer


def test_conv1x1_chain_plan_counts():
    """The chained form's extra stores: one 4-B reduce store per pixel
    fragment per block, issued with the next block, folded into every count."""
    p = C.conv1x1_plan(True, True, 128, 64, True, 3, 8, True)
    q = C.conv1x1_plan(True, True, 128, 64, True, 3, 8, False)
    assert p["st2"] == 4 and q["st2"] == 0
    assert p["st"] == q["st"] + 4
    assert p["n1"] == q["n1"] + 3 * 4  # (S - 1) blocks of reduce stores + the previous block's
    assert p["res_wait"] == q["res_wait"] + 2 * 4
