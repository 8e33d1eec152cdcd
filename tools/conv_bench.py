#!/usr/bin/env python3
"""Per-layer conv microbenchmark on the GPU (ResNet18 / AlexNet shapes).

Times each distinct conv of the model in isolation, for every tile config,
and reports TFLOP/s. Every measurement replays a hipGraph of REP back-to-back
launches between two hipEvents (median of --iters replays / REP): timing
single Python-launched kernels between events measures the host launch path
(a ~40 us floor), not the kernel. Used for kernel A/B work and for rocprofv3
--pmc runs (one process, interleaved configs).
"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import dmlc  # noqa: E402
from dmlc import ops  # noqa: E402

RESNET18 = [
    # name, H, W, Cin, Cout, k, s, p, pair
    ("conv1", 230, 232, 3, 64, 7, 2, 3, True),  # packed stem image: 224+2*3 rows, 232-pixel rows
    ("l1", 56, 56, 64, 64, 3, 1, 1, False),
    ("l2.ds", 56, 56, 64, 128, 1, 2, 0, False),
    ("l2.c1", 56, 56, 64, 128, 3, 2, 1, False),
    ("l2", 28, 28, 128, 128, 3, 1, 1, False),
    ("l3.c1", 28, 28, 128, 256, 3, 2, 1, False),
    ("l3", 14, 14, 256, 256, 3, 1, 1, False),
    ("l4.c1", 14, 14, 256, 512, 3, 2, 1, False),
    ("l4", 7, 7, 512, 512, 3, 1, 1, False),
]


REP = 10


def warm_gpu(seconds=1.0):
    """Run bf16 GEMMs for ~seconds first: measurements taken right after start
    caught the clocks still ramping (the first variant timed read ~10-15%
    slow, whichever it was)."""
    import time
    a = torch.randn(8192, 8192, device="cuda").bfloat16()
    torch.cuda.synchronize()
    t0 = time.time()
    while time.time() - t0 < seconds:
        for _ in range(20):
            a @ a
        torch.cuda.synchronize()


def time_us(f, iters):
    """Median per-launch time (us) of f() replayed from a captured graph."""
    f()  # allocate workspaces / warm up outside the capture
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        f()
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            for _ in range(REP):
                f()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
        e0.record()
        g.replay()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3 / REP)
    return statistics.median(ts)


def _stamps():
    torch.cuda.synchronize()
    st = ops.BT_STAMPS.view(-1, 4).cpu()
    st = st[st[:, 3] > 0].double() / 100.0  # 100 MHz -> us
    ops.BT_STAMPS.zero_()
    if st.numel() == 0:
        return "no stamps"
    t0 = st[:, 0].min()
    q = lambda v: f"{v.median().item():.1f}/{v.max().item():.1f}"
    return (f"[stamps n={st.shape[0]} start {q(st[:, 0] - t0)} pro {q(st[:, 1] - st[:, 0])} "
            f"loop {q(st[:, 2] - st[:, 1])} epi {q(st[:, 3] - st[:, 2])} end {q(st[:, 3] - t0)}]")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--tiles", default="-1,0,1,2,3,4,5,6")
    ap.add_argument("--only", default="")
    ap.add_argument("--persist", type=int, default=0, help="persistent grid size (0 = one block per tile)")
    ap.add_argument("--split", type=int, default=1, help="split-K factor (big-tile configs 11/12: K slices, 1 = auto)")
    ap.add_argument("--variants", default="0", help="register-weight stream conv variants to time (A/B hook)")
    ap.add_argument("--ref", action="store_true", help="also time hipBLASLt GEMM and MIOpen conv on each shape")
    ap.add_argument("--stamps", action="store_true", help="per-workgroup phase stamps of the stream convs")
    a = ap.parse_args()
    ops.set_phase_stamps(a.stamps)
    dev = torch.device("cuda", 0)
    B = a.batch
    tiles = [] if a.tiles == "none" else [int(t) for t in a.tiles.split(",")]
    warm_gpu()
    for name, H, W, Cin, Cout, k, s, p, pair in RESNET18:
        if a.only and name not in a.only.split(","):
            continue
        x = (torch.randn(B, H, W, Cin, device=dev) * 0.5).bfloat16()
        cin_real = 3 if pair else Cin
        w = torch.randn(Cout, cin_real, k, k) / (cin_real * k * k) ** 0.5
        wp = ops.pack_conv_weight(w, stem=pair, device=dev)
        bias = torch.zeros(Cout, device=dev)
        Ho = (H + 2 * (0 if pair else p) - k) // s + 1
        flops = 2.0 * B * Ho * Ho * Cout * cin_real * k * k
        row = []
        for t in tiles:
            if t in (2, 5) and Cout % 256:
                continue
            if t in (0, 2, 3, 5, 6, 8, 10) and Cout % 128:
                continue
            if (t == 11 and Cout % 256) or (t == 12 and Cout != 128) or (t == 13 and Cout % 128) or (t >= 11 and pair):
                continue
            try:
                f = lambda: ops.conv2d(x, wp, Cout, k, k, s, p, bias=bias, relu=True, tile=t, stem=pair,
                                       out_hw=(Ho, Ho) if pair else None, max_blocks=a.persist,
                                       split_k=(a.split if a.split != 1 else 0) if t in (11, 12) else a.split)
                us = time_us(f, a.iters)
                row.append(f"tile{t}={us:7.1f}us {flops/us/1e6:6.0f}TF")
            except Exception as e:  # noqa: BLE001
                row.append(f"tile{t}=ERR({e})")
        if name in ("l2", "l3", "l4", "l2.c1", "l3.c1", "l4.c1"):  # direct conv, streamed weights (conv3x3_stream.hip)
            for use_res in (False, True) if s == 1 else (False,):
                r = torch.randn(B, H, W, Cout, device=dev).bfloat16() if use_res else None
                f = lambda: ops.conv3x3_stream(x, wp, bias, r, True, stride=s)
                us = time_us(f, a.iters)
                row.append(f"stream{'+res' if use_res else ''}={us:7.1f}us {flops/us/1e6:6.0f}TF")
                if ops.BT_STAMPS is not None:
                    f()
                    row.append(_stamps())
                # register-weight kernels (fragment-order weights), per A/B variant
                nat = dmlc.native()
                if nat.conv3x3_stream_uses_frag(H, W, Cin, Cout, s) and s == 2:
                    # stride 2 as the engine runs it: with the fused downsample
                    wdp = ops.pack_conv_weight(torch.randn(Cout, Cin, 1, 1) / Cin ** 0.5, device=dev)
                    ds = (wdp, bias, ops.stream_weight_frag(wdp, Cout))
                    wf = ops.stream_weight_frag(wp, Cout)
                    for v in [int(t) for t in a.variants.split(",")]:
                        nat.conv3x3_stream_set_variant(v)
                        try:
                            f = lambda: ops.conv3x3_stream(x, wp, bias, None, True, stride=2, downsample=ds, frag=wf)
                            us = time_us(f, a.iters)
                            row.append(f"wr{v}+ds={us:7.1f}us {flops/us/1e6:6.0f}TF")
                            if ops.BT_STAMPS is not None:
                                f()
                                row.append(_stamps())
                        except Exception as e:  # noqa: BLE001
                            row.append(f"wr{v}=ERR({e})")
                        finally:
                            nat.conv3x3_stream_set_variant(0)
                if nat.conv3x3_stream_uses_frag(H, W, Cin, Cout, s) and s == 1:
                    for v in [int(t) for t in a.variants.split(",")]:
                        nat.conv3x3_stream_set_variant(v)
                        try:
                            wf = ops.stream_weight_frag(wp, Cout)
                            f = lambda: ops.conv3x3_stream(x, wp, bias, r, True, stride=s, frag=wf)
                            us = time_us(f, a.iters)
                            row.append(f"wr{v}{'+res' if use_res else ''}={us:7.1f}us {flops/us/1e6:6.0f}TF")
                            if ops.BT_STAMPS is not None:
                                f()
                                row.append(_stamps())
                        except Exception as e:  # noqa: BLE001
                            row.append(f"wr{v}=ERR({e})")
                        finally:
                            nat.conv3x3_stream_set_variant(0)
        if name == "l1":  # direct row-streaming conv (conv3x3_rows.hip)
            for use_res in (False, True):
                r = torch.randn(B, H, W, Cout, device=dev).bfloat16() if use_res else None
                f = lambda: ops.conv3x3_rows(x, wp, bias, r, True)
                us = time_us(f, a.iters)
                row.append(f"rows{'+res' if use_res else ''}={us:7.1f}us {flops/us/1e6:6.0f}TF")
        if a.ref:
            # vendor references on the same shape: plain GEMM (hipBLASLt via
            # torch.mm) and MIOpen conv (bf16, channels_last)
            M, K = B * Ho * Ho, cin_real * k * k
            A = torch.randn(M, K, device=dev).bfloat16()
            Bm = torch.randn(K, Cout, device=dev).bfloat16()
            xc = torch.randn(B, cin_real, H - (2 * p if pair else 0), W - (2 * p if pair else 0),
                             device=dev).bfloat16().to(memory_format=torch.channels_last)
            wc = torch.randn(Cout, cin_real, k, k, device=dev).bfloat16().to(memory_format=torch.channels_last)
            for tag, f in (("gemm", lambda: torch.mm(A, Bm)),
                           ("miopen", lambda: torch.nn.functional.conv2d(xc, wc, None, s, p))):
                us = time_us(f, a.iters)
                row.append(f"{tag}={us:7.1f}us {flops/us/1e6:6.0f}TF")
        print(f"{name:6s} M={B*Ho*Ho:8d} N={Cout:4d} K={cin_real*k*k:5d}  " + "  ".join(row), flush=True)


if __name__ == "__main__":
    main()
