#!/usr/bin/env python3
"""Where does the DP step loop lose time against a bare two-lane loop?
Two B=256 ResNet18 engines alternate on two streams (graph replay), plus:
  raw      nothing else
  sync1    the host waits for step i-1 before issuing step i+1 (the
           pipeline's collect depth)
  d2h      + each step's answers copied to pinned host on a third stream
  runner   the native DpRunner (bench.py's loop, lanes=2, default slots)
Images/s over --iters steps, same process, same box."""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=400)
    ap.add_argument("--modes", default="raw,sync1,d2h,runner,raw")
    a = ap.parse_args()
    import dmlc
    from dmlc.models import build, state_dict_f32
    from dmlc.runtime import InferenceEngine
    C = dmlc.native()
    dev = torch.device("cuda", 0)
    sd = state_dict_f32(build("resnet18", seed=0))
    B = 256
    pool = torch.randint(0, 256, (2 * B, 224, 224, 3), dtype=torch.uint8, device=dev)
    engs = [InferenceEngine("resnet18", sd, device=0, max_batch=B) for _ in range(2)]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    side = torch.cuda.Stream(priority=-1)
    outs = [(torch.empty(B, dtype=torch.int32, device=dev), torch.empty(B, dtype=torch.float32, device=dev))
            for _ in range(2)]
    host = [torch.empty(B, dtype=torch.int32).pin_memory() for _ in range(2)]
    runner = C.DpRunner(engs[0]._e, 1, 0, b"", b"", B, scatter=False, lanes=2)

    def loop(mode, n):
        evs = []
        for i in range(n):
            k = i % 2
            with torch.cuda.stream(streams[k]):
                engs[k].predict(pool[k * B:(k + 1) * B], out=outs[k])
                ev = torch.cuda.Event()
                ev.record()
            if mode == "d2h":
                side.wait_event(ev)
                with torch.cuda.stream(side):
                    host[k].copy_(outs[k][0], non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record()
            evs.append(ev)
            if mode in ("sync1", "d2h") and i >= 1:
                evs[i - 1].synchronize()

    for mode in a.modes.split(","):
        if mode == "runner":
            runner.run(pool.data_ptr(), 2 * B, 0, 20)
            runner.sync()
            t = time.perf_counter()
            runner.run(pool.data_ptr(), 2 * B, 20, a.iters)
            runner.sync()
        else:
            loop(mode, 20)
            torch.cuda.synchronize()
            t = time.perf_counter()
            loop(mode, a.iters)
            torch.cuda.synchronize()
        dt = time.perf_counter() - t
        print(f"{mode:7s} {B * a.iters / dt:10,.0f} img/s  {dt / a.iters * 1e3:.4f} ms/step", flush=True)


if __name__ == "__main__":
    main()
