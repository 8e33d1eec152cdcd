"""Data-parallel batch inference across the GPUs of a node (one process per
GPU, RCCL over xGMI through torch.distributed's "nccl" backend).

Reference counterpart: the leader's `run_job` fans single-image queries out
to a random member over TCP (src/services.rs:407-433, 2 queries/s/job) and
every member holds full model replicas (src/services.rs:513-524). Here the
coordinator (rank 0) holds the staged u8 image pool in HBM and, per step:

  1. sends one u8 shard [B,224,224,3] to every other rank (one batch of RCCL
     point-to-point sends, one xGMI link per peer; the u8 layout is 2x
     smaller than bf16 and is normalised on the receiving GPU) and reads its
     own shard in place,
  2. every rank classifies its shard (hipGraph-replayed HIP engine),
  3. (top-1 class, probability) pairs come back to rank 0 as point-to-point
     receives (8 bytes per image).
DMLC_DP_P2P=0 selects dist.scatter / dist.gather instead.

The scatter of step i+1 is issued before the compute of step i and lands in
the other input slot, so the xGMI transfer overlaps compute; RCCL runs on
its own stream and torch.distributed orders it against the compute stream
with events. Works with "gloo" + CPU tensors too (used by the CPU tests).
"""
from __future__ import annotations

import os
import time
from typing import Callable

import torch
import torch.distributed as dist

PredictFn = Callable[[torch.Tensor, tuple], None]  # (images u8 [B,H,W,3], (idx_out, prob_out))


class _Range:
    """roctx range (torch.cuda.nvtx maps to roctx on ROCm); no-op on CPU."""

    def __init__(self, name: str, on: bool):
        self.name, self.on = name, on

    def __enter__(self):
        if self.on:
            torch.cuda.nvtx.range_push(self.name)

    def __exit__(self, *exc):
        if self.on:
            torch.cuda.nvtx.range_pop()


class _Works:
    """wait() on a batch of point-to-point works (one handle, like async_op)."""

    def __init__(self, works):
        self.works = works or []

    def wait(self):
        for w in self.works:
            w.wait()


class DPInference:
    def __init__(self, predict_fn: PredictFn, per_rank_batch: int, device: torch.device,
                 image_shape=(224, 224, 3), src: int = 0, slots: int = 2, input_mode: str = "scatter"):
        self.predict_fn = predict_fn
        self.B = per_rank_batch
        self.device = device
        self.src = src
        self.slots = slots
        self.input_mode = input_mode
        self.distributed = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size() if self.distributed else 1
        self.rank = dist.get_rank() if self.distributed else 0
        self.cuda = device.type == "cuda"
        H, W, C = image_shape
        self.inbuf = [torch.empty(self.B, H, W, C, dtype=torch.uint8, device=device) for _ in range(slots)]
        self.outbuf = [torch.empty(2, self.B, dtype=torch.int32, device=device) for _ in range(slots)]
        self.gathered = [[torch.empty(2, self.B, dtype=torch.int32, device=device) for _ in range(self.world)]
                         if self.rank == src else None for _ in range(slots)]
        self.transfer = self.distributed and input_mode == "scatter"
        # point-to-point form (default): the coordinator sends only the other
        # ranks' shards and reads its own straight from the pool, and receives
        # only the other ranks' answers; dist.scatter/gather would also copy
        # the coordinator's own 38.5 MB shard, on its compute stream, every
        # step (measured ~55 us per step with the stream joins: DMLC_DP_P2P=0)
        self.p2p = self.distributed and os.environ.get("DMLC_DP_P2P", "1") != "0"
        self.t_start: dict[int, object] = {}
        self.t_end: dict[int, object] = {}

    # ---------------------------------------------------------------- helpers
    def shards(self, pool: torch.Tensor, step: int) -> list[torch.Tensor]:
        """Per-rank u8 shards of global batch `step` from the staged pool."""
        gb = self.B * self.world
        n_batches = pool.shape[0] // gb
        base = (step % n_batches) * gb
        return [pool[base + r * self.B: base + (r + 1) * self.B] for r in range(self.world)]

    def _stamp(self, store: dict, step: int) -> None:
        if self.cuda:
            e = torch.cuda.Event(enable_timing=True)
            e.record(torch.cuda.current_stream(self.device))
            store[step] = e
        else:
            store[step] = time.perf_counter()

    def latency_ms(self, step: int) -> float:
        a, b = self.t_start[step], self.t_end[step]
        if self.cuda:
            return a.elapsed_time(b)
        return (b - a) * 1e3

    def _issue_input(self, pool, step):
        if not self.transfer:
            return None
        s = step % self.slots
        shards = self.shards(pool, step) if self.rank == self.src else None
        with _Range("dp.scatter", self.cuda):
            if not self.p2p:
                return dist.scatter(self.inbuf[s], shards, src=self.src, async_op=True)
            if self.rank == self.src:
                ops = [dist.P2POp(dist.isend, shards[r], r) for r in range(self.world) if r != self.src]
            else:
                ops = [dist.P2POp(dist.irecv, self.inbuf[s], self.src)]
            return _Works(dist.batch_isend_irecv(ops) if ops else [])

    def _issue_gather(self, ob, s):
        if not self.p2p:
            return dist.gather(ob, self.gathered[s] if self.rank == self.src else None, dst=self.src, async_op=True)
        if self.rank == self.src:
            ops = [dist.P2POp(dist.irecv, self.gathered[s][r], r) for r in range(self.world) if r != self.src]
        else:
            ops = [dist.P2POp(dist.isend, ob, self.src)]
        return _Works(dist.batch_isend_irecv(ops) if ops else [])

    def _local_input(self, pool, step):
        if self.transfer and self.p2p and self.rank == self.src:
            return self.shards(pool, step)[self.src]  # the coordinator's own shard: no copy
        if self.transfer:
            return self.inbuf[step % self.slots]
        # single process (the coordinator's shard is already resident in its
        # HBM) or local mode (every rank reads its own staged shard)
        n_batches = pool.shape[0] // self.B
        b = step % n_batches
        return pool[b * self.B:(b + 1) * self.B]

    # ---------------------------------------------------------------- run
    def run(self, pool: torch.Tensor | None, first: int, n: int, stamps: bool = True) -> None:
        """Pipelined steps [first, first+n). `pool` (u8 [N,H,W,3] on this
        rank's device) is needed on the coordinator in scatter mode and on
        every rank in local mode.

        stamps=True records a timing event pair per step (latency_ms) and
        joins each step's gather into the compute stream right away, so a
        step's latency is scatter issue -> gathered top-1. stamps=False is
        the throughput mode: no timing events (each is a release barrier on
        the stream, ~10 us of idle GPU between forwards) and the gather of
        step i is joined only before step i + slots reuses its output slot, so
        no rank's next forward waits for the slowest rank's previous one."""
        stamp = self._stamp if stamps else (lambda store, step: None)
        pending = {}  # slot -> gather work not yet joined
        stamp(self.t_start, first)
        h = self._issue_input(pool, first)
        for i in range(first, first + n):
            if h is not None:
                h.wait()
            h = None
            if i + 1 < first + n and self.transfer:
                # batch i+1's transfer may start once compute(i-1) is done
                stamp(self.t_start, i + 1)
                h = self._issue_input(pool, i + 1)
            s = i % self.slots
            if s in pending:
                pending.pop(s).wait()  # gather(i - slots) has read this output slot
            ob = self.outbuf[s]
            with _Range("dp.predict", self.cuda):
                self.predict_fn(self._local_input(pool, i), (ob[0], ob[1].view(torch.float32)))
            if self.distributed:
                with _Range("dp.gather", self.cuda):
                    g = self._issue_gather(ob, s)
                    if stamps:
                        g.wait()
                    else:
                        pending[s] = g
            stamp(self.t_end, i)
            if not self.transfer and i + 1 < first + n:
                stamp(self.t_start, i + 1)
        for g in pending.values():
            g.wait()

    def results(self, step: int) -> tuple[torch.Tensor, torch.Tensor]:
        """Top-1 (class int32 [world*B], prob f32 [world*B]) of `step` at the
        coordinator, in global batch order."""
        s = step % self.slots
        if self.distributed:
            if self.rank != self.src:
                raise RuntimeError("results are gathered on the coordinator only")
            parts = list(self.gathered[s])
            if self.p2p:
                parts[self.src] = self.outbuf[s]  # the coordinator's own answers were not sent to itself
            cat = torch.cat(parts, dim=1)
        else:
            cat = self.outbuf[s]
        return cat[0].clone(), cat[1].clone().view(torch.float32)


def broadcast_state_dict(state: dict | None, src: int, device: torch.device) -> dict:
    """Distribute model weights from `src` to every rank over the collective
    backend (the `train` verb's 'copy the model file to every VM',
    src/services.rs:139-144, as one broadcast per tensor)."""
    if not (dist.is_available() and dist.is_initialized()):
        return state
    meta = [[(k, tuple(v.shape)) for k, v in state.items()]] if dist.get_rank() == src else [None]
    dist.broadcast_object_list(meta, src=src)
    out = {}
    for k, shape in meta[0]:
        t = state[k].to(device, torch.float32).contiguous() if dist.get_rank() == src else \
            torch.empty(shape, dtype=torch.float32, device=device)
        dist.broadcast(t, src=src)
        out[k] = t.cpu()
    return out
