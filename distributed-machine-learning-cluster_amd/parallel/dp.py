"""Data-parallel inference across the GPUs of a node: Python face of the
native layer in csrc/comm (dp::Rank / dp::Group over RCCL).

Reference counterpart: ``predict`` fans query images out to the members and
each member classifies its share (src/services.rs:146-151, 407-433, 475-497).
Within a node that fan-out is RCCL over xGMI:

* :class:`DataParallelRunner` - one rank of a multi-process job (one process
  per GPU; ``bench.py``): rank 0 scatters u8 shards with grouped
  ncclSend/ncclRecv on a high-priority comm stream, every rank runs the
  engine, the (class, prob) answers are gathered back on a second
  communicator; steps are double-buffered with HIP events, and with
  ``lanes=2`` consecutive steps alternate between two model instances so
  step i+1's forward overlaps step i's tail.
* :class:`NodeGroup` - one process owning several GPUs (the serving
  executor's form, ``dmlc-node --gpus N``): ncclCommInitAll, and on the loss
  of a GPU the group aborts its communicators, rebuilds them over the
  survivors and redoes the uncommitted images (every image answered exactly
  once).

The protocol itself (shard order, exactly-once answers, rank loss) is
covered on the CPU over an in-process fake transport by
tests/test_dp_native_cpu.py.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .. import native


class DataParallelRunner:
    """One rank of a multi-process data-parallel job.

    engine: this rank's :class:`dmlc.runtime.InferenceEngine`.
    ids: two ``native().rccl_unique_id()`` byte strings created on rank 0 and
    shared with every rank (any side channel; bench.py uses gloo).
    """

    def __init__(self, engine, world: int, rank: int, ids: tuple[bytes, bytes] = (b"", b""),
                 batch_per_rank: int = 256, scatter: bool = True, use_graph: bool = True, lanes: int = 2,
                 timeout_ms: int = -1):
        C = native()
        self.world, self.rank, self.batch_per_rank = world, rank, batch_per_rank
        self._r = C.DpRunner(engine._e, world, rank, ids[0], ids[1], batch_per_rank, scatter=scatter,
                             image_size=engine.image_size, use_graph=use_graph, timeout_ms=timeout_ms, lanes=lanes)
        self._engine = engine  # the runner borrows the engine

    def run(self, pool: torch.Tensor | None, first: int, n: int, pipelined: bool = True) -> dict:
        """Steps [first, first+n) over a staged u8 pool [N, S, S, 3] (rank 0 in
        scatter mode; every rank's own pool in local mode). Returns
        {steps, images, step_ms} (step_ms: unpipelined runs only)."""
        ptr, count = (pool.data_ptr(), pool.shape[0]) if pool is not None else (0, 0)
        if pool is not None:
            # the native streams do not wait on torch's: whatever produced
            # the pool on the current stream must be done first
            torch.cuda.current_stream(pool.device).synchronize()
        return self._r.run(ptr, count, first, n, pipelined=pipelined)

    def last_results(self) -> tuple[list[int], list[float]]:
        """(class ids, probabilities) of the last step (coordinator)."""
        return self._r.last_results()

    def synchronize(self) -> None:
        self._r.sync()


class NodeGroup:
    """Several GPUs of one process: classify any number of u8 images held in
    the first engine's GPU memory, sharded over the group, elastic on GPU
    loss."""

    def __init__(self, engines: list, batch_per_rank: int = 256, use_graph: bool = True, timeout_ms: int = 30000):
        C = native()
        self._engines = engines
        self._g = C.DpGroup([e._e for e in engines], batch_per_rank, engines[0].image_size, use_graph, timeout_ms)

    def classify(self, images: torch.Tensor):
        """images: contiguous u8 [N, S, S, 3] on the coordinator's GPU.
        Returns (idx int32 [N], prob f32 [N], stats dict)."""
        if not images.is_contiguous() or images.dtype != torch.uint8:
            raise ValueError("images must be contiguous uint8 [N, S, S, 3]")
        # the native streams do not wait on torch's current stream
        torch.cuda.current_stream(images.device).synchronize()
        idx, prob, st = self._g.classify(images.data_ptr(), images.shape[0])
        return torch.from_numpy(idx), torch.from_numpy(prob), st

    @property
    def members(self) -> list[int]:
        return self._g.members


def broadcast_state_dict(state: dict | None, src: int, device: torch.device) -> dict:
    """Distribute model weights from `src` to every rank of a torch.distributed
    job (multi-process setups that hold weights as tensors; the serving
    executor broadcasts its packed weight arena with RCCL natively). The
    `train` verb's 'copy the model file to every VM' (src/services.rs:139-144)
    as one broadcast per tensor."""
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
