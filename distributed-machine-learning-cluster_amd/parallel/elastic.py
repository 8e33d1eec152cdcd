"""Elastic data-parallel inference: survive the loss of a rank mid-job by
rebuilding the collective group over the survivors and re-sharding.

Reference counterpart: node-level elasticity only. Job re-assignment over
the active members every 3 s and re-issue of the lost queries
(src/services.rs:199-211, 407-433; SURVEY.md §5 "Elastic recovery"). Inside
one node the GPUs are ranks of one RCCL communicator, and a collective with
a dead rank never completes. So recovery has to happen at the communicator
level:

  1. A failed collective raises. Gloo raises on a closed peer connection.
     RCCL raises after its timeout once the watchdog aborts the
     communicator; this needs TORCH_NCCL_ASYNC_ERROR_HANDLING=2, which
     cleans up without tearing the process down. ``ElasticDPInference``
     sets it when missing.
  2. Every survivor reports itself alive under ``e<epoch>/alive/<rank>``
     in the job's TCPStore. The store is the one the first group was
     created with; it is hosted by the coordinator.
  3. The coordinator waits a grace period, publishes the member list
     ``e<epoch>/members``, and every survivor re-initialises the process
     group with its new rank and world size on ``PrefixStore("e<epoch+1>")``.
  4. The step that failed is not committed. It reruns at the same image
     cursor over the new world, so every image is classified exactly once.

The coordinator (global rank 0) holds the image pool and the results, and it
must survive. Losing it is a node failure, which is handled by the control
plane's leader fail-over and job resume.
"""
from __future__ import annotations

import datetime
import os
import time
from typing import Callable

import torch
import torch.distributed as dist

PredictFn = Callable[[torch.Tensor, tuple], None]


class RankLost(RuntimeError):
    pass


class ElasticDPInference:
    def __init__(self, predict_fn: PredictFn, per_rank_batch: int, device: torch.device, image_shape=(224, 224, 3),
                 timeout_s: float = 30.0, grace_s: float | None = None):
        if not (dist.is_available() and dist.is_initialized()):
            raise RuntimeError("ElasticDPInference needs an initialised default process group")
        self.predict_fn = predict_fn
        self.B = per_rank_batch
        self.device = device
        self.image_shape = tuple(image_shape)
        self.timeout_s = timeout_s
        self.grace_s = grace_s if grace_s is not None else 2 * timeout_s
        self.backend = dist.get_backend()
        if self.backend == "nccl":
            os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "2")
        self.store = dist.distributed_c10d._get_default_store()
        self.global_rank = dist.get_rank()  # identity across epochs
        self.members = list(range(dist.get_world_size()))  # global ranks of the current group
        self.epoch = 0
        self.recoveries: list[dict] = []
        self._alloc()

    # ------------------------------------------------------------ group state
    @property
    def world(self) -> int:
        return len(self.members)

    @property
    def rank(self) -> int:
        return self.members.index(self.global_rank)

    @property
    def coordinator(self) -> bool:
        return self.global_rank == 0

    def _alloc(self):
        H, W, C = self.image_shape
        self.inbuf = torch.empty(self.B, H, W, C, dtype=torch.uint8, device=self.device)
        self.outbuf = torch.empty(2, self.B, dtype=torch.int32, device=self.device)
        self.gathered = [torch.empty(2, self.B, dtype=torch.int32, device=self.device)
                         for _ in range(self.world)] if self.rank == 0 else None

    def _recover(self, err: Exception, cursor: int) -> int:
        """Agree on the survivors and the resume cursor (the coordinator's:
        a step it did not commit is redone), then rebuild the group."""
        t0 = time.time()
        e = self.epoch
        self.store.set(f"e{e}/alive/{self.global_rank}", "1")
        if self.coordinator:
            deadline = time.time() + self.grace_s
            alive = []
            while time.time() < deadline:
                alive = [g for g in self.members if self.store.check([f"e{e}/alive/{g}"])]
                if len(alive) == len(self.members):
                    break
                time.sleep(0.05)
            self.store.set(f"e{e}/cursor", str(cursor))
            self.store.set(f"e{e}/members", ",".join(str(g) for g in sorted(alive)))
        self.store.wait([f"e{e}/members"], datetime.timedelta(seconds=self.grace_s + self.timeout_s))
        members = [int(g) for g in self.store.get(f"e{e}/members").decode().split(",")]
        cursor = int(self.store.get(f"e{e}/cursor").decode())
        if self.global_rank not in members:
            raise RankLost(f"rank {self.global_rank} was dropped from the group in epoch {e}") from err
        try:
            dist.destroy_process_group()
        except Exception:  # noqa: BLE001  (the old group may already be aborted)
            pass
        self.epoch = e + 1
        self.members = members
        dist.init_process_group(self.backend, store=dist.PrefixStore(f"e{self.epoch}", self.store),
                                rank=self.rank, world_size=self.world,
                                timeout=datetime.timedelta(seconds=self.timeout_s))
        self._alloc()
        self.recoveries.append({"epoch": self.epoch, "members": list(members), "cursor": cursor,
                                "error": (str(err).splitlines() or [""])[0], "seconds": time.time() - t0})
        return cursor

    # ------------------------------------------------------------ run
    def _step(self, pool: torch.Tensor | None, cursor: int, n_images: int):
        """One global step at image `cursor`: scatter, classify, gather.
        Returns the number of images it covers (coordinator view)."""
        count = min(self.B * self.world, n_images - cursor)
        # the coordinator announces how many images this step covers; ranks
        # past the end classify a padded shard that is dropped
        hdr = torch.tensor([count], dtype=torch.int64, device=self.device)
        dist.broadcast(hdr, src=0)
        count = int(hdr.item())
        shards = None
        if self.rank == 0:
            sl = pool[cursor:cursor + count]
            pad = self.B * self.world - count
            if pad:
                sl = torch.cat([sl, sl[-1:].expand(pad, *sl.shape[1:])])
            shards = list(sl.to(self.device).split(self.B))
        dist.scatter(self.inbuf, shards, src=0)
        self.predict_fn(self.inbuf, (self.outbuf[0], self.outbuf[1].view(torch.float32)))
        dist.gather(self.outbuf, self.gathered, dst=0)
        return count

    def run_dataset(self, pool: torch.Tensor | None, n_images: int):
        """Classify images [0, n_images) of the coordinator's `pool` (u8
        [N,H,W,3]). Returns (class int32 [n], prob f32 [n]) on the
        coordinator, None elsewhere."""
        idx = torch.empty(n_images, dtype=torch.int32) if self.coordinator else None
        prob = torch.empty(n_images, dtype=torch.float32) if self.coordinator else None
        cursor = 0
        while cursor < n_images:
            try:
                count = self._step(pool, cursor, n_images)
            except RankLost:
                raise
            except Exception as err:  # noqa: BLE001  (a peer is gone: rebuild and redo this step)
                cursor = self._recover(err, cursor)
                continue
            if self.coordinator:
                cat = torch.cat(self.gathered, dim=1)[:, :count].cpu()
                idx[cursor:cursor + count] = cat[0]
                prob[cursor:cursor + count] = cat[1].view(torch.float32)
            cursor += count
        return (idx, prob) if self.coordinator else None
