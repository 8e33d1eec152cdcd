"""Multi-process weight distribution over torch.distributed (gloo, CPU):
``dmlc.parallel.broadcast_state_dict`` gives every rank the source rank's
exact weights, and a model loaded from them classifies like the source's.
(The data-parallel scatter/gather protocol is native, csrc/comm; it is
tested over an in-process fake transport in tests/test_dp_native_cpu.py.)"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from dmlc.models import build, state_dict_f32
from dmlc.parallel import broadcast_state_dict


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sd = state_dict_f32(build("resnet18", seed=3)) if rank == 0 else None
        sd = broadcast_state_dict(sd, 0, torch.device("cpu"))
        model = build("resnet18", seed=None)
        model.load_state_dict(sd, strict=False)
        model.eval()
        g = torch.Generator().manual_seed(7)
        x = torch.randn(2, 3, 64, 64, generator=g)
        with torch.no_grad():
            q.put((rank, model(x), sum(float(v.double().sum()) for v in sd.values())))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_broadcast_state_dict_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict((r, (y, s)) for r, y, s in (q.get(timeout=240) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = build("resnet18", seed=3).eval()
    with torch.no_grad():
        y_ref = ref(torch.randn(2, 3, 64, 64, generator=torch.Generator().manual_seed(7)))
    for r in range(world):
        assert torch.equal(got[r][0], got[0][0])
        assert got[r][1] == got[0][1]
        assert torch.allclose(got[r][0], y_ref, rtol=1e-5, atol=1e-5)
