"""Data-parallel inference coordinator (scatter u8 shards -> per-rank
forward -> gather top-1) with world_size 2 on the gloo backend (CPU). The
same code path runs over RCCL on GPUs in bench.py."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from dmlc.models import build, state_dict_f32
from dmlc.parallel import DPInference, broadcast_state_dict

MEAN = torch.tensor([0.485, 0.456, 0.406]).view(1, 3, 1, 1)
STD = torch.tensor([0.229, 0.224, 0.225]).view(1, 3, 1, 1)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _predict_fn(model):
    def f(imgs, out):
        x = (imgs.permute(0, 3, 1, 2).float() / 255 - MEAN) / STD
        with torch.no_grad():
            p = torch.softmax(model(x), -1)
        v, i = p.max(-1)
        out[0].copy_(i.int())
        out[1].copy_(v)
    return f


def _worker(rank, world, port, B, steps, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sd = state_dict_f32(build("resnet18", seed=3)) if rank == 0 else None
        sd = broadcast_state_dict(sd, 0, torch.device("cpu"))
        model = build("resnet18", seed=None)
        model.load_state_dict(sd, strict=False)
        model.eval()
        dev = torch.device("cpu")
        pool = None
        if rank == 0:
            g = torch.Generator().manual_seed(7)
            pool = torch.randint(0, 256, (2 * B * world, 64, 64, 3), generator=g, dtype=torch.uint8)
        dp = DPInference(_predict_fn(model), B, dev, image_shape=(64, 64, 3))
        dp.run(pool, 0, steps, stamps=False)  # bench.py's timed loop (no timing events)
        dp.run(pool, steps, steps)            # its latency pass
        if rank == 0:
            res = [dp.results(s) for s in range(2 * steps - 2, 2 * steps)]
            lat = [dp.latency_ms(s) for s in range(steps, 2 * steps)]
            q.put((res, [dp.shards(pool, s) for s in range(2 * steps - 2, 2 * steps)], lat))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,p2p", [(2, "1"), (3, "1"), (2, "0")])
def test_dp_scatter_gather_gloo(monkeypatch, world, p2p):
    """p2p=1: point-to-point sends of the other ranks' shards (the
    coordinator's own shard read in place); p2p=0: dist.scatter/gather."""
    monkeypatch.setenv("DMLC_DP_P2P", p2p)
    B, steps = 3, 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, B, steps, q)) for r in range(world)]
    for p in procs:
        p.start()
    res, shards, lat = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    model = build("resnet18", seed=3)
    f = _predict_fn(model)
    for (idx, prob), sh in zip(res, shards):
        imgs = torch.cat(sh)
        exp = (torch.empty(world * B, dtype=torch.int32), torch.empty(world * B))
        f(imgs, exp)
        assert torch.equal(idx, exp[0])
        assert torch.allclose(prob, exp[1], rtol=1e-5, atol=1e-6)
    assert all(x > 0 for x in lat)


def _elastic_worker(rank, world, port, B, n_images, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    import datetime
    from dmlc.parallel import ElasticDPInference
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=4))
    model = build("resnet18", seed=5)
    model.eval()
    f = _predict_fn(model)
    calls = [0]

    def predict(imgs, out):
        calls[0] += 1
        if rank == world - 1 and calls[0] == 2:
            os._exit(17)  # this "GPU" dies mid-step: shard received, result never sent
        f(imgs, out)

    pool = None
    if rank == 0:
        g = torch.Generator().manual_seed(9)
        pool = torch.randint(0, 256, (n_images, 48, 48, 3), generator=g, dtype=torch.uint8)
    dp = ElasticDPInference(predict, B, torch.device("cpu"), image_shape=(48, 48, 3), timeout_s=4.0)
    res = dp.run_dataset(pool, n_images)
    if rank == 0:
        q.put((res, pool, dp.recoveries, dp.world))
    dist.barrier()
    dist.destroy_process_group()


def test_elastic_dp_survives_rank_loss():
    """world 3 over gloo; rank 2 dies inside its 2nd step. The survivors
    rebuild a 2-rank group, redo the uncommitted step and classify every
    image exactly once."""
    world, B, n = 3, 2, 19
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_elastic_worker, args=(r, world, port, B, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    (idx, prob), pool, recoveries, final_world = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
    assert [p.exitcode for p in procs] == [0, 0, 17]
    assert final_world == 2 and len(recoveries) == 1 and recoveries[0]["members"] == [0, 1]
    exp = (torch.empty(n, dtype=torch.int32), torch.empty(n))
    _predict_fn(build("resnet18", seed=5).eval())(pool, exp)
    assert torch.equal(idx, exp[0])
    assert torch.allclose(prob, exp[1], rtol=1e-4, atol=1e-6)
