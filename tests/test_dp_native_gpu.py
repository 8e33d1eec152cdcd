"""Native data-parallel layer on a real GPU: the HIP worker (engine on a
compute stream, answers over the comm streams, pinned D2H) must give the same
answers as a direct engine forward, for full and ragged steps, pipelined and
unpipelined. librccl itself runs here through one-rank loopback
communicators (test_rccl_loopback); RCCL send/recv between ranks needs >= 2
GPUs: the driver's multi-GPU bench runs that, and the protocol itself is
covered on CPU by tests/test_dp_native_cpu.py."""
import pytest
import torch

import dmlc
from dmlc.runtime import InferenceEngine

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    return InferenceEngine("resnet18", device=0, max_batch=64, seed=3)


def _pool(n, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return torch.randint(0, 256, (n, 224, 224, 3), dtype=torch.uint8, device="cuda", generator=g)


@pytest.mark.parametrize("pipelined,lanes", [(True, 1), (False, 1), (True, 2), (False, 2)])
def test_runner_world1_matches_engine(gpu, eng, pipelined, lanes):
    """lanes=2: odd steps run on a second model instance on its own stream
    (weights copied on the device); the last of 4 steps is such a step."""
    C = dmlc.native()
    pool = _pool(128, 1)
    torch.cuda.synchronize()
    r = C.DpRunner(eng._e, 1, 0, b"", b"", 64, lanes=lanes)
    out = r.run(pool.data_ptr(), 128, 0, 4, pipelined=pipelined)
    r.sync()
    assert out["steps"] == 4 and out["images"] == 4 * 64
    if not pipelined:
        assert len(out["step_ms"]) == 4 and all(t > 0 for t in out["step_ms"])
    idx, prob = r.last_results()
    # step 3 reads pool batch 3 % 2 = 1
    ref_i, ref_p = eng.predict(pool[64:].contiguous(), use_graph=False)
    torch.cuda.synchronize()
    assert idx == ref_i.cpu().tolist()
    assert torch.allclose(torch.tensor(prob), ref_p.cpu(), atol=1e-6)


def test_group_one_gpu_ragged(gpu, eng):
    C = dmlc.native()
    n = 64 * 3 + 17
    pool = _pool(n, 2)
    torch.cuda.synchronize()
    g = C.DpGroup([eng._e], 64)
    idx, prob, st = g.classify(pool.data_ptr(), n)
    assert st["images"] == n and st["steps"] == 4 and st["recoveries"] == 0
    ref_i, ref_p = [], []
    for s in range(0, n, 64):
        i, p = eng.predict(pool[s:s + 64].contiguous(), use_graph=False)
        ref_i.append(i.cpu())
        ref_p.append(p.cpu())
    torch.cuda.synchronize()
    assert idx.tolist() == torch.cat(ref_i).tolist()
    assert torch.allclose(torch.from_numpy(prob), torch.cat(ref_p), atol=1e-6)
    assert g.members == [0]


def test_python_wrappers(gpu, eng):
    """dmlc.parallel.DataParallelRunner / NodeGroup over the same native
    layer: answers equal a direct engine forward."""
    from dmlc.parallel import DataParallelRunner, NodeGroup
    pool = _pool(128, 5)
    torch.cuda.synchronize()
    r = DataParallelRunner(eng, 1, 0, batch_per_rank=64, lanes=2)
    out = r.run(pool, 0, 2)
    r.synchronize()
    assert out["steps"] == 2
    idx, _ = r.last_results()
    ref_i, _ = eng.predict(pool[64:].contiguous(), use_graph=False)
    g = NodeGroup([eng], batch_per_rank=64)
    gi, gp, st = g.classify(pool[:100].contiguous())
    ref_g, ref_p = eng.predict(pool[:64].contiguous(), use_graph=False)
    torch.cuda.synchronize()
    assert idx == ref_i.cpu().tolist()
    assert gi[:64].tolist() == ref_g.cpu().tolist() and st["images"] == 100
    assert torch.allclose(gp[:64], ref_p.cpu(), atol=1e-6)


@pytest.mark.parametrize("max_ctas,nbytes", [(0, 1 << 20), (1, 1 << 20), (1, 2048), (4, 38535168)])
def test_rccl_loopback(gpu, max_ctas, nbytes):
    """librccl through the RcclComm wrapper on one GPU: a one-rank
    communicator (plain, or CTA-capped as the answer communicator is) moves a
    buffer to itself by grouped send/recv and by broadcast, bit-exact
    (38.5 MB = one 256-image u8 shard)."""
    assert dmlc.native().rccl_loopback(0, nbytes, max_ctas)


def test_runner_stage_then_local_run(gpu, eng):
    """bench.py's default input mode: DpRunner.stage copies the coordinator's
    shard into the rank's own HBM pool (world 1: a device copy; at N > 1 the
    other shards go over the shard communicator), then a local-mode run
    classifies it like a direct forward."""
    C = dmlc.native()
    src = _pool(64, 5)
    dst = torch.zeros_like(src)
    torch.cuda.synchronize()
    r = C.DpRunner(eng._e, 1, 0, b"", b"", 64, scatter=False, lanes=1)
    r.stage(src.data_ptr(), dst.data_ptr())
    assert torch.equal(dst, src)
    out = r.run(dst.data_ptr(), 64, 0, 2)
    r.sync()
    assert out["images"] == 2 * 64
    idx, prob = r.last_results()
    ref_i, _ = eng.predict(src, use_graph=False)
    torch.cuda.synchronize()
    assert idx == ref_i.cpu().tolist()
