"""The multi-rank data-parallel protocol ON the GPU:
several virtual ranks on one MI355X, each a dp::Runner (or dp::Group member)
over its own HIP worker, engines and streams, exchanging device buffers over
the device-loopback communicator (csrc/comm/loopback_comm.cpp: the host
fake's rendezvous and per-pair FIFO matching, with every matched send/recv a
stream-ordered device copy between events on the two ranks' streams and no
host synchronisation). The host fake (tests/test_dp_native_cpu.py) moves
bytes synchronously, so it cannot catch a slot reused before its stream has
sent it or an answer read before its copy landed; here those show up as wrong
answers.

Reference behaviour: the leader's fan-out of queries to members and their
replies (src/services.rs:414-421), rebuilt as RCCL scatter/gather.

Every step's gathered answers on the coordinator must equal direct engine
forwards of the same images at the same per-rank batch (same kernels, so
bit-identical), for every step of pipelined and unpipelined runs.
"""
import numpy as np
import pytest
import torch

import dmlc
from dmlc.models import build, state_dict_f32
from dmlc.runtime import InferenceEngine

pytestmark = pytest.mark.gpu

C = dmlc.native()


@pytest.fixture(scope="module")
def sd():
    return state_dict_f32(build("resnet18", seed=61, randomize_bn=True))


def _engines(sd, n, max_batch):
    return [InferenceEngine("resnet18", sd, device=0, max_batch=max_batch) for _ in range(n)]


def _direct(ref, imgs, counts):
    """Answers of a direct engine forward of each rank's shard (batch = that
    rank's count), concatenated in rank order."""
    idx, prob, off = [], [], 0
    for c in counts:
        i, p = ref.predict(imgs[off:off + c])
        idx.append(i.cpu())
        prob.append(p.cpu())
        off += c
    return torch.cat(idx).numpy(), torch.cat(prob).numpy()


@pytest.mark.parametrize("world,mode,coord_weight,calib", [
    (2, "scatter", 1.0, 0),
    (4, "scatter", 0.75, 0),    # weighted counts: the coordinator takes 3/4 of a share
    (4, "staged", 1.0, 0),      # shards staged in every rank's HBM once (stage()), then used in place
    (2, "scatter", 1.0, 3),     # bench.py --coord-weight auto: calibration rounds, then the timed run
])
def test_runner_on_device_loopback_matches_direct_forwards(gpu, sd, world, mode, coord_weight, calib):
    per = 24
    engs = _engines(sd, world, per)
    ref = InferenceEngine("resnet18", sd, device=0, max_batch=per)
    counts0 = C.dp_weighted_counts(per, world, coord_weight)
    G0 = sum(counts0)
    g = torch.Generator().manual_seed(62 + world)
    pool = torch.randint(0, 256, (2 * G0, 224, 224, 3), generator=g, dtype=torch.uint8).to(gpu)
    torch.cuda.synchronize()
    out = C.dp_loopback_bench([e._e for e in engs], pool.data_ptr(), per, coord_weight, mode, lanes=2, prime=4,
                              steps=50, unpipelined=6, calib_rounds=calib, calib_steps=4)
    counts = out["counts"]
    G = sum(counts)
    assert all(r == out["runs"][0] for r in out["runs"]), out["runs"]  # every rank ran the same steps
    answers = out["answers"]
    timed = [a for a in answers if a[0] >= 1000]
    assert len(timed) == 50 + 6, len(timed)
    if calib:
        assert out["calibration"]["rounds"], out["calibration"]
    nb = 2 if mode == "staged" else max(1, (2 * G0) // G)
    cache = {}
    for step, idx, prob in timed:
        k = step % nb
        if k not in cache:
            imgs = pool[k * (G0 if mode == "staged" else G):][:G]
            cache[k] = _direct(ref, imgs, counts)
        ei, ep = cache[k]
        np.testing.assert_array_equal(idx, ei, err_msg=f"step {step}")
        np.testing.assert_array_equal(prob, ep, err_msg=f"step {step}")


def test_group_on_device_loopback_ragged_and_lost_member(gpu, sd):
    """dp::Group (the serving fleet's scatter): a ragged last step (n not a
    multiple of the group batch), then the same query with member 2 lost
    after one step: the group rebuilds its communicators over the survivors,
    redoes the uncommitted images and commits every image exactly once; the
    answers equal direct forwards (a full-size shard runs the same kernels
    as the direct batch of that size; redone shards may run at another batch
    size, so those are compared by class on clear margins)."""
    world, per = 4, 24
    engs = _engines(sd, world, per)
    ref = InferenceEngine("resnet18", sd, device=0, max_batch=per)
    n = world * per * 2 + 37
    g = torch.Generator().manual_seed(64)
    imgs = torch.randint(0, 256, (n, 224, 224, 3), generator=g, dtype=torch.uint8).to(gpu)
    torch.cuda.synchronize()
    # direct answers in batches of the group's full shards (24 images) and the tail
    ri, rp, rl = [], [], []
    for s0 in range(0, n, per):
        i, p, lg = ref.predict(imgs[s0:s0 + per], return_logits=True)
        ri.append(i.cpu())
        rp.append(p.cpu())
        rl.append(lg.float().cpu())
    ri, rp = torch.cat(ri).numpy(), torch.cat(rp).numpy()
    sm = torch.softmax(torch.cat(rl), -1).topk(2, -1).values
    clear = ((sm[:, 0] - sm[:, 1]) / sm[:, 0] > 0.02).numpy()
    full = world * per * 2  # images in full 24-image shards (no loss): the same batches as the direct forwards
    out = C.dp_loopback_group([e._e for e in engs], imgs.data_ptr(), n, per, repeats=2)
    assert (out["commits"] == 1).all()
    assert out["stats"]["recoveries"] == 0
    np.testing.assert_array_equal(out["idx"][:full], ri[:full])
    np.testing.assert_array_equal(out["prob"][:full], rp[:full])
    assert (out["idx"] == ri)[clear].all()
    np.testing.assert_allclose(out["prob"], rp, rtol=2e-2, atol=1e-6)
    lost = C.dp_loopback_group([e._e for e in _engines(sd, world, per)], imgs.data_ptr(), n, per, fail_member=2,
                               fail_after=1)
    assert (lost["commits"] == 1).all()
    assert lost["stats"]["recoveries"] >= 1 and 2 not in lost["members"], lost["stats"]
    assert len(lost["builds"]) >= 2 and lost["builds"][-1] == [0, 1, 3], lost["builds"]
    assert (lost["idx"] == ri)[clear].all()
    np.testing.assert_allclose(lost["prob"], rp, rtol=2e-2, atol=1e-6)
