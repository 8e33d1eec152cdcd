"""The serving fleet of one node (csrc/comm/fleet.h) on host workers and the
rendezvous host communicator: what `dmlc-node --gpus N` does with its GPUs.

Reference behaviour being rebuilt: the leader splits the
active members between the two concurrent jobs, the first floor(n/2) to
ResNet18 and the rest to AlexNet, every 3 s (src/services.rs:199-211), and
sends every query to one member of the job's set (:414-421). Here:

* the GPUs of a node are split with that rule, per job (disjoint partitions,
  so no two models ever hold communicators on one GPU), and re-split when a
  GPU is lost;
* a small query runs on ONE GPU of its model's partition, the least loaded,
  so concurrent queries spread over the partition; a large batch is
  scattered over the partition with RCCL (dp::Group);
* a GPU that moves to another job gets that job's weights by a broadcast
  from a live instance (a host worker's class depends on the first bytes of
  its weight arena, and a replica starts with an empty arena, so a wrong or
  missing broadcast shows up as wrong answers);
* every query is answered exactly once, in order, across losses.
"""
import numpy as np
import pytest

import dmlc

C = dmlc.native()
H = W = 8
SEEDS = {"resnet18": 11, "alexnet": 377}


def _imgs(n, seed=0):
    return np.random.default_rng(seed).integers(0, 256, size=(n, H, W, 3), dtype=np.uint8)


def _expect(imgs, model):
    flat = imgs.reshape(imgs.shape[0], -1).astype(np.int64)
    return ((flat.sum(1) + SEEDS[model]) % 1000).astype(np.int32), (imgs[:, 0, 0, 0].astype(np.float32) + 1) / 257


def _fleet(devices=8, lanes=2, delay_us=0, max_per_rank=8, min_shard=4, jobs=("resnet18", "alexnet")):
    f = C.HostFleet(list(range(devices)), H, W, lanes, delay_us, max_per_rank, min_shard, SEEDS)
    f.set_jobs(list(jobs))
    for m in jobs:
        f.load(m)
    return f


def _check(out, imgs, queries):
    assert all(e == "" for e in out["errors"]), out["errors"]
    for q, (model, first, count) in enumerate(queries):
        ei, ep = _expect(imgs[first:first + count], model)
        np.testing.assert_array_equal(out["idx"][q], ei, err_msg=f"query {q} {model}")
        np.testing.assert_array_equal(out["prob"][q], ep)


def _small_queries(n_imgs, k, seed=0, models=("resnet18", "alexnet"), max_n=3):
    rng = np.random.default_rng(seed)
    qs = []
    for i in range(k):
        c = int(rng.integers(1, max_n + 1))
        f = int(rng.integers(0, n_imgs - c))
        qs.append((models[i % len(models)], f, c))
    return qs


@pytest.mark.parametrize("n,devices,want", [
    (1000, list(range(8)), [(d, 125 * d, 125) for d in range(8)]),
    (10, [0, 1, 2, 4], [(0, 0, 2), (1, 2, 3), (2, 5, 2), (4, 7, 3)]),   # after a loss: the live GPUs only
    (3, list(range(8)), [(0, 0, 1), (1, 1, 1), (2, 2, 1)]),             # no empty slice
    (7, [5], [(5, 0, 7)]),
])
def test_shard_replica_slices_one_per_live_gpu(n, devices, want):
    """A staged shard replica lives in HBM as one contiguous slice per live
    GPU (csrc/serve/shard.h shard_slices, used by the GPU executor's
    stage_blob); shard queries then prefer the GPU holding their slice."""
    got = C.shard_slices(n, devices)
    assert got == want
    assert sum(c for _, _, c in got) == n


@pytest.mark.parametrize("live,jobs,want", [
    (list(range(8)), 2, [[0, 1, 2, 3], [4, 5, 6, 7]]),
    ([0, 1, 2, 4, 5, 6, 7], 2, [[0, 1, 2], [4, 5, 6, 7]]),   # first floor(7/2) to job 1
    ([0, 1, 2, 3, 4, 6, 7], 2, [[0, 1, 2], [3, 4, 6, 7]]),
    ([7, 3, 5, 1], 2, [[1, 3], [5, 7]]),                      # sorted first
    (list(range(8)), 3, [[0, 1], [2, 3, 4], [5, 6, 7]]),
    ([2], 2, [[2], [2]]),                                     # fewer GPUs than jobs: shared, one each
    ([0, 5], 3, [[0], [5], [0]]),
    ([], 2, [[], []]),
])
def test_partition_rule(live, jobs, want):
    assert C.dp_partition_devices(live, jobs) == want


def test_two_jobs_disjoint_halves_and_spread():
    f = _fleet(delay_us=3000)
    st = f.state()
    assert st["partitions"] == {"resnet18": [0, 1, 2, 3], "alexnet": [4, 5, 6, 7]}
    imgs = _imgs(256, seed=1)
    qs = _small_queries(256, 96, seed=2)
    out = f.run(imgs, qs, threads=24)
    _check(out, imgs, qs)
    assert not any(r["scattered"] for r in out["routes"])
    st = f.state()
    # every GPU of each partition served queries of its model, and no other
    for model, part in st["partitions"].items():
        served = {d: n for d, n in st["served"][model].items() if n}
        assert set(served) == set(part), (model, served)
    assert st["overlapping_worlds"] == []


def test_large_batch_is_scattered_over_the_partition():
    f = _fleet(max_per_rank=8, min_shard=4)
    imgs = _imgs(200, seed=3)
    qs = [("resnet18", 0, 100), ("alexnet", 50, 150), ("resnet18", 7, 9)]
    out = f.run(imgs, qs, threads=2)
    _check(out, imgs, qs)
    r = out["routes"]
    assert r[0]["scattered"] and r[0]["devices_used"] == 4
    assert r[1]["scattered"] and r[1]["devices_used"] == 4
    assert r[2]["scattered"] and r[2]["devices_used"] == 2  # 9 images, >= 4 per GPU
    st = f.state()
    assert st["overlapping_worlds"] == []
    # the scattered queries' shards were answered on every GPU of the partition
    assert all(st["served"]["resnet18"][d] > 0 for d in (0, 1, 2, 3))


def test_loss_rebalances_and_broadcasts_weights_to_moved_gpu():
    f = _fleet(delay_us=1000)
    f.lose(5)
    st = f.state()
    # live [0,1,2,3,4,6,7]: first floor(7/2) = 3 to job 1, GPU 3 moves to alexnet
    assert st["partitions"] == {"resnet18": [0, 1, 2], "alexnet": [3, 4, 6, 7]}
    assert ("alexnet", 3, True) in st["worker_builds"]  # a replica: weights by broadcast
    imgs = _imgs(256, seed=4)
    qs = _small_queries(256, 120, seed=5)
    out = f.run(imgs, qs, threads=24)
    _check(out, imgs, qs)
    st = f.state()
    assert st["served"]["alexnet"].get(3, 0) > 0  # the moved GPU answered, correctly
    assert st["served"]["alexnet"].get(5, 0) == 0
    assert st["overlapping_worlds"] == []
    # big batches still scatter over the new partitions
    out = f.run(imgs, [("alexnet", 0, 64), ("resnet18", 64, 64)], threads=2)
    _check(out, imgs, [("alexnet", 0, 64), ("resnet18", 64, 64)])
    assert out["routes"][0]["devices_used"] == 4 and out["routes"][1]["devices_used"] == 3


def test_abrupt_gpu_failure_under_concurrent_queries_exactly_once():
    f = _fleet(delay_us=2000)
    imgs = _imgs(300, seed=6)
    qs = _small_queries(300, 60, seed=7)
    out = f.run(imgs, qs, threads=16)
    _check(out, imgs, qs)
    f.fail(2)  # GPU 2 dies: found by the next query routed to it
    qs2 = _small_queries(300, 160, seed=8)
    out = f.run(imgs, qs2, threads=24)
    _check(out, imgs, qs2)  # every query answered once, correctly
    assert any(r["retries"] > 0 for r in out["routes"])
    st = f.state()
    assert 2 not in st["live"]
    assert st["partitions"] == {"resnet18": [0, 1, 3], "alexnet": [4, 5, 6, 7]}
    assert st["overlapping_worlds"] == []


def test_abrupt_member_failure_during_scatter():
    f = _fleet(max_per_rank=8, min_shard=4)
    f.fail(6)  # a non-coordinator GPU of alexnet's partition
    imgs = _imgs(160, seed=9)
    qs = [("alexnet", 0, 160)]
    out = f.run(imgs, qs, threads=1)
    _check(out, imgs, qs)
    st = f.state()
    assert 6 not in st["live"]
    assert st["partitions"] == {"resnet18": [0, 1, 2], "alexnet": [3, 4, 5, 7]}


def test_coordinator_failure_during_scatter_redone_on_rebalanced_fleet():
    f = _fleet(max_per_rank=8, min_shard=4)
    f.fail(0)  # resnet18's coordinator
    imgs = _imgs(100, seed=10)
    qs = [("resnet18", 0, 100)]
    out = f.run(imgs, qs, threads=1)
    _check(out, imgs, qs)
    assert out["routes"][0]["retries"] >= 1
    assert f.state()["partitions"]["resnet18"] == [1, 2, 3]


def test_fewer_gpus_than_jobs_share_without_communicators():
    f = _fleet(devices=1)
    st = f.state()
    assert st["partitions"] == {"resnet18": [0], "alexnet": [0]}
    imgs = _imgs(64, seed=11)
    qs = _small_queries(64, 40, seed=12, max_n=8) + [("alexnet", 0, 64)]
    out = f.run(imgs, qs, threads=8)
    _check(out, imgs, qs)
    assert f.state()["comm_builds"] == []


def test_losing_every_gpu_of_a_partition_rebuilds_from_host_weights():
    f = _fleet(devices=4)
    assert f.state()["partitions"] == {"resnet18": [0, 1], "alexnet": [2, 3]}
    f.lose(3)
    assert f.state()["partitions"] == {"resnet18": [0], "alexnet": [1, 2]}
    f.lose(2)
    f.lose(1)
    st = f.state()
    assert st["partitions"] == {"resnet18": [0], "alexnet": [0]}
    assert ("alexnet", 0, False) in st["worker_builds"]  # no live alexnet left: from the host weights
    imgs = _imgs(40, seed=13)
    qs = _small_queries(40, 20, seed=14)
    _check(f.run(imgs, qs, threads=4), imgs, qs)


def test_single_job_takes_every_gpu():
    f = _fleet(jobs=("resnet18",))
    assert f.state()["partitions"] == {"resnet18": list(range(8))}
    imgs = _imgs(64, seed=15)
    qs = _small_queries(64, 64, seed=16, models=("resnet18",))
    _check(f.run(imgs, qs, threads=16), imgs, qs)


def test_hot_swap_broadcasts_new_weights_to_every_gpu_of_the_partition():
    """`train`: the model is rebuilt from the new host weights on the first
    GPU of its partition and broadcast to the others, then swapped in; the
    other job keeps running on its own GPUs untouched."""
    f = _fleet(delay_us=500)
    imgs = _imgs(128, seed=17)
    before = f.state()["worker_builds"]
    f.set_seed("resnet18", 999)
    f.load("resnet18")
    new = f.state()["worker_builds"][len(before):]
    assert new == [("resnet18", 0, False), ("resnet18", 1, True), ("resnet18", 2, True), ("resnet18", 3, True)]
    qs = _small_queries(128, 64, seed=18)
    out = f.run(imgs, qs, threads=16)
    SEEDS_OLD = dict(SEEDS)
    try:
        SEEDS["resnet18"] = 999
        _check(out, imgs, qs)
    finally:
        SEEDS.update(SEEDS_OLD)
    assert f.state()["partitions"] == {"resnet18": [0, 1, 2, 3], "alexnet": [4, 5, 6, 7]}
