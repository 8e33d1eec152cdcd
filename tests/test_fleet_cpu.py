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


# ---------------------------------------------------------------- coalescing
# The reference runs each query as its own batch-1 forward under the model's
# mutex (src/services.rs:475-497); SURVEY.md §7.6 #12 asks for real batching.
# Concurrent direct queries to one (model, GPU) instance queue there and
# share forwards of up to max_per_rank images.

def _coalescing_fleet(devices=1, jobs=("resnet18",), max_per_rank=16, window_us=50000, eager=False, delay_us=2000,
                      lanes=2):
    f = C.HostFleet(list(range(devices)), H, W, lanes, delay_us, max_per_rank, 4, SEEDS,
                    batch_window_us=window_us, eager_when_idle=eager)
    f.set_jobs(list(jobs))
    for m in jobs:
        f.load(m)
    return f


@pytest.mark.parametrize("n", [16, 40, 64])
def test_concurrent_single_image_queries_share_forwards(n):
    """n concurrent 1-image queries on one GPU: at most ceil(n / max) forwards,
    every answer exactly once and in order."""
    # a 200 ms window: starting n threads on a loaded host can take longer than the default 50 ms
    f = _coalescing_fleet(window_us=200000)
    imgs = _imgs(n, seed=20)
    qs = [("resnet18", i, 1) for i in range(n)]
    out = f.run(imgs, qs, threads=n)
    _check(out, imgs, qs)
    st = f.state()
    assert st["served"]["resnet18"][0] == n
    assert st["forwards"]["resnet18"][0] <= -(-n // 16), st["forwards"]


def test_eager_idle_first_query_goes_alone_then_batches():
    """Serving default: an idle instance runs the first query at once (no
    batching delay for a lone query); queries arriving while it runs batch."""
    f = _coalescing_fleet(eager=True, window_us=20000, delay_us=20000)
    imgs = _imgs(33, seed=21)
    qs = [("resnet18", i, 1) for i in range(33)]
    out = f.run(imgs, qs, threads=33)
    _check(out, imgs, qs)
    st = f.state()
    fw = st["forwards"]["resnet18"][0]
    # the lone first (a size-1 forward), the rest batched: 1 + ceil(32 / 16)
    # on an idle host; thread start-up on a loaded one spreads the arrivals
    # over a few more 20 ms forwards (5 measured), never 33
    assert st["forward_sizes"]["resnet18"].get(1, 0) >= 1, st["forward_sizes"]
    assert fw <= 8, fw
    # a lone query on an idle instance: one forward, no window wait
    out = f.run(imgs, [("resnet18", 3, 1)], threads=1)
    _check(out, imgs, [("resnet18", 3, 1)])


def test_large_query_chunks_run_on_every_lane():
    """A direct query bigger than max_per_rank is cut into max-sized chunks
    queued together: one forward per chunk, issued on both lanes at once."""
    f = _coalescing_fleet(window_us=0, delay_us=1000)
    imgs = _imgs(5 * 16 + 3, seed=22)
    qs = [("resnet18", 0, 5 * 16 + 3)]
    out = f.run(imgs, qs, threads=1)
    _check(out, imgs, qs)
    assert f.state()["forwards"]["resnet18"][0] == 6


def test_coalesced_queries_mixed_sizes_exactly_once_in_order():
    f = _coalescing_fleet(devices=4, jobs=("resnet18", "alexnet"), window_us=2000, delay_us=1500)
    imgs = _imgs(400, seed=23)
    qs = _small_queries(400, 200, seed=24, max_n=12)
    out = f.run(imgs, qs, threads=48)
    _check(out, imgs, qs)
    st = f.state()
    for model in ("resnet18", "alexnet"):
        imgs_model = sum(c for m, _, c in qs if m == model)
        assert sum(st["served"][model].values()) == imgs_model
        assert sum(st["forwards"][model].values()) < sum(1 for m, _, _ in qs if m == model)  # some shared


def test_coalesced_queries_survive_gpu_failure_exactly_once():
    """A GPU dies while coalesced batches are queued and running on it: every
    query is still answered exactly once and in order (the lost GPU's
    requests are redone on the rebalanced fleet)."""
    f = _coalescing_fleet(devices=4, jobs=("resnet18", "alexnet"), window_us=3000, delay_us=2000)
    imgs = _imgs(300, seed=25)
    qs = [("resnet18" if i % 3 else "alexnet", (7 * i) % 290, 1 + i % 4) for i in range(150)]
    f.fail(1)
    out = f.run(imgs, qs, threads=40)
    _check(out, imgs, qs)
    st = f.state()
    assert 1 not in st["live"]
    assert any(r["retries"] > 0 for r in out["routes"])
    assert st["partitions"] == {"resnet18": [0], "alexnet": [2, 3]}


def test_failed_worker_build_keeps_serving_and_retries():
    """A worker build that fails during a rebalance (OOM, HIP error) leaves
    the model on its old GPUs without a group: queries still run (direct, no
    scatter through a half-built group) and the next query retries the
    rebalance (fleet.cpp:270)."""
    f = _fleet(delay_us=0)
    f.fail_next_builds(1)
    with pytest.raises(Exception):
        f.lose(5)  # GPU 3 moves to alexnet: its replica build fails
    imgs = _imgs(200, seed=26)
    qs = [("alexnet", 0, 100), ("resnet18", 10, 3), ("alexnet", 5, 2)]
    out = f.run(imgs, qs, threads=3)  # rebalances again first (build succeeds now)
    _check(out, imgs, qs)
    st = f.state()
    assert st["partitions"] == {"resnet18": [0, 1, 2], "alexnet": [3, 4, 6, 7]}
    assert st["overlapping_worlds"] == []


# ------------------------------------------------- shard replica placement
@pytest.mark.parametrize("n,parts,want", [
    # two jobs on disjoint halves: one full copy per partition, sliced over its GPUs
    (1000, [[0, 1, 2, 3], [4, 5, 6, 7]],
     [(0, d, 250 * d, 250) for d in range(4)] + [(1, 4 + d, 250 * d, 250) for d in range(4)]),
    # after a loss the partitions are uneven (first floor(7/2) to job 1)
    (10, [[0, 1, 2], [3, 4, 6, 7]], [(0, 0, 0, 3), (0, 1, 3, 3), (0, 2, 6, 4),
                                     (1, 3, 0, 2), (1, 4, 2, 3), (1, 6, 5, 2), (1, 7, 7, 3)]),
    # fewer GPUs than jobs: both models share GPU 0 -> one copy
    (7, [[0], [0]], [(0, 0, 0, 7)]),
    # a partition's GPUs are taken in sorted order; copies follow the partitions
    (4, [[3, 2], [1, 0]], [(0, 2, 0, 2), (0, 3, 2, 2), (1, 0, 0, 2), (1, 1, 2, 2)]),
])
def test_shard_placement_one_copy_per_partition(n, parts, want):
    """A staged shard replica is held in HBM once per serving partition,
    sliced over that partition's GPUs, so each model reads every image of
    its queries from a GPU it serves on (GPU executor stage_blob; both jobs
    run over the same shards)."""
    got = C.shard_placement(n, parts)
    assert got == want
    for c in {p[0] for p in got}:  # every copy covers the shard exactly once
        cover = sorted((f, k) for cc, _, f, k in got if cc == c)
        assert cover[0][0] == 0 and all(a[0] + a[1] == b[0] for a, b in zip(cover, cover[1:]))
        assert cover[-1][0] + cover[-1][1] == n


@pytest.mark.parametrize("b,want", [(1, 1), (3, 4), (33, 64), (64, 64), (65, 96), (129, 160), (200, 224),
                                    (225, 256), (256, 256)])
def test_bucket_batch_pow2_then_multiples_of_32(b, want):
    """Forward sizes: powers of two up to 64, then multiples of 32 (VERDICT r4
    item 7: a 129-image coalesced forward used to pay for 256)."""
    assert C.fleet_bucket_batch(b, 256) == want


def test_coalesced_forward_sizes_are_buckets():
    """Forwards of 1..max coalesced images run at the bucketed sizes only; a
    lone 129-image query runs one 160-image forward."""
    f = _coalescing_fleet(max_per_rank=256, window_us=0, delay_us=0)
    imgs = _imgs(300, seed=27)
    qs = [("resnet18", 0, 129)]
    out = f.run(imgs, qs, threads=1)
    _check(out, imgs, qs)
    assert f.state()["forward_sizes"]["resnet18"] == {160: 1}
    qs = [("resnet18", i, 1 + i % 7) for i in range(60)]
    out = f.run(imgs, qs, threads=24)
    _check(out, imgs, qs)
    allowed = {1, 2, 4, 8, 16, 32, 64} | set(range(96, 257, 32))
    assert set(f.state()["forward_sizes"]["resnet18"]) <= allowed


def test_stage_error_in_a_shared_forward_fails_that_query_only():
    """One query whose stage throws (a bad image) inside a coalesced forward:
    it alone gets the error, every other query sharing the forward is
    answered exactly once (the failure used to be published
    outside the instance lock while the failing request stayed in the flight,
    a use-after-free once its owner returned)."""
    f = _coalescing_fleet(devices=1, max_per_rank=32, window_us=3000, delay_us=1500)
    imgs = _imgs(200, seed=28)
    qs = [("resnet18", (5 * i) % 190, 1 + i % 3) for i in range(90)]
    bad = list(range(0, 90, 7))
    for _ in range(3):
        out = f.run(imgs, qs, threads=30, bad=bad)
        for q, (model, first, count) in enumerate(qs):
            if q in bad:
                assert "bad image size" in out["errors"][q]
                continue
            assert out["errors"][q] == "", out["errors"][q]
            ei, ep = _expect(imgs[first:first + count], model)
            np.testing.assert_array_equal(out["idx"][q], ei)
            np.testing.assert_array_equal(out["prob"][q], ep)


@pytest.mark.parametrize("san", ["tsan", "asan"])
def test_coalescing_under_sanitizers(san):
    """The coalesced direct path (concurrent small queries, some failing in
    their stage, a GPU lost halfway) under ThreadSanitizer and under
    AddressSanitizer+UBSan (csrc/tests/fleet_stress.cpp). With the round-4
    code (a stage failure published outside the instance lock) TSan reports
    races on Req::state and ASan a heap-use-after-free in Fleet::direct."""
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "build", "bin",
                       f"dmlc-fleet-stress-{san}")
    if not os.path.exists(exe):
        pytest.fail(f"{exe} not built (python tools/build.py)")
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 exitcode=66", ASAN_OPTIONS="detect_leaks=1")
    r = subprocess.run([exe, "300", "16"], capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "WARNING" not in r.stderr and "ERROR" not in r.stderr, r.stderr[-4000:]
    assert " 0 wrong" in r.stdout, r.stdout
