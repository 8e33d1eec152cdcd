"""Native data-parallel layer (csrc/comm/dp.cpp) on the in-process host fake
communicator: the same Rank / pipeline / Group code that drives RCCL on the
GPUs, with a deterministic CPU classifier (class = byte sum % 1000).

Checks shard order (every answer lands at its image's position), exactly-once
commits, ragged last steps, the one-thread-per-rank (multi-process) issue
order, local mode, and recovery from the loss of a non-coordinator rank —
both a drained drop and an abrupt death that surfaces as a communicator
error (reference behaviour being replaced: queries re-sent to a surviving
member after a failure, src/services.rs:199-211, 407-433)."""
import numpy as np
import pytest

import dmlc

C = dmlc.native()
H = W = 8


def _images(n, seed=0):
    rng = np.random.default_rng(seed)
    return rng.integers(0, 256, size=(n, H, W, 3), dtype=np.uint8)


def _expected(imgs):
    flat = imgs.reshape(imgs.shape[0], -1).astype(np.int64)
    return (flat.sum(1) % 1000).astype(np.int32), ((imgs[:, 0, 0, 0].astype(np.float32) + 1) / 257)


def _check(out, imgs):
    ei, ep = _expected(imgs)
    np.testing.assert_array_equal(out["idx"], ei)
    np.testing.assert_allclose(out["prob"], ep, rtol=0, atol=0)
    np.testing.assert_array_equal(out["commits"], np.ones(len(imgs), np.int32))


def test_shard_counts():
    assert C.dp_shard_counts(10, 4, 3) == [3, 3, 2, 2]
    assert C.dp_shard_counts(8, 8, 1) == [1] * 8
    assert C.dp_shard_counts(0, 3, 5) == [0, 0, 0]
    with pytest.raises(ValueError):
        C.dp_shard_counts(13, 4, 3)


@pytest.mark.parametrize("world", [1, 2, 3, 5, 8])
@pytest.mark.parametrize("n", [1, 7, 64, 101])
def test_group_exactly_once_in_order(world, n):
    imgs = _images(n, seed=world * 1000 + n)
    out = C.dp_host_run(imgs, world, 4, mode="group")
    _check(out, imgs)
    assert out["stats"]["recoveries"] == 0
    assert out["stats"]["steps"] == -(-n // (4 * world))


@pytest.mark.parametrize("world", [2, 3, 4, 8])
@pytest.mark.parametrize("scatter", [True, False])
@pytest.mark.parametrize("pipelined", [True, False])
def test_threads_one_rank_per_thread(world, scatter, pipelined):
    """One thread per rank = the multi-process issue order (each rank's
    pipeline runs independently; groups pair up across threads)."""
    n = 4 * world * 5 + 3  # ragged last step
    imgs = _images(n, seed=world)
    out = C.dp_host_run(imgs, world, 4, mode="threads", scatter=scatter, pipelined=pipelined)
    _check(out, imgs)
    assert all(s == out["steps"][0] for s in out["steps"])


@pytest.mark.parametrize("world", [1, 2, 4])
@pytest.mark.parametrize("slots", [3, 4])
@pytest.mark.parametrize("steps", [1, 2, 3, 7])
def test_threads_deeper_pipeline(world, slots, steps):
    """Ranks with 3-4 slots (bench.py --lanes 3/4: that many steps in
    flight, the host collecting step i-(slots-1)): every image answered
    exactly once, including runs shorter than the pipeline depth."""
    n = 4 * world * steps
    imgs = _images(n, seed=40 + slots + steps)
    out = C.dp_host_run(imgs, world, 4, mode="threads", slots=slots)
    _check(out, imgs)
    assert out["steps"] == [steps] * world


@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("abrupt", [False, True])
@pytest.mark.parametrize("after", [0, 1, 3])
def test_group_survives_rank_loss(world, abrupt, after):
    n = 4 * world * 6 + 1
    imgs = _images(n, seed=7 + world)
    lost = world - 1 if world > 2 else 1
    out = C.dp_host_run(imgs, world, 4, mode="group", fail_member=lost, fail_after=after, abrupt=abrupt)
    _check(out, imgs)
    st = out["stats"]
    assert st["recoveries"] == 1
    assert lost not in out["members"]
    assert len(out["members"]) == world - 1
    # the communicators were rebuilt over the survivors, coordinator first
    # (a lone survivor needs none)
    if len(out["members"]) > 1:
        assert out["builds"][-1] == out["members"]
        assert out["builds"][-1][0] == 0
    if abrupt:
        assert st["redone_images"] > 0  # the step that hit the dead rank is redone


def test_group_loss_down_to_coordinator_alone():
    imgs = _images(50, seed=3)
    out = C.dp_host_run(imgs, 2, 4, mode="group", fail_member=1, fail_after=2, abrupt=True)
    _check(out, imgs)
    assert out["members"] == [0]


def test_group_rejects_coordinator_failure():
    imgs = _images(10)
    with pytest.raises(ValueError):
        C.dp_host_run(imgs, 3, 4, mode="group", fail_member=0)


# ---- the host fake behaves like RCCL point-to-point, not like a mailbox

def test_fake_is_rendezvous_a_misordered_exchange_times_out():
    """Both ranks send before they receive: RCCL would hang (a send needs its
    receive posted), and so must the fake (it used to buffer the sends and
    pass). Both sides fail with a timeout and nothing is left posted."""
    bad = C.host_order_probe(bad=True, timeout_ms=300)
    assert "timed out" in bad["err0"] and "timed out" in bad["err1"], bad
    assert not bad["ok"]
    assert bad["pending"] == 0
    good = C.host_order_probe(bad=False, timeout_ms=2000)
    assert good["err0"] == "" and good["err1"] == "" and good["ok"], good
    assert good["pending"] == 0


# ---- bench.py's per-rank protocol, one thread per rank (= one process per GPU)

@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("mode", ["scatter", "staged"])
@pytest.mark.parametrize("weight", [1.0, 0.85])
def test_bench_protocol(world, mode, weight):
    """stage (staged mode), prime run, warmup, timed run and the unpipelined
    latency run, exactly as bench.py issues them, with the coordinator's
    shard weighted down (--coord-weight): every rank runs every step and the
    coordinator's last answers are its images' classes in global order."""
    per = 6
    counts = C.dp_weighted_counts(per, world, weight)
    G = sum(counts)
    assert counts[1:] == [per] * (world - 1) and counts[0] == (per if world == 1 or weight == 1.0 else 5)
    pool = np.random.default_rng(world).integers(0, 256, size=(2 * G, H, W, 3), dtype=np.uint8)
    out = C.dp_host_bench(pool, world, per, coord_weight=weight, input_mode=mode, lanes=2, prime=4, warmup=3,
                          steps=7, latency=2)
    assert out["answers_ok"]
    assert out["steps"] == [[4, 3, 7, 2]] * world
    assert out["counts"] == counts


@pytest.mark.parametrize("per,world,w,want", [
    (256, 8, 1.0, [256] * 8),
    (256, 8, 0.85, [218] + [256] * 7),   # the others never above 256: no second, nearly empty round
    (256, 2, 0.5, [128, 256]),
    (10, 1, 0.5, [10]),
])
def test_weighted_counts(per, world, w, want):
    assert C.dp_weighted_counts(per, world, w) == want


def test_weighted_counts_rejects_raising_the_coordinator():
    with pytest.raises(ValueError):
        C.dp_weighted_counts(256, 8, 1.2)


# ---- coordinator share calibration (bench.py at N > 1, and dp::Group)

def test_calibration_equalises_coordinator_and_worker_forward_times():
    """bench.py's calibration on the host fake: the coordinator's forward is
    slowed by a fixed 3 ms per step (standing for the CUs its scatter legs'
    copy kernels take on a GPU) on top of 0.4 ms per image (sleeps long
    enough that host scheduling noise stays small next to them). Starting from an
    even split, the calibration rounds converge to the count whose forward
    time matches the other ranks' within 5%, and the timed run then uses it
    (every rank computing the same counts from the gathered times)."""
    world, per = 4, 20
    counts = C.dp_weighted_counts(per, world, 1.0)
    pool = np.random.default_rng(5).integers(0, 256, size=(2 * sum(counts), H, W, 3), dtype=np.uint8)
    out = C.dp_host_bench(pool, world, per, coord_weight=1.0, input_mode="scatter", lanes=2, prime=2, warmup=2,
                          steps=4, latency=1, us_per_image=400, coord_extra_us=3000, calib_rounds=6, calib_steps=4)
    assert out["answers_ok"]
    cal = out["calibration"]
    rounds = cal["rounds"]
    # The host worker's events read a synthetic device clock (forward cost =
    # us_per_image * B + extra_us), so the calibration is exact: round 0 runs
    # the even split (20 * 0.4 + 3 = 11 vs 8 ms per step), round 1 the first
    # estimate (c0 = 15: 9 vs 8), round 2 c0 = 13 (8.2 vs 8, within 5%).
    got = [v for r in rounds for v in (r["weight"], r["busy_coord_ms"], r["busy_worker_ms"])]
    assert got == pytest.approx([1.0, 11.0, 8.0, 8 / 11, 9.0, 8.0, 0.6464646, 8.2, 8.0], rel=1e-6)
    assert cal["weight"] == pytest.approx(0.6464646, rel=1e-6)
    assert out["counts"] == [13, 20, 20, 20]
    assert all(len(s) == 4 and s == out["steps"][0] for s in out["steps"])


def test_calibration_keeps_an_even_split_without_interference():
    world, per = 3, 12
    pool = np.random.default_rng(6).integers(0, 256, size=(2 * per * world, H, W, 3), dtype=np.uint8)
    out = C.dp_host_bench(pool, world, per, coord_weight=1.0, lanes=2, prime=2, warmup=1, steps=3, latency=1,
                          us_per_image=300, coord_extra_us=0, calib_rounds=4, calib_steps=3)
    assert out["answers_ok"]
    assert out["calibration"]["weight"] == 1.0
    assert out["counts"] == [12, 12, 12]


@pytest.mark.parametrize("n,world,cap,w0,want", [
    (64, 4, 16, 1.0, [16, 16, 16, 16]),
    (59, 4, 16, 0.75, [12, 16, 16, 15]),
    (20, 4, 16, 0.5, [3, 6, 6, 5]),
    (60, 4, 16, 0.75, [12, 16, 16, 16]),
])
def test_weighted_shards(n, world, cap, w0, want):
    got = C.dp_weighted_shards(n, world, cap, w0)
    assert sum(got) == n and all(0 <= c <= cap for c in got)
    assert got == want


def test_group_auto_balances_the_coordinator_share():
    """Serving scatters (dp::Group): each classify re-estimates the
    coordinator's share from per-image forward times; with the coordinator
    slowed as above the weight falls from 1.0 towards the equal-time point
    (0.53 here) and every answer is still committed exactly once."""
    imgs = _images(16 * 4 * 4, seed=31)
    out = C.dp_host_run(imgs, 4, 16, mode="group", us_per_image=400, coord_extra_us=3000, repeats=6)
    _check(out, imgs)
    w = out["coord_weights"]
    # exact (synthetic device clock, see above): falls monotonically towards
    # the equal-time point
    assert w == pytest.approx([0.84042553, 0.71751006, 0.63945679, 0.58966704, 0.55598002, 0.53605453], rel=1e-6)
    flat = C.dp_host_run(imgs, 4, 16, mode="group", us_per_image=400, coord_extra_us=0, repeats=3)
    _check(flat, imgs)
    assert flat["coord_weights"] == [1.0, 1.0, 1.0]


def test_fake_group_may_span_several_communicators():
    """RCCL lets one group hold operations of several communicators, posted in
    any order by the peers; the host fake used to refuse such a group (a
    stricter fake would fail only in CPU tests). Now it posts into every
    world before waiting on any."""
    out = C.host_multi_world_probe(timeout_ms=2000)
    assert out["err0"] == "" and out["err1"] == "" and out["ok"], out
    assert out["pending"] == 0
