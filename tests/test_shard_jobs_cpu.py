"""Predict jobs over SDFS-staged labelled u8 shards (BASELINE config 3), run
through the whole control plane under ThreadSanitizer (`dmlc-node-tsan`,
whose "digest" executor classifies an image as FNV-1a(pixels) % 1000).

Reference: `run_job` walks the dataset labels, sends each query to a member
of the job's set and scores correctness by label (src/services.rs:407-433);
the `jobs` report gives accuracy and latency percentiles (src/main.rs:271-314).
Here `predict <shard>` makes both jobs take their queries from the shard's
images instead: each query (a range of images of one shard) goes to a
replica holder, which classifies it from its resident copy (HBM on GPU
members), and image i of the shard is class label0 + i.

The shard's tiny images are crafted so that the digest of 12 of the 16 hits
its label: the report must say exactly 12/16 for both jobs, and every
printed prediction must be the digest's label text.
"""
import os
import re
import time

import numpy as np
import pytest

from dmlc import REPO_ROOT
from dmlc.serve.cluster import LocalCluster
from dmlc.utils.dataset import make_synthetic_dataset, synthetic_labels, write_labels
from dmlc.utils.shards import shard_info, write_shard

pytestmark = pytest.mark.slow

TSAN_BIN = os.path.join(REPO_ROOT, "build", "bin", "dmlc-node-tsan")
TSAN_ENV = {"TSAN_OPTIONS": "halt_on_error=0 second_deadlock_stack=1 report_signal_unsafe=0"}
FNV_OFF, FNV_PRIME = np.uint64(1469598103934665603), np.uint64(1099511628211)


def _fnv_state(b: np.ndarray) -> np.uint64:
    h = FNV_OFF
    with np.errstate(over="ignore"):
        for v in b.tolist():
            h = (h ^ np.uint64(v)) * FNV_PRIME
    return h


def _digest(img: np.ndarray) -> int:
    return int(_fnv_state(img.reshape(-1)) % np.uint64(1000))


def _craft(target: int, rng) -> np.ndarray:
    """An 8x8 RGB image whose digest is `target` (the last two bytes searched)."""
    for _ in range(64):
        img = rng.integers(0, 256, size=(8, 8, 3), dtype=np.uint8)
        flat = img.reshape(-1)
        h = _fnv_state(flat[:-2])
        a = np.arange(256, dtype=np.uint64)
        with np.errstate(over="ignore"):
            h1 = (h ^ a) * FNV_PRIME                                    # [256]
            h2 = (h1[:, None] ^ a[None, :]) * FNV_PRIME                 # [256, 256]
        hit = np.argwhere(h2 % np.uint64(1000) == np.uint64(target))
        if len(hit):
            flat[-2], flat[-1] = hit[0]
            assert _digest(img) == target
            return img
    raise RuntimeError("no image found")


@pytest.fixture(scope="module")
def tsan_bin():
    if not os.path.exists(TSAN_BIN):
        pytest.fail("dmlc-node-tsan not built (python tools/build.py)")
    return TSAN_BIN


def _no_reports(nodes):
    bad = [(nd.address, nd.output()) for nd in nodes if "ThreadSanitizer" in nd.output()]
    assert not bad, "\n\n".join(f"== {a}\n{o[-6000:]}" for a, o in bad)


def _wait_jobs(node, want, timeout=90):
    deadline = time.time() + timeout
    out = ""
    while time.time() < deadline:
        out = node.cmd("jobs", 20)
        blocks = re.split(r"^Job \d+:", out, flags=re.M)[1:]
        done = []
        for b in blocks:
            m = re.search(r"Accuracy: \d+/(\d+)", b)
            u = re.search(r"Unanswered: (\d+)", b)
            done.append((int(m.group(1)) if m else 0) + (int(u.group(1)) if u else 0))
        if len(done) == 2 and all(d >= w for d, w in zip(done, want)):
            return out
        time.sleep(0.3)
    raise AssertionError(out + "\n" + node.output()[-4000:])


def test_jobs_over_labelled_shard(tsan_bin, tmp_path):
    labels = synthetic_labels(1000)
    lab = write_labels(str(tmp_path / "synset_words.txt"), labels)
    ds = make_synthetic_dataset(str(tmp_path / "train"), labels[:4], size=(48, 64))
    rng = np.random.default_rng(5)
    label0, n = 100, 16
    targets = [label0 + i if i % 4 else (label0 + i + 500) % 1000 for i in range(n)]  # 12 right, 4 wrong
    imgs = np.stack([_craft(t, rng) for t in targets])
    shard = write_shard(str(tmp_path / "val.u8s"), imgs, label0=label0)
    assert shard_info(shard) == {"n": 16, "h": 8, "w": 8, "label0": 100}
    cl = LocalCluster(3, 20700, str(tmp_path / "c"), lab, n_leaders=2, executor="digest", dataset=ds,
                      models="resnet18=-,alexnet=-", binary=tsan_bin, env=TSAN_ENV,
                      extra=["--query-batch", "3", "--adaptive-window", "2"])
    with cl:
        nd = cl.nodes
        assert "Stored on:" in nd[2].cmd(f"put {shard} val.u8s")
        deadline = time.time() + 30
        while time.time() < deadline and not all("val.u8s@v1" in x.cmd("replicas") for x in nd):
            time.sleep(0.2)
        mark = nd[1].mark()
        nd[1].cmd("predict val.u8s")
        out = _wait_jobs(nd[1], [n, n])
        assert len(re.findall(r"Accuracy: 12/16 = 75\.00%", out)) == 2, out
        assert len(re.findall(r"Data: SDFS shards val\.u8s", out)) == 2, out
        time.sleep(0.5)
        lines = re.findall(r"^(resnet18|alexnet) - (n\d+): (.*?) \(100\.00%\)( \(should be .*\))?$",
                           nd[0].output(), re.M)
        wnid_label = dict(labels)
        seen = {}
        for model, wnid, got, wrong in lines:
            i = [w for w, _ in labels].index(wnid) - label0
            assert 0 <= i < n
            assert got == labels[targets[i]][1], (model, wnid, got)
            assert bool(wrong) == (targets[i] != label0 + i)
            seen[(model, i)] = got
        assert len(seen) == 2 * n, sorted(seen)
        assert wnid_label  # labels table loaded
        # `predict` again resumes (nothing left); `predict dataset` switches
        # the jobs back to the per-label JPEGs and starts them over
        nd[1].cmd("predict dataset")
        out = _wait_jobs(nd[1], [4, 4])
        assert "Data: SDFS shards" not in out
        del mark
    _no_reports(nd)


def test_unservable_queries_are_dropped_not_retried_forever(tsan_bin, tmp_path):
    """A job whose model no member can serve: each query is tried on the
    members, requeued with a back-off, and dropped after --max-attempts
    sends in all; the job ends and reports the images as unanswered (the
    reference dropped failed queries) while the other job completes."""
    labels = synthetic_labels(1000)
    lab = write_labels(str(tmp_path / "synset_words.txt"), labels)
    ds = make_synthetic_dataset(str(tmp_path / "train"), labels[:6], size=(48, 64))
    cl = LocalCluster(2, 20760, str(tmp_path / "c"), lab, n_leaders=1, executor="digest", dataset=ds,
                      models="resnet18=-", binary=tsan_bin, env=TSAN_ENV,
                      extra=["--job-limit", "6", "--query-interval-ms", "20", "--max-attempts", "2",
                             "--quiet-predictions"])
    with cl:
        nd = cl.nodes
        time.sleep(1.0)
        nd[0].cmd("predict")
        out = _wait_jobs(nd[0], [6, 6])
        assert re.search(r"Model: resnet18\n\tAccuracy: \d+/6", out), out
        assert re.search(r"Model: alexnet\n\tAccuracy: 0/0 .*\n.*\n.*\n\tUnanswered: 6 images", out), out
    _no_reports(nd)


def test_shard_job_loops_to_job_limit(tsan_bin, tmp_path):
    """Sustained runs (tools/bench_jobs.py --job-limit): a shard job whose
    --job-limit exceeds its shards' images loops over them, each image scored
    against its own label on every pass: 40 queries over the 16-image shard
    = 2.5 passes, 12 + 12 + 6 right."""
    labels = synthetic_labels(1000)
    lab = write_labels(str(tmp_path / "synset_words.txt"), labels)
    ds = make_synthetic_dataset(str(tmp_path / "train"), labels[:4], size=(48, 64))
    rng = np.random.default_rng(6)
    label0, n = 200, 16
    targets = [label0 + i if i % 4 else (label0 + i + 500) % 1000 for i in range(n)]
    imgs = np.stack([_craft(t, rng) for t in targets])
    shard = write_shard(str(tmp_path / "loop.u8s"), imgs, label0=label0)
    cl = LocalCluster(2, 20820, str(tmp_path / "c"), lab, n_leaders=1, executor="digest", dataset=ds,
                      models="resnet18=-,alexnet=-", binary=tsan_bin, env=TSAN_ENV,
                      extra=["--query-batch", "3", "--adaptive-window", "2", "--job-limit", "40",
                             "--quiet-predictions"])
    with cl:
        nd = cl.nodes
        assert "Stored on:" in nd[1].cmd(f"put {shard} loop.u8s")
        deadline = time.time() + 30
        while time.time() < deadline and not all("loop.u8s@v1" in x.cmd("replicas") for x in nd):
            time.sleep(0.2)
        nd[0].cmd("predict loop.u8s")
        out = _wait_jobs(nd[0], [40, 40])
        assert len(re.findall(r"Accuracy: 30/40 = 75\.00%", out)) == 2, out
    _no_reports(nd)
