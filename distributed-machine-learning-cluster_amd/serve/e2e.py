"""End-to-end query latency with the reference's definition.

The reference times each query from before the TCP connect to the member
until its answer is back: connect + RPC + JPEG decode + resize + forward +
softmax/top-1 (``Instant`` around ``MemberClient::spawn(..).predict(..)``,
src/services.rs:419-424; published mean 158.94 ms for ResNet18,
CS425MP4Report.pdf p.2). This runs the same thing through this framework: a
one-node cluster (a new TCP connection per query, as the reference's
``MemberClient::spawn``; the default reuses pooled connections) (leader + member with the GPU executor) runs a ResNet18
predict job with one query in flight at a time (``--adaptive-window 1``,
batch 1), over JPEGs that are decoded per query (no HBM prefetch), and the
leader records every query's latency exactly as the reference's job does.
"""
from __future__ import annotations

import json
import os
import re
import shutil
import statistics
import tempfile
import time

from .. import REPO_ROOT
from ..utils.dataset import make_synthetic_dataset, synthetic_labels, write_labels
from ..utils.ot import write_random_checkpoint
from .cluster import LocalCluster

REAL_SUBSET = os.path.join(REPO_ROOT, "data", "imagenet_1k_subset", "train")
REAL_LABELS = os.path.join(REPO_ROOT, "data", "synset_words.txt")


def _pct(xs, q):
    xs = sorted(xs)
    k = (len(xs) - 1) * q / 100
    lo, hi = int(k), min(int(k) + 1, len(xs) - 1)
    return xs[lo] + (xs[hi] - xs[lo]) * (k - lo)


def query_latency(n: int = 200, model: str = "resnet18", device: int = 0, port: int = 23500,
                  dataset: str | None = None, labels: str | None = None, skip: int = 5,
                  timeout: float = 180.0, executor: str = "gpu") -> dict:
    """Per-query latency (ms) of a predict job through the whole control
    plane. Uses the reference's real JPEGs when ``data/imagenet_1k_subset``
    is present (tools/make_subset.py), else synthetic 500x375 JPEGs."""
    root = tempfile.mkdtemp(prefix="dmlc_e2e_")
    try:
        if dataset is None and os.path.isdir(REAL_SUBSET) and os.path.exists(REAL_LABELS):
            dataset, labels = REAL_SUBSET, REAL_LABELS
        if dataset:
            n = min(n, len(os.listdir(dataset)))
            desc = f"real imagenet_1k JPEGs from the reference ({n})"
        else:
            ents = synthetic_labels(1000)
            labels = write_labels(os.path.join(root, "synset_words.txt"), ents)
            dataset = make_synthetic_dataset(os.path.join(root, "train"), ents[:n], size=(375, 500))
            desc = f"synthetic 500x375 JPEGs ({n})"
        ckpt = write_random_checkpoint(model, os.path.join(root, f"{model}.ot"), seed=0)
        extra = ["--jobs", model, "--job-limit", str(n), "--adaptive-window", "1", "--query-batch", "1",
                 "--quiet-predictions", "--device", str(device), "--max-batch", "8", "--new-conn-per-query"]
        cl = LocalCluster(1, port, os.path.join(root, "c"), labels, n_leaders=1, executor=executor,
                          dataset=dataset, models=f"{model}={ckpt}", extra=extra)
        with cl:
            nd = cl.nodes[0]
            time.sleep(1.0)  # one assignment round (fast periods: 500 ms)
            nd.cmd("predict")
            deadline = time.time() + timeout
            while time.time() < deadline:
                m = re.search(r"Accuracy: \d+/(\d+)", nd.cmd("jobs"))
                if m and int(m.group(1)) >= n:
                    break
                time.sleep(0.25)
            dump = os.path.join(root, "jobs.json")
            nd.cmd(f"jobs-dump {dump}")
            jobs = json.load(open(dump))
        d = [x / 1000 for x in jobs[0]["durations_us"]][skip:]
        if not d:
            raise RuntimeError("no query completed")
        return {"n": len(d), "mean_ms": statistics.mean(d), "p50_ms": _pct(d, 50), "p95_ms": _pct(d, 95),
                "p99_ms": _pct(d, 99), "data": desc}
    finally:
        shutil.rmtree(root, ignore_errors=True)
