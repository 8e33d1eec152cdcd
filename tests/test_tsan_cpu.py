"""Race detection for the control plane: the same `dmlc-node` sources built
with -fsanitize=thread (`build/bin/dmlc-node-tsan`, see tools/build.py and
csrc/serve/executor_stub.cpp) driven through membership churn, SDFS
replication, predict jobs and a leader fail-over. Any ThreadSanitizer report
from any node fails the test.

The reference relied on Rust's ownership rules for data-race freedom
(src/membership.rs, src/services.rs use Arc<Mutex<..>> everywhere); a C++
control plane has no such guarantee, so it is checked dynamically instead.
"""
import os
import re
import subprocess
import time

import pytest

from dmlc import REPO_ROOT
from dmlc.serve.cluster import LocalCluster
from dmlc.utils.dataset import make_synthetic_dataset, synthetic_labels, write_labels

pytestmark = pytest.mark.slow

TSAN_BIN = os.path.join(REPO_ROOT, "build", "bin", "dmlc-node-tsan")
TSAN_ENV = {"TSAN_OPTIONS": "halt_on_error=0 second_deadlock_stack=1 report_signal_unsafe=0"}


@pytest.fixture(scope="module")
def tsan_bin():
    if not os.path.exists(TSAN_BIN):
        pytest.fail("dmlc-node-tsan not built (python tools/build.py)")
    return TSAN_BIN


def _no_reports(nodes):
    bad = [(nd.address, nd.output()) for nd in nodes if "ThreadSanitizer" in nd.output()]
    assert not bad, "\n\n".join(f"== {a}\n{o[-6000:]}" for a, o in bad)


def test_tsan_selftest(tsan_bin):
    r = subprocess.run([tsan_bin, "selftest"], capture_output=True, text=True, timeout=120,
                       env={**os.environ, **TSAN_ENV})
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failed" in r.stdout and "ThreadSanitizer" not in r.stderr, r.stderr[-6000:]


def _rows(text):
    return re.findall(r"\| (127\.0\.0\.1:\d+) ", text)


def test_tsan_cluster_workload(tsan_bin, tmp_path):
    labels = synthetic_labels(1000)
    lab = write_labels(str(tmp_path / "synset_words.txt"), labels)
    ds = make_synthetic_dataset(str(tmp_path / "train"), labels[:48], size=(48, 64))
    src = tmp_path / "data.txt"
    src.write_text("payload\n" * 1000)
    cl = LocalCluster(5, 19900, str(tmp_path / "c"), lab, n_leaders=2, executor="digest", dataset=ds,
                      models="resnet18=-,alexnet=-", binary=tsan_bin, env=TSAN_ENV,
                      extra=["--job-limit", "40", "--query-interval-ms", "100", "--quiet-predictions"])
    with cl:
        n = cl.nodes
        # SDFS traffic from several clients at once
        assert "Stored on:" in n[3].cmd(f"put {src} a.txt")
        assert "Stored on:" in n[4].cmd(f"put {src} a.txt")
        assert "Retrieved version: 2" in n[2].cmd(f"get a.txt {tmp_path / 'g.txt'}")
        # predict jobs on all members while two of them stage the dataset
        # into their executor cache; then kill a member and the leader mid-run
        n[3].cmd("prefetch")
        n[4].cmd("predict")
        n[1].cmd("prefetch")
        time.sleep(1.0)
        n[2].kill()
        time.sleep(1.0)
        n[0].kill()
        survivors = [n[1], n[3], n[4]]
        cl.wait_members(3, 40, survivors)
        deadline = time.time() + 90
        done = False
        while time.time() < deadline and not done:
            try:
                out = n[4].cmd("jobs", 20)
                tot = [int(q) for q in re.findall(r"Queries: (\d+) total", out)]
                done = len(tot) == 2 and all(q >= 40 for q in tot)
            except TimeoutError:
                pass
            time.sleep(1.0)
        assert done, n[4].output()[-4000:]
        assert f"leader {n[1].address}" in n[4].cmd("info")  # the standby took over mid-run
        # re-replication after two failures: every survivor (3 < RF=4) holds a replica
        deadline = time.time() + 30
        while time.time() < deadline:
            rows = _rows(n[1].cmd("ls a.txt"))
            if len(rows) == 3 and all(nd.address in rows for nd in survivors):
                break
            time.sleep(0.5)
        assert sorted(rows) == sorted(nd.address for nd in survivors), rows
        assert re.search(r"cache hits \d+ misses \d+ staged [1-9]", n[3].cmd("info")), n[3].cmd("info")
        assert "Leaving group" in n[3].cmd("leave")
        cl.wait_members(2, 20, [n[1], n[4]])
    _no_reports(n)


def test_tsan_adaptive_rate(tsan_bin, tmp_path):
    """Adaptive-rate jobs (per-job windows, least-outstanding routing over
    the shared per-member counts) with a member killed mid-run: no races."""
    labels = synthetic_labels(1000)
    lab = write_labels(str(tmp_path / "synset_words.txt"), labels)
    ds = make_synthetic_dataset(str(tmp_path / "train"), labels[:48], size=(48, 64))
    cl = LocalCluster(4, 19950, str(tmp_path / "c"), lab, n_leaders=1, executor="digest", dataset=ds,
                      models="resnet18=-,alexnet=-", binary=tsan_bin, env=TSAN_ENV,
                      extra=["--job-limit", "40", "--adaptive-window", "2", "--quiet-predictions"])
    with cl:
        n = cl.nodes
        time.sleep(1.0)
        n[0].cmd("predict")
        time.sleep(0.3)
        n[3].kill()
        deadline = time.time() + 90
        done = False
        while time.time() < deadline and not done:
            try:
                out = n[0].cmd("jobs", 20)
                tot = [int(q) for q in re.findall(r"Queries: (\d+) total", out)]
                done = len(tot) == 2 and all(q >= 40 for q in tot)
            except TimeoutError:
                pass
            time.sleep(0.5)
        assert done, n[0].output()[-4000:]
    _no_reports(n)
