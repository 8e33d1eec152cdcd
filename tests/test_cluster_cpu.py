"""Control plane end to end on one machine: N `dmlc-node` processes on
localhost (CPU executor), driven through their stdin REPL.

The reference had no such harness (manual tests on 10 VMs);
these tests cover its behaviours: join/ring membership and failure
detection, SDFS put/get/ls/store/get-versions/delete with replication factor
4 and re-replication after a failure, predict jobs with fair-share
assignment, `jobs`/`assign` reports, and leader fail-over with job resume.
"""
import os
import re
import subprocess
import time

import pytest
import torch

import dmlc
from dmlc.serve.cluster import NODE_BIN, LocalCluster
from dmlc.utils.dataset import make_synthetic_dataset, synthetic_labels, write_labels
from dmlc.utils.ot import write_random_checkpoint

pytestmark = pytest.mark.slow


@pytest.fixture(scope="module")
def env(tmp_path_factory):
    if not os.path.exists(NODE_BIN):
        pytest.fail("dmlc-node not built (python tools/build.py)")
    root = tmp_path_factory.mktemp("cluster")
    labels = synthetic_labels(1000)
    lab = write_labels(str(root / "synset_words.txt"), labels)
    ds = make_synthetic_dataset(str(root / "train"), labels[:48], size=(120, 160))
    models = {
        "resnet18": write_random_checkpoint("resnet18", str(root / "resnet18.ot"), seed=1),
        "alexnet": write_random_checkpoint("alexnet", str(root / "alexnet.ot"), seed=2),
    }
    return {"root": root, "labels": lab, "dataset": ds, "models": models, "entries": labels}


def test_selftest():
    r = subprocess.run([NODE_BIN, "selftest"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failed" in r.stdout


def test_classify_cpu_matches_reference(env):
    """Single-image classification from a .ot checkpoint on the CPU executor
    (BASELINE config: 'AlexNet single-image classify on CPU via libtorch .ot
    load'), checked against the torch.nn reference on the same decoded
    pixels and the same resize rule."""
    import torch.nn.functional as F
    from dmlc.models import build
    wnid = env["entries"][3][0]
    d = os.path.join(env["dataset"], wnid)
    img_path = os.path.join(d, sorted(os.listdir(d))[0])
    r = subprocess.run([NODE_BIN, "classify", "--model", "alexnet", "--weights", env["models"]["alexnet"],
                        "--labels", env["labels"], "--image", img_path, "--executor", "cpu"],
                       capture_output=True, text=True, timeout=120, env={**os.environ, "OMP_NUM_THREADS": "4"})
    assert r.returncode == 0, r.stderr
    m = re.search(r"class=(\d+)", r.stdout)
    assert m, r.stdout
    rgb = torch.from_numpy(dmlc.native().decode_jpeg(open(img_path, "rb").read())).float()
    H, W = rgb.shape[:2]
    rh, rw = (224, 224 * W // H) if H <= W else (224 * H // W, 224)
    x = F.interpolate(rgb.permute(2, 0, 1)[None], size=(rh, rw), mode="bilinear", align_corners=False)
    oy, ox = (rh - 224) // 2, (rw - 224) // 2
    x = x[:, :, oy:oy + 224, ox:ox + 224] / 255
    x = (x - torch.tensor([0.485, 0.456, 0.406]).view(1, 3, 1, 1)) / torch.tensor([0.229, 0.224, 0.225]).view(1, 3, 1, 1)
    with torch.no_grad():
        ref = build("alexnet", seed=2)(x)
    assert int(m.group(1)) == int(ref.argmax())


def _rows(text):
    return re.findall(r"\| (127\.0\.0\.1:\d+) ", text)


def test_sdfs_replication_and_membership(env, tmp_path):
    src = tmp_path / "data.txt"
    src.write_text("version one\n")
    cl = LocalCluster(5, 19100, str(tmp_path / "c"), env["labels"], n_leaders=2, executor="cpu")
    with cl:
        n = cl.nodes
        out = n[3].cmd(f"put {src} data.txt")
        assert out.startswith("Stored on:"), out
        assert len(_rows(out)) == 4  # replication factor 4
        holders = [nd for nd in n if "data.txt" in nd.cmd("store")]
        assert len(holders) == 4
        dest = tmp_path / "got.txt"
        assert "Retrieved version: 1" in n[4].cmd(f"get data.txt {dest}")
        assert dest.read_text() == "version one\n"
        assert "File not found!" in n[4].cmd("get nothere.txt x")
        # version 2 and the get-versions merge format
        src.write_text("version two\n")
        assert "Stored on:" in n[2].cmd(f"put {src} data.txt")
        merged = tmp_path / "merged.txt"
        assert "Retrieved versions: {1, 2}" in n[1].cmd(f"gv data.txt 2 {merged}")
        txt = merged.read_text()
        assert txt == ("============== Version 2 ===============\nversion two\n\n"
                       "============== Version 1 ===============\nversion one\n\n")
        ls = n[0].cmd("ls data.txt")
        assert len(_rows(ls)) == 4 and ls.count("| 2 ") == 4, ls
        # kill one replica holder (not a leader candidate): re-replication restores 4
        victim = next(nd for nd in n[2:] if nd in holders)
        victim.kill()
        survivors = [nd for nd in n if nd is not victim]
        cl.wait_members(4, 20, survivors)
        deadline = time.time() + 20
        while True:
            rows = _rows(n[0].cmd("ls data.txt"))
            if (len(rows) == 4 and victim.address not in rows) or time.time() > deadline:
                break
            time.sleep(0.5)
        assert len(rows) == 4 and victim.address not in rows, rows
        # the new replica holds the latest version's bytes
        newcomer = next(nd for nd in survivors if nd not in holders)
        assert "data.txt" in newcomer.cmd("store")
        # delete removes metadata and replica files
        assert "Deleted!" in n[0].cmd("delete data.txt")
        assert _rows(n[0].cmd("ls data.txt")) == []
        for nd in survivors:
            sd = os.path.join(cl.root, f"n{nd.port}", "storage")
            assert not any(f.endswith("data.txt") for f in os.listdir(sd))


def test_failure_detection_and_rejoin(env, tmp_path):
    cl = LocalCluster(4, 19300, str(tmp_path / "c"), env["labels"], n_leaders=1, executor="cpu")
    with cl:
        n = cl.nodes
        n[3].kill()
        n[0].expect(r"Detected failure of|Updating membership for 127\.0\.0\.1:19330: Active -> Failed", 15, 0)
        cl.wait_members(3, 20, n[:3])
        # voluntary leave is propagated (Leave message), faster than the timeout
        t0 = time.time()
        assert "Leaving group" in n[2].cmd("leave")
        cl.wait_members(2, 10, n[:2])
        assert time.time() - t0 < 10
        # rejoin with a new incarnation
        n[2].run(f"join {n[0].address}", r"Joined!")
        cl.wait_members(3, 20, n[:3])


def _job_counts(node):
    out = node.cmd("jobs")
    return [(int(a), int(b), int(c)) for a, b, c in
            re.findall(r"Accuracy: (\d+)/(\d+) = .*\n\tQueries: (\d+) total", out)]


def test_predict_jobs_assign_and_leader_failover(env, tmp_path):
    models = f"resnet18={env['models']['resnet18']},alexnet={env['models']['alexnet']}"
    cl = LocalCluster(4, 19500, str(tmp_path / "c"), env["labels"], n_leaders=2, executor="cpu",
                      dataset=env["dataset"], models=models,
                      extra=["--job-limit", "40", "--query-interval-ms", "100", "--quiet-predictions"])
    with cl:
        n = cl.nodes
        time.sleep(1.0)  # one assignment round
        out = n[3].cmd("assign")
        j1, j2 = out.split("Job 2:")
        assert len(_rows(j1)) == 2 and len(_rows(j2)) == 2, out  # fair 50/50 split
        n[3].cmd("predict")
        time.sleep(1.5)
        early = _job_counts(n[3])
        assert len(early) == 2 and all(c[1] > 0 for c in early), early
        # kill the leader mid-run; the standby takes over and resumes
        n[0].kill()
        deadline = time.time() + 60
        counts = []
        while time.time() < deadline:
            try:
                counts = _job_counts(n[3])
            except Exception:  # noqa: BLE001  (leader switch in progress)
                counts = []
            if len(counts) == 2 and all(c[1] >= 40 for c in counts):
                break
            time.sleep(1.0)
        assert len(counts) == 2 and all(c[1] >= 40 for c in counts), counts
        assert all(c[2] == c[1] for c in counts)
        rep = n[3].cmd("jobs")
        assert "Model: resnet18" in rep and "Model: alexnet" in rep and "ms p95" in rep


@pytest.mark.parametrize("victim", ["leader", "member"])
def test_hung_node_failover(env, tmp_path, victim):
    """A node that hangs (SIGSTOP: its sockets stay open, nothing answers, no
    FIN or RST) instead of crashing, with the reference's periods (1 s pings,
    3 s failure timeout, 3 s loops): a hung leader is found by the members'
    heartbeat (csrc/control/member.cpp leader_watch_loop) and the standby
    takes over and resumes the jobs; a hung member costs a query its adaptive
    deadline (csrc/serve/leader.cpp query_timeout), then the query goes to
    another member. Either way answers flow again within a few seconds and
    both jobs finish."""
    models = f"resnet18={env['models']['resnet18']},alexnet={env['models']['alexnet']}"
    base = 21000 if victim == "leader" else 21100  # (ports no other test uses: the suite runs in parallel)
    cl = LocalCluster(4, base, str(tmp_path / "c"), env["labels"], n_leaders=2, executor="cpu",
                      dataset=env["dataset"], models=models, fast=False,
                      extra=["--job-limit", "48", "--query-interval-ms", "250", "--quiet-predictions",
                             "--standby-copy-ms", "3000"])
    with cl:
        n = cl.nodes
        time.sleep(4.0)  # one assignment round at the reference's 3 s period
        n[3].cmd("predict")
        time.sleep(4.0)
        before = _job_counts(n[3])
        assert len(before) == 2 and all(c[1] > 0 for c in before), before
        hung = n[0] if victim == "leader" else n[2]
        t0 = time.time()
        hung.freeze()
        deadline = t0 + 90
        counts, resumed = [], None
        while time.time() < deadline:
            try:
                counts = _job_counts(n[3])
            except Exception:  # noqa: BLE001  (leader switch in progress, or the hung leader timed out)
                counts = []
            if resumed is None and len(counts) == 2 and sum(c[1] for c in counts) > sum(c[1] for c in before) + 4:
                resumed = time.time() - t0
            if len(counts) == 2 and all(c[1] >= 48 for c in counts):
                break
            time.sleep(0.5)
        assert len(counts) == 2 and all(c[1] >= 48 for c in counts), counts
        assert resumed is not None and resumed < 15, resumed
        hung.kill()


def test_adaptive_rate_jobs(env, tmp_path):
    """--adaptive-window: no tick, each job keeps a window of queries in flight
    per assigned member (least-outstanding routing), so with a 10 s tick set
    the jobs still finish at the members' own speed."""
    models = f"resnet18={env['models']['resnet18']},alexnet={env['models']['alexnet']}"
    cl = LocalCluster(4, 19600, str(tmp_path / "c"), env["labels"], n_leaders=1, executor="cpu",
                      dataset=env["dataset"], models=models,
                      extra=["--job-limit", "40", "--query-interval-ms", "10000", "--adaptive-window", "2",
                             "--quiet-predictions"])
    with cl:
        n = cl.nodes
        time.sleep(1.0)  # one assignment round
        n[0].cmd("predict")
        deadline = time.time() + 60
        counts = []
        while time.time() < deadline:
            counts = _job_counts(n[0])
            if len(counts) == 2 and all(c[1] >= 40 for c in counts):
                break
            time.sleep(0.5)
        # a fixed 10 s tick would have finished 6 queries per job by now
        assert len(counts) == 2 and all(c[1] == 40 and c[2] == 40 for c in counts), counts
        rep = n[0].cmd("jobs")
        rates = [float(x) for x in re.findall(r"Throughput: ([\d.]+) queries/s", rep)]
        assert len(rates) == 2 and all(r > 0.5 for r in rates), rep


def test_clock_skew_does_not_fail_live_node(env, tmp_path):
    """A node whose wall clock is 5 s behind (4x the 1.2 s failure timeout)
    stays Active: the detector ages entries by the local time since their
    heartbeat last advanced, not by comparing clocks.
    A killed node is still detected."""
    from dmlc.serve.cluster import NodeProcess
    cl = LocalCluster(2, 19700, str(tmp_path / "c"), env["labels"], n_leaders=1, executor="cpu")
    with cl:
        p = 19700 + 20
        skewed = NodeProcess(p, cl.leaders, str(tmp_path / "c" / f"n{p}"), env["labels"], executor="cpu",
                             extra=["--clock-skew-ms", "-5000"])
        cl.nodes.append(skewed)
        skewed.expect(r"Address is", 20)
        skewed.run(f"join {cl.nodes[0].address}", r"Joined!", 20)
        cl.wait_members(3, 20)
        time.sleep(4.0)
        for nd in cl.nodes:
            rows = re.findall(r"\| 127\.0\.0\.1:\d+ .*\| Active", nd.cmd("lm"))
            assert len(rows) == 3, nd.cmd("lm")
        flaps = [ln for nd in cl.nodes for ln in nd.lines if "Detected failure" in ln]
        assert not flaps, flaps
        cl.nodes[1].kill()
        cl.wait_members(2, 20, [cl.nodes[0], skewed])
