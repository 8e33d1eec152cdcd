"""`train` and SDFS-staged shards through the whole control plane (CPU
executor, so it runs here):

* `put new.ot` + `train new.ot resnet18` distributes the checkpoint to every
  member, which hot-swaps it (M_LOAD_MODEL); the job starts over and the next
  `predict` answers with the NEW weights — the reference copied the file and
  never loaded it (src/services.rs:139-144 vs :513-524).
* a u8 image shard `put` into the SDFS is staged by every replica holder
  into its executor's blob store (HBM on GPU members; host memory here) and
  `predict-shard` classifies it where it lives (BASELINE config 3's
  "SDFS-staged imagenet_1k shards"); answers match torch.nn on the same
  pixels.
"""
import os
import re
import subprocess
import time

import numpy as np
import pytest
import torch

from dmlc.models import build
from dmlc.serve.cluster import NODE_BIN, LocalCluster
from dmlc.utils.dataset import make_synthetic_dataset, synthetic_labels, write_labels
from dmlc.utils.ot import write_random_checkpoint
from dmlc.utils.shards import read_shard, synthetic_shard

pytestmark = pytest.mark.slow

PRED = re.compile(r"^resnet18 - (n\d+): (.*?) \((\d+\.\d+)%\)", re.M)
MEAN = torch.tensor([0.485, 0.456, 0.406]).view(1, 3, 1, 1)
STD = torch.tensor([0.229, 0.224, 0.225]).view(1, 3, 1, 1)


@pytest.fixture(scope="module")
def env(tmp_path_factory):
    root = tmp_path_factory.mktemp("train")
    labels = synthetic_labels(1000)
    lab = write_labels(str(root / "synset_words.txt"), labels)
    ds = make_synthetic_dataset(str(root / "train"), labels[:4], size=(96, 128), seed=3)
    return {"root": root, "labels": lab, "dataset": ds, "entries": labels,
            "a": write_random_checkpoint("resnet18", str(root / "a.ot"), seed=11),
            "b": write_random_checkpoint("resnet18", str(root / "b.ot"), seed=12)}


def _predict(node, n=4, timeout=120):
    mark = node.mark()
    node.cmd("predict")
    deadline = time.time() + timeout
    while time.time() < deadline:
        m = re.search(r"Accuracy: \d+/(\d+)", node.cmd("jobs"))
        if m and int(m.group(1)) >= n:
            break
        time.sleep(0.3)
    time.sleep(0.3)
    got = {w: lbl for w, lbl, _ in PRED.findall(node.output(mark))}
    assert len(got) == n, node.output(mark)[-3000:]
    return got


def _classify(env, ckpt, wnid):
    d = os.path.join(env["dataset"], wnid)
    img = os.path.join(d, sorted(os.listdir(d))[0])
    r = subprocess.run([NODE_BIN, "classify", "--model", "resnet18", "--weights", ckpt, "--labels", env["labels"],
                        "--image", img, "--executor", "cpu"], capture_output=True, text=True, timeout=120,
                       env={**os.environ, "OMP_NUM_THREADS": "4"})
    assert r.returncode == 0, r.stderr
    return re.search(r"\] (.*?) \(\d", r.stdout).group(1)


def test_train_hot_swaps_and_predict_uses_new_weights(env, tmp_path):
    cl = LocalCluster(2, 20600, str(tmp_path / "c"), env["labels"], n_leaders=1, executor="cpu",
                      dataset=env["dataset"], models=f"resnet18={env['a']}",
                      extra=["--jobs", "resnet18", "--job-limit", "4", "--query-interval-ms", "20"])
    with cl:
        n = cl.nodes
        time.sleep(1.0)
        before = _predict(n[0])
        assert "Stored on:" in n[1].cmd(f"put {env['b']} new.ot")
        out = n[1].cmd("train new.ot resnet18", 180)
        assert "Training complete!" in out, out
        after = _predict(n[0])
    wnids = [w for w, _ in env["entries"][:4]]
    assert before == {w: _classify(env, env["a"], w) for w in wnids}
    assert after == {w: _classify(env, env["b"], w) for w in wnids}
    assert before != after


def test_shard_staged_and_classified_where_it_lives(env, tmp_path):
    shard = synthetic_shard(str(tmp_path / "imgs.u8s"), 6, 224, seed=5)
    cl = LocalCluster(2, 20650, str(tmp_path / "c"), env["labels"], n_leaders=1, executor="cpu",
                      dataset=env["dataset"], models=f"resnet18={env['a']}")
    with cl:
        n = cl.nodes
        assert "Stored on:" in n[1].cmd(f"put {shard} imgs.u8s")
        deadline = time.time() + 30
        while time.time() < deadline and "imgs.u8s@v1" not in n[0].cmd("replicas"):
            time.sleep(0.2)
        assert "imgs.u8s@v1" in n[0].cmd("replicas")
        out = n[0].cmd("predict-shard imgs.u8s resnet18", 180)
    m = re.search(r"Classified 6 images of imgs.u8s v1 on (\S+) \[(.*?)\]", out)
    assert m, out
    got = [int(x) for x in re.findall(r"(\d+):\d", out.split("first:")[1])]
    x = torch.from_numpy(read_shard(shard).copy()).permute(0, 3, 1, 2).float() / 255
    with torch.no_grad():
        ref = build("resnet18", seed=11)((x - MEAN) / STD).argmax(-1).tolist()
    assert got == ref, (got, ref)
