"""dmlc-node with the GPU executor (hand-written HIP engine) on a real GPU:
classification agrees with the CPU (libtorch) executor, and a two-node
cluster serves predict jobs from the GPU."""
import os
import re
import subprocess
import time

import pytest

from dmlc.serve.cluster import NODE_BIN, LocalCluster
from dmlc.utils.dataset import make_synthetic_dataset, synthetic_labels, write_labels
from dmlc.utils.ot import write_random_checkpoint

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def env(tmp_path_factory):
    root = tmp_path_factory.mktemp("gpunode")
    labels = synthetic_labels(1000)
    lab = write_labels(str(root / "synset_words.txt"), labels)
    ds = make_synthetic_dataset(str(root / "train"), labels[:16], size=(300, 400))
    ckpt = write_random_checkpoint("resnet18", str(root / "resnet18.ot"), seed=4)
    ckpt_a = write_random_checkpoint("alexnet", str(root / "alexnet.ot"), seed=5)
    ckpt_rb = write_random_checkpoint("resnet18", str(root / "resnet18_rb.ot"), seed=6, randomize_bn=True)
    return {"root": root, "labels": lab, "dataset": ds, "ckpt": ckpt, "ckpt_a": ckpt_a, "ckpt_rb": ckpt_rb,
            "entries": labels}


def _classify(env, executor, images):
    r = subprocess.run([NODE_BIN, "classify", "--model", "resnet18", "--weights", env["ckpt"], "--labels",
                        env["labels"], "--image", ",".join(images), "--executor", executor],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    return [int(x) for x in re.findall(r"class=(\d+)", r.stdout)], r.stdout


def test_gpu_executor_agrees_with_cpu(gpu, env):
    imgs = []
    for wnid, _ in env["entries"][:16]:
        d = os.path.join(env["dataset"], wnid)
        imgs.append(os.path.join(d, sorted(os.listdir(d))[0]))
    g, out = _classify(env, "gpu", imgs)
    c, _ = _classify(env, "cpu", imgs)
    assert "[gpu:0]" in out
    assert len(g) == len(c) == 16
    agree = sum(a == b for a, b in zip(g, c))
    assert agree >= 14, (g, c)  # bf16 vs fp32: only near-ties may flip


def test_gpu_executor_ragged_batch_agrees_with_cpu(gpu, env, tmp_path):
    """Mixed-size JPEGs in one query: the GPU executor resizes them into one
    u8 batch (resize.hip) and runs one forward; the CPU executor applies the
    same resize rule per image."""
    sizes = [(224, 224), (375, 500), (500, 333), (256, 300), (480, 640), (199, 211), (224, 300), (640, 427)]
    ds = make_synthetic_dataset(str(tmp_path / "ragged"), env["entries"][:16], size=sizes, seed=9)
    imgs = []
    for wnid, _ in env["entries"][:16]:
        d = os.path.join(ds, wnid)
        imgs.append(os.path.join(d, sorted(os.listdir(d))[0]))
    g, _ = _classify(env, "gpu", imgs)
    c, _ = _classify(env, "cpu", imgs)
    assert len(g) == len(c) == 16
    agree = sum(a == b for a, b in zip(g, c))
    assert agree >= 14, (g, c)


def test_gpu_cluster_predict(gpu, env, tmp_path):
    cl = LocalCluster(2, 19700, str(tmp_path / "c"), env["labels"], n_leaders=1, executor="gpu",
                      dataset=env["dataset"], models=f"resnet18={env['ckpt']}",
                      extra=["--jobs", "resnet18", "--job-limit", "16", "--query-interval-ms", "20",
                             "--query-batch", "4", "--quiet-predictions"])
    with cl:
        n = cl.nodes
        assert "executor gpu:0" in n[0].cmd("info")
        n[1].cmd("predict")
        deadline = time.time() + 60
        done = 0
        while time.time() < deadline:
            m = re.search(r"Accuracy: \d+/(\d+)", n[1].cmd("jobs"))
            done = int(m.group(1)) if m else 0
            if done >= 16:
                break
            time.sleep(0.5)
        assert done == 16


def test_gpu_hbm_image_cache(gpu, env, tmp_path):
    """--prefetch stages every class's query image into HBM on a side
    stream; the job's queries then hit the resident copies (no JPEG decode,
    no host->device copy on the query path)."""
    cl = LocalCluster(1, 19750, str(tmp_path / "c"), env["labels"], n_leaders=1, executor="gpu",
                      dataset=env["dataset"], models=f"resnet18={env['ckpt']}",
                      extra=["--jobs", "resnet18", "--job-limit", "16", "--query-interval-ms", "20",
                             "--query-batch", "4", "--quiet-predictions", "--prefetch"])
    with cl:
        n = cl.nodes[0]
        deadline = time.time() + 60
        while time.time() < deadline:
            m = re.search(r"prefetched (\d+)", n.cmd("info"))
            if m and int(m.group(1)) >= 16:
                break
            time.sleep(0.2)
        info = n.cmd("info")
        assert re.search(r"staged 16 ", info), info
        n.cmd("predict")
        deadline = time.time() + 60
        done = 0
        while time.time() < deadline:
            m = re.search(r"Accuracy: \d+/(\d+)", n.cmd("jobs"))
            done = int(m.group(1)) if m else 0
            if done >= 16:
                break
            time.sleep(0.5)
        assert done == 16
        m = re.search(r"cache hits (\d+) misses (\d+)", n.cmd("info"))
        assert m and int(m.group(1)) >= 16 and int(m.group(2)) == 0, n.cmd("info")


def test_gpu_shard_served_from_hbm_without_host_io(gpu, env, tmp_path):
    """A u8 shard put into the SDFS is staged into the member's HBM when the
    replica arrives; with the replica FILES deleted from every node's disk,
    predict-shard still classifies it (from HBM, through the executor's
    dp::Group) with the same answers as the in-process engine."""
    import glob
    import torch
    from dmlc.runtime import InferenceEngine
    from dmlc.utils.shards import read_shard, synthetic_shard
    shard = synthetic_shard(str(tmp_path / "s.u8s"), 40, 224, seed=8)
    cl = LocalCluster(2, 19800, str(tmp_path / "c"), env["labels"], n_leaders=1, executor="gpu",
                      dataset=env["dataset"], models=f"resnet18={env['ckpt']}", extra=["--max-batch", "64"])
    with cl:
        n = cl.nodes
        assert "Stored on:" in n[1].cmd(f"put {shard} s.u8s")
        deadline = time.time() + 60
        while time.time() < deadline and "s.u8s@v1" not in n[0].cmd("replicas"):
            time.sleep(0.2)
        assert re.search(r"s\.u8s@v1 in hbm:gpu0", n[0].cmd("replicas")), n[0].cmd("replicas")
        removed = [p for p in glob.glob(str(tmp_path / "c" / "*" / "storage" / "v1.s.u8s"))]
        assert removed
        for p in removed:
            os.remove(p)
        out = n[0].cmd("predict-shard s.u8s resnet18", 120)
    m = re.search(r"Classified 40 images of s.u8s v1 on (\S+) \[hbm:gpu0 -> gpu:0\]", out)
    assert m, out
    got = [int(x) for x in re.findall(r"(\d+):\d", out.split("first:")[1])]
    eng = InferenceEngine("resnet18", env["ckpt"], device=0, max_batch=64)
    idx, _ = eng.predict(torch.from_numpy(read_shard(shard).copy()).cuda())
    torch.cuda.synchronize()
    assert got == idx[:8].cpu().tolist()


def test_gpu_jobs_over_hbm_shard(gpu, env, tmp_path):
    """Both jobs over a labelled SDFS shard (`predict <shard>`): every query
    is a range of the shard classified in place from its HBM slice on the
    replica holder (no JPEG decode, no host I/O: the replica files are
    deleted first). The report's accuracy must equal the count of images the
    in-process engine puts in their label class, and every printed
    prediction must be the engine's."""
    import glob
    import torch
    from dmlc.runtime import InferenceEngine
    from dmlc.utils.shards import synthetic_shard, read_shard, write_shard
    label0, n = 0, 48
    imgs = read_shard(synthetic_shard(str(tmp_path / "raw.u8s"), n, 224, seed=21))
    shard = write_shard(str(tmp_path / "val.u8s"), imgs, label0=label0)
    cl = LocalCluster(1, 19850, str(tmp_path / "c"), env["labels"], n_leaders=1, executor="gpu",
                      dataset=env["dataset"], models=f"resnet18={env['ckpt_rb']},alexnet={env['ckpt_a']}",
                      extra=["--max-batch", "16", "--query-batch", "8", "--adaptive-window", "2"])
    with cl:
        nd = cl.nodes[0]
        assert re.search(r"placement alexnet=gpu0 resnet18=gpu0", nd.cmd("info")), nd.cmd("info")
        assert "Stored on:" in nd.cmd(f"put {shard} val.u8s")
        deadline = time.time() + 60
        while time.time() < deadline and "val.u8s@v1" not in nd.cmd("replicas"):
            time.sleep(0.2)
        for p in glob.glob(str(tmp_path / "c" / "*" / "storage" / "v1.val.u8s")):
            os.remove(p)
        mark = nd.mark()
        nd.cmd("predict val.u8s")
        deadline = time.time() + 120
        out = ""
        while time.time() < deadline:
            out = nd.cmd("jobs")
            if len(re.findall(rf"Accuracy: \d+/{n} ", out)) == 2:
                break
            time.sleep(0.5)
        text = nd.output(mark)
    # the oracle at the queries' batch size (8): the same kernel paths
    eng = InferenceEngine("resnet18", env["ckpt_rb"], device=0, max_batch=8)
    x = torch.from_numpy(imgs.copy()).cuda()
    idx = []
    for s in range(0, n, 8):
        i, _ = eng.predict(x[s:s + 8].contiguous())
        idx += i.cpu().tolist()
    correct = sum(int(c == label0 + i) for i, c in enumerate(idx))
    m = re.search(rf"Model: resnet18\n\tAccuracy: (\d+)/{n} ", out)
    assert m and int(m.group(1)) == correct, out
    assert re.search(r"Data: SDFS shards val\.u8s", out)
    got = dict(re.findall(r"^resnet18 - (n\d+): (.*?) \(\d", text, re.M))
    wnids = [w for w, _ in env["entries"]]
    texts = dict(env["entries"])
    for i in range(n):
        assert got[wnids[label0 + i]] == texts[wnids[idx[i]]], i
