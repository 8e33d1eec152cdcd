"""Untrusted-input hardening of the native control plane, under
AddressSanitizer + UndefinedBehaviorSanitizer builds (tools/build.py:
build/bin/dmlc-fuzz-asan, build/bin/dmlc-node-asan):

* mutation fuzzing of the JPEG decoder, the membership datagram codec and
  the leader's job/directory payload readers (csrc/cli/fuzz.cpp);
* hostile peers: random and malformed RPC frames against a live node's
  member and leader ports; the node must keep serving, with no sanitizer
  report;
* peers may only read/write `storage:`/`models:` files and the paths this
  node's own put/get commands grant (M_READ_CHUNK of /etc/passwd used to be
  served to anyone).

The reference (Rust) got memory safety from the language; the C++ rebuild
checks it with sanitizers instead (SURVEY.md §5 "Race detection /
sanitizers")."""
import os
import random
import struct
import subprocess
import time

import pytest

from dmlc import REPO_ROOT
from dmlc.serve import rpc
from dmlc.serve.cluster import LocalCluster
from dmlc.utils.dataset import make_synthetic_dataset, synthetic_labels, write_labels

pytestmark = pytest.mark.slow

FUZZ_BIN = os.path.join(REPO_ROOT, "build", "bin", "dmlc-fuzz-asan")
ASAN_BIN = os.path.join(REPO_ROOT, "build", "bin", "dmlc-node-asan")
ASAN_ENV = {"ASAN_OPTIONS": "detect_leaks=0:abort_on_error=0", "UBSAN_OPTIONS": "print_stacktrace=1"}


def _seed_jpegs(root):
    from PIL import Image
    import numpy as np
    rng = np.random.default_rng(0)
    out = []
    specs = [((48, 64), 0, None), ((40, 56), 2, None), ((33, 17), 1, None), ((64, 48), 0, "L"),
             ((56, 40), 2, "restart")]
    for i, ((h, w), sub, mode) in enumerate(specs):
        base = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
        img = Image.fromarray(base)
        p = os.path.join(root, f"seed{i}.jpg")
        kw = {"quality": 85, "subsampling": sub}
        if mode == "L":
            img = img.convert("L")
            kw.pop("subsampling")
        if mode == "restart":
            kw["restart_marker_blocks"] = 2
        try:
            img.save(p, **kw)
        except TypeError:  # older PIL: no restart markers
            kw.pop("restart_marker_blocks", None)
            img.save(p, **kw)
        out.append(p)
    return out


@pytest.mark.parametrize("seed", [1, 2])
def test_fuzz_parsers_asan(tmp_path, seed):
    assert os.path.exists(FUZZ_BIN), "python tools/build.py"
    seeds = _seed_jpegs(str(tmp_path))
    r = subprocess.run([FUZZ_BIN, "--iters", "15000", "--seed", str(seed), *seeds], capture_output=True, text=True,
                       timeout=600, env={**os.environ, **ASAN_ENV})
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-6000:]
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-6000:]
    assert "fuzz: 15000 iterations" in r.stdout


def _sanitizer_clean(nodes):
    bad = [(nd.address, nd.output()) for nd in nodes
           if "AddressSanitizer" in nd.output() or "runtime error" in nd.output()]
    assert not bad, "\n\n".join(f"== {a}\n{o[-6000:]}" for a, o in bad)


@pytest.fixture()
def asan_cluster(tmp_path):
    assert os.path.exists(ASAN_BIN), "python tools/build.py"
    labels = synthetic_labels(1000)
    lab = write_labels(str(tmp_path / "synset_words.txt"), labels)
    ds = make_synthetic_dataset(str(tmp_path / "train"), labels[:24], size=(48, 64))
    cl = LocalCluster(3, 20400, str(tmp_path / "c"), lab, n_leaders=1, executor="digest", dataset=ds,
                      models="resnet18=-,alexnet=-", binary=ASAN_BIN, env=ASAN_ENV,
                      extra=["--job-limit", "24", "--query-interval-ms", "20", "--quiet-predictions"])
    with cl:
        yield cl, tmp_path


def test_hostile_rpc_frames(asan_cluster):
    cl, tmp = asan_cluster
    n = cl.nodes
    src = tmp / "f.txt"
    src.write_text("hello\n" * 100)
    assert "Stored on:" in n[1].cmd(f"put {src} f.txt")
    rng = random.Random(5)
    methods = list(range(1, 11)) + list(range(20, 28)) + [0, 99, 65535]
    for port in (20400 + 1, 20400 + 2, 20410 + 2):  # leader of n0, members of n0 and n1
        for _ in range(120):
            m = rng.choice(methods)
            kind = rng.random()
            if kind < 0.4:  # random payload in a well-formed frame
                payload = bytes(rng.getrandbits(8) for _ in range(rng.randint(0, 64)))
                body = struct.pack("<H", m) + payload
                frame = struct.pack("<I", len(body)) + body
            elif kind < 0.7:  # huge counts / lengths
                payload = struct.pack("<I", rng.choice([0xFFFFFFFF, 0x7FFFFFFF, 1 << 28])) * rng.randint(1, 4)
                body = struct.pack("<H", m) + payload
                frame = struct.pack("<I", len(body)) + body
            elif kind < 0.85:  # frame length lies
                frame = struct.pack("<I", rng.choice([0, 1, 3, 1 << 29, 0xFFFFFFFF])) + struct.pack("<H", m)
            else:  # garbage
                frame = bytes(rng.getrandbits(8) for _ in range(rng.randint(1, 40)))
            rpc.send_raw("127.0.0.1", port, frame, timeout=1.0)
    # still alive and correct
    assert "Retrieved version: 1" in n[2].cmd(f"get f.txt {tmp / 'back.txt'}")
    assert (tmp / "back.txt").read_text() == src.read_text()
    st, body = rpc.call("127.0.0.1", 20400 + 1, rpc.L_ALIVE)
    assert st == 0
    _sanitizer_clean(n)


def test_peers_cannot_touch_arbitrary_files(asan_cluster):
    cl, tmp = asan_cluster
    secret = tmp / "secret.txt"
    secret.write_text("do not serve me\n")
    member = 20400 + 2
    # read an arbitrary absolute path: refused
    st, body = rpc.call("127.0.0.1", member, rpc.M_READ_CHUNK,
                        rpc.s(str(secret)) + struct.pack("<QI", 0, 1 << 20))
    assert st == 1 and b"refused" in body, (st, body)
    st, body = rpc.call("127.0.0.1", member, rpc.M_READ_CHUNK,
                        rpc.s("../secret.txt") + struct.pack("<QI", 0, 1 << 20))
    assert st == 1 and b"refused" in body
    # make the member write an arbitrary absolute path: refused
    target = tmp / "planted.txt"
    st, body = rpc.call("127.0.0.1", member, rpc.M_FETCH,
                        rpc.s("127.0.0.1") + struct.pack("<i", 20412) + rpc.s("storage:v1.f.txt") + rpc.s(str(target)))
    assert st == 0 and body[:1] == b"\x00" and not target.exists()
    # load a "model" from an arbitrary path: refused
    st, body = rpc.call("127.0.0.1", member, rpc.M_LOAD_MODEL, rpc.s("resnet18") + rpc.s(str(secret)))
    assert st == 0 and body[:1] == b"\x00" and b"refused" in body
    # the legitimate flows still work: put (source granted while it runs), get
    src = tmp / "ok.txt"
    src.write_text("fine\n")
    assert "Stored on:" in cl.nodes[1].cmd(f"put {src} ok.txt")
    assert "Retrieved version: 1" in cl.nodes[2].cmd(f"get ok.txt {tmp / 'ok_back.txt'}")
    assert (tmp / "ok_back.txt").read_text() == "fine\n"
    _sanitizer_clean(cl.nodes)


def test_jobs_complete_with_a_member_missing_the_model(tmp_path):
    """ADVICE r1 (leader.cpp adaptive routing): a member that answers
    ok=false (no such model) must not swallow queries. It is benched and its
    queries move to other members; every query of both jobs completes."""
    from dmlc.serve.cluster import NodeProcess
    labels = synthetic_labels(1000)
    lab = write_labels(str(tmp_path / "synset_words.txt"), labels)
    ds = make_synthetic_dataset(str(tmp_path / "train"), labels[:40], size=(48, 64))
    extra = ["--job-limit", "40", "--adaptive-window", "2", "--quiet-predictions"]
    cl = LocalCluster(3, 20500, str(tmp_path / "c"), lab, n_leaders=1, executor="digest", dataset=ds,
                      models="resnet18=-,alexnet=-", binary=ASAN_BIN, env=ASAN_ENV, extra=extra)
    with cl:
        # a 4th node with NO models joins
        bad = NodeProcess(20530, cl.leaders, str(tmp_path / "c" / "bad"), lab, dataset=ds, models="",
                          executor="digest", binary=ASAN_BIN, env=ASAN_ENV, extra=extra)
        cl.nodes.append(bad)
        bad.expect(r"Address is", 20)
        bad.run(f"join {cl.nodes[0].address}", r"Joined!", 20)
        cl.wait_members(4, 30)
        time.sleep(1.5)  # the fair-share loop gives the model-less node to a job
        cl.nodes[0].cmd("predict")
        deadline = time.time() + 60
        out = ""
        while time.time() < deadline:
            out = cl.nodes[0].cmd("jobs")
            tot = [int(q) for q in __import__("re").findall(r"Accuracy: \d+/(\d+)", out)]
            if len(tot) == 2 and all(q >= 40 for q in tot):
                break
            time.sleep(0.3)
        assert tot == [40, 40], out
        _sanitizer_clean(cl.nodes)
