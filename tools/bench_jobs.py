#!/usr/bin/env python3
"""Serving benchmark through the whole control plane (BASELINE config:
"AlexNet + ResNet18 two concurrent predict jobs (fair-share coordinator, jobs
percentile reporting)").

Starts N `dmlc-node` processes (one per GPU when there are several; all on
GPU 0 on a one-GPU box), runs the reference's `predict` (both jobs over the
imagenet_1k-shaped dataset: one JPEG per class, decoded on the member, then
preprocess/forward/top-1 on the GPU), and reports from the leader's job
state the quantities the reference publishes (CS425MP4Report.pdf pp.2-3):
  * per-query latency mean/std (+ p50/p95/p99) per job (ref: ResNet18
    158.94 ms / AlexNet 149.52 ms mean),
  * time for the 2nd job to start executing queries (ref: 138.33 ms),
  * optionally the time to resume normal operation after killing a
    non-coordinator member (ref: 1.262 s) or the coordinator (ref: 3.593 s).

With --shards DIR (labelled u8 shards, tools/make_shards.py) the jobs run
over SDFS-staged shards instead (BASELINE config 3): the shards are `put`
into the SDFS, every replica holder stages its copy into HBM (one slice per
GPU), and `predict <shard>...` sends each query (a range of one shard) to a
replica holder, which classifies it in place: no JPEG decode, no host I/O.

usage: python tools/bench_jobs.py [--nodes 4] [--executor gpu] [--images 1000]
         [--interval-ms 50] [--batch 1] [--kill member|leader] [--fast-periods]
         [--shards data/shards]
"""
import argparse
import json
import os
import statistics
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dmlc.serve.cluster import LocalCluster  # noqa: E402
from dmlc.utils.dataset import make_synthetic_dataset, synthetic_labels, write_labels  # noqa: E402
from dmlc.utils.ot import write_random_checkpoint  # noqa: E402

REF = {"resnet18_mean_ms": 158.94, "alexnet_mean_ms": 149.52, "second_job_start_ms": 138.33,
       "member_failure_recovery_s": 1.262, "leader_failure_recovery_s": 3.593}


def pct(xs, q):
    xs = sorted(xs)
    if not xs:
        return None
    k = (len(xs) - 1) * q / 100
    lo, hi = int(k), min(int(k) + 1, len(xs) - 1)
    return xs[lo] + (xs[hi] - xs[lo]) * (k - lo)


def recovery_s(jobs, t_fail_us):
    """Longest gap between consecutive query completions (any job) after the
    failure, minus the median gap before it: how long the cluster stopped
    producing answers."""
    done = sorted(d for j in jobs for d in j["done_us"] if d > 0)
    before = [b - a for a, b in zip(done, done[1:]) if b < t_fail_us]
    after = [b - a for a, b in zip(done, done[1:]) if a >= t_fail_us - 5e6 and b > t_fail_us]
    if not after:
        return None
    base = statistics.median(before) if before else 0
    return max(0.0, (max(after) - base) / 1e6)


def resume_s(jobs, t_fail_us, window_s=3.0, frac=0.75):
    """Time from the failure to the first completion from which answers flow
    at the normal rate again: at least `frac` of the pre-failure completion
    rate over the following window_s (the report's "time to resume normal
    operation", measured from the failure instant)."""
    done = sorted(d for j in jobs for d in j["done_us"] if d > 0)
    pre = [d for d in done if t_fail_us - 10e6 <= d < t_fail_us]
    if len(pre) < 2 or pre[-1] <= pre[0]:
        return None
    rate = (len(pre) - 1) / ((pre[-1] - pre[0]) / 1e6)  # completions per second before the failure
    after = [d for d in done if d > t_fail_us]
    for i, t in enumerate(after):
        if t + window_s * 1e6 > done[-1]:
            break  # too close to the end of the jobs to judge
        n = sum(1 for x in after[i:] if x < t + window_s * 1e6)
        if n >= frac * rate * window_s:
            return (t - t_fail_us) / 1e6
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=4)
    ap.add_argument("--executor", default="gpu")
    ap.add_argument("--gpus", type=int, default=0, help="devices to spread nodes over (0 = all visible)")
    ap.add_argument("--images", type=int, default=1000)
    ap.add_argument("--interval-ms", type=int, default=50)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--adaptive-window", type=int, default=0,
                    help="closed-loop rate: queries in flight per member (0 = fixed --interval-ms tick)")
    ap.add_argument("--kill", choices=["none", "member", "leader"], default="none")
    ap.add_argument("--fail-mode", choices=["kill", "stop"], default="kill",
                    help="kill: SIGKILL the victim's process (the kernel closes its sockets: peers see a FIN); "
                         "stop: SIGSTOP it (a hung node: sockets stay open, nothing answers, no FIN or RST)")
    ap.add_argument("--keep-logs", action="store_true", help="write every node's console to <tmp root>/node<port>.log")
    ap.add_argument("--standby-copy-ms", type=int, default=250,
                    help="dmlc-node --standby-copy-ms (the reference copies job state at its 3 s loop period)")
    ap.add_argument("--fast-periods", action="store_true", help="200 ms pings, 1.2 s failure timeout, 500 ms loops")
    ap.add_argument("--port", type=int, default=21000)
    ap.add_argument("--out", default="")
    ap.add_argument("--dataset", default="", help="imagenet_1k layout dir (default: synthetic 500x375 JPEGs)")
    ap.add_argument("--labels", default="", help="synset_words.txt matching --dataset")
    ap.add_argument("--prefetch", action="store_true", help="stage every query image into HBM before predict")
    ap.add_argument("--node-gpus", type=int, default=1, help="GPUs per node (RCCL scatter inside a node)")
    ap.add_argument("--shards", default="", help="dir of labelled u8 shards: the jobs run over them from the SDFS")
    ap.add_argument("--job-limit", type=int, default=0,
                    help="images per job (shard jobs loop over their shards to reach it; default: one pass)")
    ap.add_argument("--max-batch", type=int, default=256, help="dmlc-node --max-batch (coalesced forward size)")
    ap.add_argument("--warm-frac", type=float, default=0.1,
                    help="steady state: the first this fraction of each job's queries is excluded")
    a = ap.parse_args()
    shards = sorted(f for f in os.listdir(a.shards) if f.endswith(".u8s")) if a.shards else []
    if shards:
        from dmlc.utils.shards import shard_info
        a.images = sum(shard_info(os.path.join(a.shards, f))["n"] for f in shards)
        if a.job_limit > 0:
            a.images = a.job_limit

    ngpu = a.gpus
    if a.executor == "gpu" and ngpu == 0:
        import torch
        ngpu = torch.cuda.device_count()
    root = tempfile.mkdtemp(prefix="dmlc_jobs_")
    if shards:  # the jobs read the shards; the members need no JPEG dataset
        ds = os.path.join(root, "empty")
        os.makedirs(ds)
        if a.labels:
            lab = os.path.abspath(a.labels)
        else:
            lab = write_labels(os.path.join(root, "synset_words.txt"), synthetic_labels(1000))
        data_desc = "shards"
    elif a.dataset:
        ds, lab = os.path.abspath(a.dataset), os.path.abspath(a.labels)
        n_avail = len(os.listdir(ds))
        if a.images > n_avail:
            a.images = n_avail
        data_desc = f"real imagenet_1k JPEGs from the reference ({a.images} classes, {ds}), random-init weights"
    else:
        labels = synthetic_labels(1000)
        lab = write_labels(os.path.join(root, "synset_words.txt"), labels)
        t = time.time()
        ds = make_synthetic_dataset(os.path.join(root, "train"), labels[:a.images], size=(375, 500))
        print(f"# dataset: {a.images} JPEGs 500x375 in {time.time() - t:.1f}s", file=sys.stderr)
        data_desc = "synthetic 500x375 JPEGs (imagenet_1k layout), random-init weights"
    ck = {m: write_random_checkpoint(m, os.path.join(root, f"{m}.ot"), seed=i) for i, m in
          enumerate(["resnet18", "alexnet"])}
    models = ",".join(f"{m}={p}" for m, p in ck.items())
    extra = ["--job-limit", str(a.images), "--query-interval-ms", str(a.interval_ms), "--query-batch",
             str(a.batch), "--quiet-predictions", "--max-batch", str(max(a.max_batch, a.batch)),
             "--adaptive-window", str(a.adaptive_window), "--standby-copy-ms", str(a.standby_copy_ms)] + \
        (["--prefetch"] if a.prefetch else [])
    cl = LocalCluster(a.nodes, a.port, os.path.join(root, "c"), lab, n_leaders=2, executor=a.executor,
                      dataset=ds, models=models, fast=a.fast_periods, extra=extra)
    if a.kill == "member" and a.nodes < 3:
        raise SystemExit("--kill member needs >= 3 nodes (2 leader candidates + a member)")
    nodes = []
    try:
        from dmlc.serve.cluster import NodeProcess
        for i, p in enumerate(cl.ports):
            ex = list(extra) + (["--device", str((i * a.node_gpus) % ngpu)] if ngpu else [])
            if a.node_gpus > 1:
                ex += ["--gpus", str(a.node_gpus)]
            nodes.append(NodeProcess(p, cl.leaders, os.path.join(cl.root, f"n{p}"), lab, dataset=ds,
                                     models=models, executor=a.executor, fast=a.fast_periods, extra=ex))
        cl.nodes = nodes
        for nd in nodes:
            nd.expect(r"Address is", 60)
        for nd in nodes:
            nd.run(f"join {nodes[0].address}", r"Joined!", 30)
        cl.wait_members(len(nodes), 60)
        time.sleep(4 if not a.fast_periods else 1.5)  # one assignment round
        client = nodes[min(1, len(nodes) - 1)]  # standby leader candidate: survives both kill experiments
        if shards:
            t = time.time()
            for f in shards:
                out = client.cmd(f"put {os.path.abspath(os.path.join(a.shards, f))} {f}", 600)
                assert "Stored on:" in out, out
            want = min(len(nodes), 4)  # replication factor 4
            deadline = time.time() + 600
            while time.time() < deadline:
                staged = sum(all(f"{f}@v1" in nd.cmd("replicas", 30) for f in shards) for nd in nodes)
                if staged >= want:
                    break
                time.sleep(1.0)
            print(f"# {len(shards)} shards put and staged in HBM in {time.time() - t:.1f}s", file=sys.stderr)
            data_desc = (f"SDFS-staged labelled u8 shards ({a.images} images in {len(shards)} shards from "
                         f"{os.path.abspath(a.shards)}), random-init weights")
        t_predict = time.time()
        client.cmd("predict " + " ".join(shards) if shards else "predict")
        t_fail = None
        deadline = time.time() + max(300, a.images * a.interval_ms / 1000 * 4)
        while time.time() < deadline:
            time.sleep(1.0)
            try:
                out = client.cmd("jobs", 30)
            except Exception as e:  # noqa: BLE001  (leader switch)
                print(f"# {time.time() - t_predict:.0f}s: jobs command failed: {str(e)[-3000:]}", file=sys.stderr,
                      flush=True)
                continue
            import re
            counts = [int(x) for x in re.findall(r"Accuracy: \d+/(\d+)", out)]
            if a.kill != "none" and t_fail is None and counts and min(counts) >= a.images * 0.3:
                victim = nodes[0] if a.kill == "leader" else nodes[-1]
                t_fail = time.time()
                if a.fail_mode == "stop":
                    victim.freeze()
                else:
                    victim.kill()
                print(f"# {a.fail_mode} {a.kill} {victim.address} at {t_fail - t_predict:.2f}s", file=sys.stderr)
            if len(counts) == 2 and min(counts) >= a.images:
                break
            if int(time.time() - t_predict) % 10 == 0:  # progress (a silent run looks hung)
                print(f"# {time.time() - t_predict:.0f}s: answered {counts}", file=sys.stderr, flush=True)
        dump = os.path.join(root, "jobs.json")
        client.cmd(f"jobs-dump {dump}")
        jobs = json.load(open(dump))
    finally:
        for nd in nodes:
            nd.stop()
        for nd in nodes:
            nd.kill()
        if a.keep_logs:  # every node's console output, for failure timelines
            for nd in nodes:
                with open(os.path.join(root, f"node{nd.port}.log"), "w") as f:
                    f.write(nd.output())
            print(f"# node logs in {root}", file=sys.stderr)
    res = {"bench": "two concurrent predict jobs through the control plane", "nodes": a.nodes,
           "executor": a.executor, "gpus": ngpu, "images_per_job": a.images, "query_interval_ms": a.interval_ms,
           "adaptive_window": a.adaptive_window,
           "query_batch": a.batch, "data": data_desc, "prefetch": a.prefetch, "node_gpus": a.node_gpus,
           "source": "shards" if shards else "jpeg",
           "fast_periods": a.fast_periods,
           # the node's failure-detection and background-loop periods this run used
           # (dmlc-node flags; the reference's are 1 s pings / 1 s detector, a 3 s
           # failure timeout and 3 s loops: src/membership.rs:230,273,289;
           # src/services.rs:188,201,213,529)
           # (standby_copy: the standby leader's job-state copy, --standby-copy-ms;
           # the reference copies at its 3 s loop period)
           "periods_ms": ({"ping": 200, "detect": 200, "fail": 1200, "bg": 500, "standby_copy": 250}
                          if a.fast_periods else
                          {"ping": 1000, "detect": 1000, "fail": 3000, "bg": 3000,
                           "standby_copy": a.standby_copy_ms}),
           "fail_mode": a.fail_mode,
           "kill": a.kill,
           "reference": REF, "jobs": []}
    for j in jobs:
        d = [x / 1000 for x in j["durations_us"]]
        span = (max(j["done_us"]) - j["started_us"]) / 1e6 if j["done_us"] else None
        # steady state: queries (equal-sized: --batch images, but a shard query
        # never spans two shards) completed after the first warm_frac of them
        done = sorted(x for x in j["done_us"] if x > 0)
        k0 = int(len(done) * a.warm_frac)
        steady = None
        if len(done) - k0 >= 2 and done[-1] > done[k0]:
            steady = round(j["finished"] * (len(done) - 1 - k0) / len(done) / ((done[-1] - done[k0]) / 1e6), 1)
        ds = d[int(len(d) * a.warm_frac):]
        res["jobs"].append({"model": j["model"], "finished": j["finished"], "correct": j["correct"],
                            "images_per_s": round(j["finished"] / span, 1) if span else None,
                            "steady_images_per_s": steady,
                            "steady_p50_ms": round(pct(ds, 50), 3) if ds else None,
                            "steady_p95_ms": round(pct(ds, 95), 3) if ds else None,
                            "mean_ms": round(statistics.mean(d), 3), "std_ms": round(statistics.pstdev(d), 3),
                            "p50_ms": round(pct(d, 50), 3), "p95_ms": round(pct(d, 95), 3),
                            "p99_ms": round(pct(d, 99), 3),
                            "queries_per_s": round(j["finished"] / span, 2) if span else None})
    fd = sorted(j["first_done_us"] for j in jobs)
    st = sorted(j["started_us"] for j in jobs)
    res["second_job_start_ms"] = round((st[-1] - st[0]) / 1000, 3)
    res["second_job_first_result_ms"] = round((fd[-1] - fd[0]) / 1000, 3)
    if t_fail is not None:
        res["t_fail_unix_s"] = round(t_fail, 3)
        res[f"{a.kill}_failure_recovery_s"] = round(recovery_s(jobs, t_fail * 1e6), 3)
        rs = resume_s(jobs, t_fail * 1e6)
        res[f"{a.kill}_failure_resume_s"] = round(rs, 3) if rs is not None else None
    line = json.dumps(res)
    print(line)
    if a.out:
        with open(a.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
