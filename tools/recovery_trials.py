#!/usr/bin/env python3
"""Failure-recovery trials with the reference's periods.

Runs tools/bench_jobs.py --kill member|leader TRIALS times each with the
dmlc-node defaults, which are the reference's periods: 1 s pings and detector
rounds, a 3 s failure timeout, 3 s re-replication / assignment / succession /
leader-check loops (src/membership.rs:230,273,289; src/services.rs:188,201,
213,529), and the reference's query rate (one query per job every 0.5 s,
src/services.rs:408). Writes one JSON per kind with every trial, the mean and
the std, next to the report's 1.262 s / 3.593 s (CS425MP4Report.pdf p.3).

usage: python tools/recovery_trials.py [--trials 3] [--nodes 6] [--executor cpu] [--out-dir profiles]
"""
import argparse
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = {"member": (1.262, 0.253, [1.21, 0.91, 1.41, 1.35, 1.62, 1.07]),
       "leader": (3.593, 0.554, [3.42, 2.67, 3.85, 4.22, 3.41, 3.99])}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=3)
    ap.add_argument("--nodes", type=int, default=6)
    ap.add_argument("--executor", default="cpu")
    ap.add_argument("--images", type=int, default=80)
    ap.add_argument("--interval-ms", type=int, default=500)
    ap.add_argument("--kinds", default="member,leader")
    ap.add_argument("--out-dir", default=os.path.join(ROOT, "profiles"))
    ap.add_argument("--tag", default="r5_recovery_refperiods")
    ap.add_argument("--fail-mode", choices=["kill", "stop"], default="kill",
                    help="kill: SIGKILL (peers see the sockets close); stop: SIGSTOP (a hung node, no FIN)")
    ap.add_argument("--standby-copy-ms", type=int, default=250)
    a = ap.parse_args()
    for kind in a.kinds.split(","):
        runs = []
        for t in range(a.trials):
            cmd = [sys.executable, os.path.join(ROOT, "tools", "bench_jobs.py"), "--nodes", str(a.nodes),
                   "--executor", a.executor, "--images", str(a.images), "--interval-ms", str(a.interval_ms),
                   "--kill", kind, "--port", str(23000 + 100 * t + (0 if kind == "member" else 50)),
                   "--fail-mode", a.fail_mode, "--standby-copy-ms", str(a.standby_copy_ms)]
            print("#", " ".join(cmd), file=sys.stderr, flush=True)
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=900)
            if r.returncode != 0:
                print(r.stderr[-3000:], file=sys.stderr)
                raise SystemExit(f"trial {t} of {kind} failed")
            res = json.loads(r.stdout.strip().splitlines()[-1])
            rec = res.get(f"{kind}_failure_recovery_s")
            resume = res.get(f"{kind}_failure_resume_s")
            print(f"# {kind} trial {t}: recovery {rec} s, resume {resume} s", file=sys.stderr, flush=True)
            runs.append({"recovery_s": rec, "resume_s": resume, "periods_ms": res["periods_ms"],
                         "fast_periods": res["fast_periods"], "fail_mode": res["fail_mode"],
                         "jobs": [{k: j[k] for k in ("model", "finished", "mean_ms", "p50_ms", "p95_ms")}
                                  for j in res["jobs"]]})
        xs = [r["recovery_s"] for r in runs if r["recovery_s"] is not None]
        ys = [r["resume_s"] for r in runs if r["resume_s"] is not None]
        ref_mean, ref_std, ref_trials = REF[kind]
        how = "killing (SIGKILL)" if a.fail_mode == "kill" else "hanging (SIGSTOP: sockets open, no FIN)"
        out = {"experiment": f"time to resume normal operation after {how} the {kind}"
                             + (" (coordinator)" if kind == "leader" else " (a non-coordinator member)"),
               "definition": "longest gap between consecutive query completions (either job) after the failure, "
                             "minus the median gap before it (tools/bench_jobs.py recovery_s)",
               "definition_resume": "time from the failure to the first completion from which the next 3 s hold at "
                                    "least 75% of the pre-failure completion rate (tools/bench_jobs.py resume_s)",
               "fail_mode": a.fail_mode,
               "resume_trials": ys, "resume_mean_s": round(statistics.mean(ys), 3) if ys else None,
               "resume_std_s": round(statistics.stdev(ys), 3) if len(ys) > 1 else None,
               "nodes": a.nodes, "executor": a.executor, "query_interval_ms": a.interval_ms,
               "periods_ms": runs[0]["periods_ms"], "fast_periods": runs[0]["fast_periods"],
               "trials": xs, "mean_s": round(statistics.mean(xs), 3),
               "std_s": round(statistics.stdev(xs), 3) if len(xs) > 1 else None,
               "reference": {"mean_s": ref_mean, "std_s": ref_std, "trials": ref_trials,
                             "source": "CS425MP4Report.pdf p.3 (10 VMs)"},
               "mechanisms": "a member's idle TCP watch on the leader's RPC port wakes its leader check as soon "
                             "as the leader's connections close (a crashed process); the new leader benches the "
                             "old one's member at take-over; standby job-state copies every "
                             f"{a.standby_copy_ms} ms "
                             "(csrc/control/member.cpp leader_watch_loop, csrc/serve/leader.cpp succession_loop)",
               "runs": runs}
        path = os.path.join(a.out_dir, f"{a.tag}_{kind}.json")
        with open(path, "w") as f:
            json.dump(out, f, indent=1)
        print(json.dumps({k: out[k] for k in ("experiment", "trials", "mean_s", "std_s", "resume_trials",
                                              "resume_mean_s", "periods_ms")}))


if __name__ == "__main__":
    main()
