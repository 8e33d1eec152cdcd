#!/bin/bash
# roctx marker trace + kernel trace of the serving path (no PMC counters:
# marker tracing and --pmc are never combined on this pool).
#   bench:  DP steps (dp.scatter / dp.predict / dp.gather) and, with
#           --profile-ops, one eager forward with a range per engine op.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --stats --output-format csv -d gpurun_out/trace -o run \
  -- python3 bench.py --steps 10 --warmup 3 --latency-queries 0 --profile-ops > gpurun_out/trace.log 2>&1
echo rc=$?
