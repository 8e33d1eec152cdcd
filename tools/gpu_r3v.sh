#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r18b -o run -- python3 bench.py --steps 20 --warmup 5 --latency-queries 0 --e2e-queries 0 > gpurun_out/prof_r18b.log 2>&1
echo rc=$?
