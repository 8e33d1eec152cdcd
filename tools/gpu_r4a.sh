#!/bin/bash
# round-4 first box: GPU tests, 1-GPU bench, kernel trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4a_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r4a_pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r4a_bench.log 2>&1 || { tail -20 gpurun_out/r4a_bench.log; exit 1; }
tail -1 gpurun_out/r4a_bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4a_prof -o run -- python3 bench.py --steps 20 --warmup 5 --latency-queries 200 --e2e-queries 0 > gpurun_out/r4a_prof.log 2>&1 || { tail -20 gpurun_out/r4a_prof.log; exit 1; }
tail -1 gpurun_out/r4a_prof.log
