#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a gpurun_out/steps.log
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc" | tee -a gpurun_out/steps.log
  tail -3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step gpu_tests 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread
step r18_bench 200 python bench.py --latency-queries 0 --e2e-queries 0 --latency-steps 10 --steps 200 --warmup 20
step r18_prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r18 -o run -- python3 bench.py --steps 20 --warmup 5 --latency-queries 0 --e2e-queries 0
