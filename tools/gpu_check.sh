#!/bin/bash
# One GPU session: numerics tests, 1-GPU bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit; a fault/abort/timeout ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a gpurun_out/steps.log
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc" | tee -a gpurun_out/steps.log
  tail -5 "gpurun_out/$name.log"
  # 0 ok, 1 test failures (no fault): continue; anything else stops the session
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = test ]; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
  step bench1 300 python bench.py --profile-ops
fi
if [ "$MODE" = all ] || [ "$MODE" = prof ]; then
  step rocprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 20 --warmup 5 --latency-queries 0
fi
