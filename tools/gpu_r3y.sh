#!/bin/bash
# round-3 re-entry check: GPU tests, smoke, the driver's bench command, a kernel trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a gpurun_out/steps.log
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc" | tee -a gpurun_out/steps.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -30 "gpurun_out/$name.log"; exit $rc; fi
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step bench 300 python bench.py --gpus 1 --steps 20 --warmup 5
step bench200 300 python bench.py --latency-queries 0 --e2e-queries 0 --latency-steps 10 --steps 200 --warmup 20
tail -3 gpurun_out/pytest_gpu.log
tail -1 gpurun_out/smoke.log
tail -1 gpurun_out/bench.log
tail -1 gpurun_out/bench200.log
