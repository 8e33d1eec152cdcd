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
grep -q " failed" gpurun_out/gpu_tests.log && { echo "gpu tests failed: stopping"; exit 1; }
step stem_bench 150 python tools/stem_knockouts.py --dbg 0 --stagger 0,2
step r18_bench 200 python bench.py --latency-queries 0 --e2e-queries 0 --latency-steps 10 --steps 200 --warmup 20
step alex_bench 200 python bench.py --model alexnet --latency-queries 0 --e2e-queries 0 --latency-steps 10 --steps 200 --warmup 20
