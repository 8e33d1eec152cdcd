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
step eng_tests 400 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_engine_gpu.py tests/test_kernels_gpu.py -k "resnet18 or rows or s2rows or block or bench_path"
grep -q " failed" gpurun_out/eng_tests.log && { echo "engine tests failed: stopping"; exit 1; }
R="python bench.py --latency-queries 0 --e2e-queries 0 --latency-steps 10"
step r18_bench 200 $R
step r18_ops 200 $R --steps 5 --warmup 2 --prime-steps 5 --profile-ops
step r18_bench2 200 $R
