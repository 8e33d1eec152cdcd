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
step stem_stagger 150 python tools/stem_knockouts.py --dbg 0
step r18_bench 200 python bench.py --latency-queries 0 --e2e-queries 0 --latency-steps 10 --steps 200 --warmup 20
step r50_tests 400 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_engine_gpu.py -k "resnet50"
grep -q " failed" gpurun_out/r50_tests.log && { echo "r50 tests failed: stopping"; exit 1; }
R="python bench.py --model resnet50_fp8 --latency-queries 0 --e2e-queries 0 --latency-steps 10 --steps 100"
step r50_bench 200 $R
step r50_nods 200 $R --engine-opt ds_into_expand=0
step r50_ops 200 $R --steps 5 --warmup 2 --prime-steps 5 --profile-ops
