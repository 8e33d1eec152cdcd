#!/bin/bash
# AlexNet direct 13x13 conv check + bench, bottleneck knockouts, shard jobs (b16 then b64)
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
step d13_tests 300 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_engine_gpu.py -k "alexnet"
grep -q " failed" gpurun_out/d13_tests.log && { echo "direct13 tests failed: stopping"; exit 1; }
B="python bench.py --model alexnet --latency-queries 0 --e2e-queries 0 --latency-steps 10"
step alex_d13 200 $B --engine-opt blaslt_fc=0
step alex_d13_ops 200 $B --engine-opt blaslt_fc=0 --steps 5 --warmup 2 --prime-steps 5 --profile-ops
step alex_nod13 200 $B --engine-opt blaslt_fc=0 --engine-opt direct13=0
step bn_knock 200 python tools/bottleneck_bench.py
step shard_jobs_b16 300 python tools/bench_jobs.py --nodes 1 --executor gpu --shards bench_data/shards --labels bench_data/synset_words.txt --batch 16 --adaptive-window 4 --fast-periods --port 21500 --out gpurun_out/shard_jobs_b16.json
step shard_jobs 300 python tools/bench_jobs.py --nodes 1 --executor gpu --shards bench_data/shards --labels bench_data/synset_words.txt --batch 64 --adaptive-window 4 --fast-periods --out gpurun_out/shard_jobs.json
