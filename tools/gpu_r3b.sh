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
step alex_tests 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_engine_gpu.py -k "alexnet"
step bench_alex 300 python bench.py --model alexnet
step prof_alex 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_alex2 -o run -- python3 bench.py --model alexnet --steps 20 --warmup 5 --latency-queries 0 --e2e-queries 0
step alex_ops 300 python bench.py --model alexnet --steps 5 --warmup 2 --prime-steps 5 --latency-queries 0 --e2e-queries 0 --profile-ops
step shard_jobs 600 python tools/bench_jobs.py --nodes 1 --executor gpu --shards bench_data/shards --labels bench_data/synset_words.txt --batch 64 --adaptive-window 4 --fast-periods --out gpurun_out/shard_jobs.json
step shard_jobs_b16 600 python tools/bench_jobs.py --nodes 1 --executor gpu --shards bench_data/shards --labels bench_data/synset_words.txt --batch 16 --adaptive-window 4 --fast-periods --port 21500 --out gpurun_out/shard_jobs_b16.json
