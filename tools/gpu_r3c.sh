#!/bin/bash
# Fused ResNet50 bottleneck check + bench A/B, AlexNet hipBLASLt classifier A/B, shard-job benchmark
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
step bn_tests 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_engine_gpu.py -k "resnet50"
grep -q "failed" gpurun_out/bn_tests.log && { echo "bottleneck tests failed: stopping"; exit 1; }
R="python bench.py --model resnet50_fp8 --latency-queries 0 --e2e-queries 0 --latency-steps 10 --steps 100"
step r50_fused 200 $R
step r50_unfused 200 $R --engine-opt fused_bottleneck=0
step r50_ops 200 $R --steps 5 --warmup 2 --prime-steps 5 --profile-ops
B="python bench.py --model alexnet --latency-queries 0 --e2e-queries 0 --latency-steps 10"
step alex_blaslt_a 200 $B
step alex_igemm_a 200 $B --engine-opt blaslt_fc=0
step alex_blaslt_b 200 $B
step alex_igemm_b 200 $B --engine-opt blaslt_fc=0
step shard_jobs 400 python tools/bench_jobs.py --nodes 1 --executor gpu --shards bench_data/shards --labels bench_data/synset_words.txt --batch 64 --adaptive-window 4 --fast-periods --out gpurun_out/shard_jobs.json
