#!/bin/bash
# Round-3 measurements: RCCL interference at the weighted coordinator share,
# AlexNet with the fused stem (bench + kernel trace), and the two predict
# jobs over SDFS-staged real imagenet_1k shards (bench_data/, made by
# tools/make_shards.py) on one GPU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a gpurun_out/steps.log
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc" | tee -a gpurun_out/steps.log
  tail -3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step interference 300 python tools/interference_probe.py --batches 256,218 --modes none,rccl0:7,rccl0:1,none --iters 30
step bench_alexnet 300 python bench.py --model alexnet --steps 40 --warmup 10 --latency-queries 50 --e2e-queries 0
step prof_alexnet 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_alex -o run -- python3 bench.py --model alexnet --steps 20 --warmup 5 --latency-queries 0 --e2e-queries 0
step shard_jobs 600 python tools/bench_jobs.py --nodes 1 --executor gpu --shards bench_data/shards --labels bench_data/synset_words.txt --batch 64 --adaptive-window 4 --fast-periods --out gpurun_out/shard_jobs.json
step r50fp8_b256 300 python bench.py --model resnet50_fp8 --steps 20 --warmup 5 --latency-queries 0 --e2e-queries 0
step r50fp8_b128 300 python bench.py --model resnet50_fp8 --batch 128 --steps 40 --warmup 5 --latency-queries 0 --e2e-queries 0
