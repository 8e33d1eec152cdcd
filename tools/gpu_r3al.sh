#!/bin/bash
# bf16 ResNet50 and ResNet34 benches on the final tree
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for m in resnet50 resnet34 alexnet; do
  timeout -k 10 300 python bench.py --model $m --latency-queries 0 --e2e-queries 0 --latency-steps 10 --steps 100 --warmup 20 > gpurun_out/b_$m.log 2>&1 || { tail -20 gpurun_out/b_$m.log; exit 1; }
  echo "$m $(grep -o '"value": [0-9.]*' gpurun_out/b_$m.log)"
done
