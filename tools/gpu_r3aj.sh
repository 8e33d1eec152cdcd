#!/bin/bash
# ResNet18 bench: prime steps 40 vs 120, lanes 2 vs 3, driver flags, interleaved on one box
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python bench.py --gpus 1 --steps 20 --warmup 5 --latency-queries 0 --e2e-queries 0 --latency-steps 5"
for rep in 1 2; do
  for arm in "--prime-steps 40" "--prime-steps 120" "--prime-steps 40 --lanes 3"; do
    timeout -k 10 200 $B $arm > gpurun_out/aj.log 2>&1 || { tail -20 gpurun_out/aj.log; exit 1; }
    echo "$arm: $(grep -o '"value": [0-9.]*' gpurun_out/aj.log)"
  done
done
