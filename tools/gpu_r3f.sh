#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for sk in 1 2 4 8 16; do
  echo "== splitk $sk"
  DMLC_FC_SPLITK=$sk timeout -k 10 120 python bench.py --model alexnet --steps 5 --warmup 2 --prime-steps 5 --latency-queries 0 --e2e-queries 0 --latency-steps 3 --profile-ops > gpurun_out/fc_sk$sk.log 2>&1 || exit 1
  grep "per-op" gpurun_out/fc_sk$sk.log | tr ',' '\n' | grep classifier
done
