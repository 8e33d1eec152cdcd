#!/bin/bash
# fused bottleneck: non-temporal y stores (nt) vs plain (tmp), whole resnet50_fp8 bench, same box
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -k "fused_bottleneck or resnet50" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_r50.log 2>&1 || { tail -30 gpurun_out/t_r50.log; exit 1; }
tail -1 gpurun_out/t_r50.log
R="python bench.py --model resnet50_fp8 --latency-queries 0 --e2e-queries 0 --latency-steps 10 --steps 100 --warmup 20"
bash tools/ab_bench.sh "$R" tmp nt tmp nt
