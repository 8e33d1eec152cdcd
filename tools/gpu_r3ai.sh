#!/bin/bash
# layer1.0 reduce+3x3 head kernel: tests, resnet50_fp8 bench A/B (base = 1db2de4 build)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py tests/test_fp8_gpu.py -k "resnet50 or bottleneck" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_h.log 2>&1 || { tail -40 gpurun_out/t_h.log; exit 1; }
tail -1 gpurun_out/t_h.log
R="python bench.py --model resnet50_fp8 --latency-queries 0 --e2e-queries 0 --latency-steps 10 --steps 100 --warmup 20"
bash tools/ab_bench.sh "$R" base head base head || exit 1
timeout -k 10 300 python bench.py --model resnet50_fp8 --latency-queries 0 --e2e-queries 0 --latency-steps 3 --steps 5 --warmup 2 --prime-steps 5 --profile-ops > gpurun_out/r50_ops.log 2>&1 || { tail -20 gpurun_out/r50_ops.log; exit 1; }
grep "per-op" gpurun_out/r50_ops.log | tr ',' '\n' | grep -E "layer1" 
