#!/bin/bash
# conv1x1 8-wave variant: fp8/1x1 tests, ResNet50 engine tests, same-box A/B (c1x8 = 8 waves, 2 stages; c1ep = slim epilogue)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_fp8_gpu.py tests/test_engine_gpu.py -k "conv1x1 or resnet50" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_c1.log 2>&1 || { tail -40 gpurun_out/t_c1.log; exit 1; }
tail -2 gpurun_out/t_c1.log
R="python bench.py --model resnet50_fp8 --latency-queries 0 --e2e-queries 0 --latency-steps 10 --steps 100 --warmup 20"
bash tools/ab_bench.sh "$R" c1x8 c1ep c1x8 c1ep || exit 1
timeout -k 10 300 python bench.py --model resnet50_fp8 --latency-queries 0 --e2e-queries 0 --latency-steps 3 --steps 5 --warmup 2 --prime-steps 5 --profile-ops > gpurun_out/r50_ops.log 2>&1 || { tail -20 gpurun_out/r50_ops.log; exit 1; }
grep "per-op" gpurun_out/r50_ops.log | tr ',' '\n' | grep -E "conv1|conv3|downsample" | head -60
