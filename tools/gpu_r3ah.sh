#!/bin/bash
# conv1x1 16-channel-per-lane e4m3 epilogue (w16) vs HEAD (nt): tests, resnet50_fp8 bench A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_fp8_gpu.py tests/test_engine_gpu.py -k "conv1x1 or resnet50" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_c1.log 2>&1 || { tail -40 gpurun_out/t_c1.log; exit 1; }
tail -1 gpurun_out/t_c1.log
R="python bench.py --model resnet50_fp8 --latency-queries 0 --e2e-queries 0 --latency-steps 10 --steps 100 --warmup 20"
bash tools/ab_bench.sh "$R" nt w16 nt w16
