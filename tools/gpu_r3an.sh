#!/bin/bash
# fused bottleneck epilogue A/B: bnep (candidate) vs base (HEAD): test, microbench, resnet50_fp8 bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -k "fused_bottleneck or resnet50" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_bn.log 2>&1 || { tail -30 gpurun_out/t_bn.log; exit 1; }
tail -1 gpurun_out/t_bn.log
bash tools/ab_bench.sh "python tools/bottleneck_bench.py --dbg 0" base bnep base bnep || exit 1
R="python bench.py --model resnet50_fp8 --latency-queries 0 --e2e-queries 0 --latency-steps 10 --steps 100 --warmup 20"
bash tools/ab_bench.sh "$R" base bnep base bnep
