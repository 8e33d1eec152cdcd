#!/bin/bash
# fused bottleneck profile: per-op eager times (engine test prints) and kernel trace of the resnet50_fp8 bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -k "bottleneck_img" -q -s --timeout 200 --timeout-method thread > gpurun_out/r4i_t.log 2>&1
rc=$?; grep -E "fused|passed|failed" gpurun_out/r4i_t.log | tail -14; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4i_prof -o run -- python3 bench.py --model resnet50_fp8 --steps 20 --warmup 5 --prime-steps 5 --latency-queries 0 --e2e-queries 0 --latency-steps 2 --engine-opt fused_bottleneck_img=1 > gpurun_out/r4i_prof.log 2>&1 || { tail -5 gpurun_out/r4i_prof.log; exit 1; }
python tools/lane_stats.py gpurun_out/r4i_prof/run_kernel_trace.csv --lat 2 2>&1 | head -30
