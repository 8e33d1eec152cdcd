#!/bin/bash
# fused bottleneck A/B after a change: numerics + per-block eager times, resnet50_fp8 bench on/off
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -k "bottleneck_img" -q -s --timeout 200 --timeout-method thread > gpurun_out/r4j_t.log 2>&1
rc=$?; grep -E "fused|passed|failed|Error" gpurun_out/r4j_t.log | tail -14; [ $rc -le 1 ] || exit $rc
R="python bench.py --model resnet50_fp8 --latency-queries 0 --e2e-queries 0 --latency-steps 10 --steps 100 --warmup 20"
for opt in 0 1 0 1; do
  timeout -k 10 300 $R --engine-opt fused_bottleneck_img=$opt > gpurun_out/r4j_r50_$opt.log 2>&1 || { tail -20 gpurun_out/r4j_r50_$opt.log; exit 1; }
  echo "fused_bottleneck_img=$opt $(tail -1 gpurun_out/r4j_r50_$opt.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
