#!/bin/bash
# fp8_3x3_out (per-channel scales) on by default: every ResNet50 engine test, bench A/B, ResNet18 bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_kernels_gpu.py -k "resnet50 or s2rows or conv1x1 or stream" -q -s --timeout 300 --timeout-method thread > gpurun_out/r4v_t.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error|rel " gpurun_out/r4v_t.log | tail -14; [ $rc -eq 0 ] || exit $rc
R="python bench.py --model resnet50_fp8 --latency-queries 0 --e2e-queries 0 --latency-steps 10 --steps 100 --warmup 20"
for i in 1 2; do
  for o in 1 0; do
    timeout -k 10 300 $R --engine-opt fp8_3x3_out=$o > gpurun_out/r4v_r50_$o$i.log 2>&1 || { tail -20 gpurun_out/r4v_r50_$o$i.log; exit 1; }
    echo "fp8_3x3_out=$o $(tail -1 gpurun_out/r4v_r50_$o$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
timeout -k 10 300 python bench.py --latency-queries 0 --e2e-queries 0 > gpurun_out/r4v_r18.log 2>&1 || { tail -20 gpurun_out/r4v_r18.log; exit 1; }
echo "resnet18 $(tail -1 gpurun_out/r4v_r18.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
