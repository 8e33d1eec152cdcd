#!/bin/bash
# fused bottleneck after the padded-grid change: numerics + knock-outs + resnet50_fp8 A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -k "bottleneck_img" -q -s --timeout 200 --timeout-method thread > gpurun_out/r4l_t.log 2>&1
rc=$?; grep -E "fused|passed|failed|Error" gpurun_out/r4l_t.log | tail -14; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python tools/bottleneck_img_bench.py --layers 3 --dbg 0,1,2,4,0 > gpurun_out/r4l_bi.log 2>&1 || { tail -20 gpurun_out/r4l_bi.log; exit 1; }
timeout -k 10 200 python tools/bottleneck_img_bench.py --layers 2,4 --dbg 0 >> gpurun_out/r4l_bi.log 2>&1 || { tail -20 gpurun_out/r4l_bi.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r4l_bi.log
R="python bench.py --model resnet50_fp8 --latency-queries 0 --e2e-queries 0 --latency-steps 10 --steps 100 --warmup 20"
for opt in 0 1 0 1; do
  timeout -k 10 300 $R --engine-opt fused_bottleneck_img=$opt > gpurun_out/r4l_r50_$opt.log 2>&1 || { tail -20 gpurun_out/r4l_r50_$opt.log; exit 1; }
  echo "fused_bottleneck_img=$opt $(tail -1 gpurun_out/r4l_r50_$opt.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
