#!/bin/bash
# fused R50 layer1 bottleneck v2: test vs unfused, knock-outs, bench A/B fused on/off
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -k "fused_bottleneck" -x -q -s --timeout 120 --timeout-method thread > gpurun_out/t_bn.log 2>&1 || { tail -40 gpurun_out/t_bn.log; exit 1; }
tail -3 gpurun_out/t_bn.log
timeout -k 10 200 python tools/bottleneck_bench.py --dbg 0,1,2,3,0 > gpurun_out/bn_ko.log 2>&1 || { tail -20 gpurun_out/bn_ko.log; exit 1; }
grep -v amdgpu.ids gpurun_out/bn_ko.log
R="python bench.py --model resnet50_fp8 --latency-queries 0 --e2e-queries 0 --latency-steps 10 --steps 100 --warmup 20"
for arm in 0 1 0 1; do
  timeout -k 10 300 $R --engine-opt fused_bottleneck=$arm > gpurun_out/r50_fb$arm.log 2>&1 || { tail -20 gpurun_out/r50_fb$arm.log; exit 1; }
  echo "fused_bottleneck=$arm $(grep -o '"value": [0-9.]*' gpurun_out/r50_fb$arm.log)"
done
