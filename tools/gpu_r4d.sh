#!/bin/bash
# (1) weight-stationary layer1 block (variant 16) test + A/B; (2) ResNet50 e4m3 fused head test + bench A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -k "conv3x3_block or fused_head" -x -q --timeout 120 --timeout-method thread > gpurun_out/r4d_t.log 2>&1 || { tail -30 gpurun_out/r4d_t.log; exit 1; }
tail -1 gpurun_out/r4d_t.log
timeout -k 10 200 python tools/block_bench.py --dbg 0,16,0,16,0,16 > gpurun_out/r4d_blk.log 2>&1 || { tail -20 gpurun_out/r4d_blk.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r4d_blk.log
R="python bench.py --model resnet50_fp8 --latency-queries 0 --e2e-queries 0 --latency-steps 10 --steps 100 --warmup 20"
for opt in 0 1 0 1; do
  timeout -k 10 300 $R --engine-opt fused_head=$opt > gpurun_out/r4d_r50_$opt.log 2>&1 || { tail -20 gpurun_out/r4d_r50_$opt.log; exit 1; }
  echo "fused_head=$opt $(tail -1 gpurun_out/r4d_r50_$opt.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
