#!/bin/bash
# strided 3x3 e4m3 outputs (fp8_3x3_out_s2: layer3.0 / layer4.0 conv2 on the implicit GEMM with an e4m3 epilogue) A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R="python bench.py --model resnet50_fp8 --latency-queries 0 --e2e-queries 0 --latency-steps 10 --steps 100 --warmup 20"
for i in 1 2; do
  for o in 0 1; do
    timeout -k 10 300 $R --engine-opt fp8_3x3_out_s2=$o > gpurun_out/r4w_r50_$o$i.log 2>&1 || { tail -20 gpurun_out/r4w_r50_$o$i.log; exit 1; }
    echo "fp8_3x3_out_s2=$o $(tail -1 gpurun_out/r4w_r50_$o$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4w_prof -o run -- python3 bench.py --model resnet50_fp8 --steps 20 --warmup 5 --prime-steps 5 --latency-queries 0 --e2e-queries 0 --latency-steps 2 > gpurun_out/r4w_prof.log 2>&1 || { tail -5 gpurun_out/r4w_prof.log; exit 1; }
python tools/lane_stats.py gpurun_out/r4w_prof/run_kernel_trace.csv --lat 2 2>&1 | head -32
