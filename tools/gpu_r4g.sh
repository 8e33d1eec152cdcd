#!/bin/bash
# round-4 re-entry: GPU tests (numerics failures reported, crashes stop), bench,
# batch-1 latency A/B (query-batch conv), block WS A/B, R50 fused-bottleneck A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
log() { echo "== $*"; }
log new-kernel tests
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -k "conv_small or stem_conv_pool_u8 or bottleneck_img or batch1" -q --timeout 120 --timeout-method thread > gpurun_out/r4g_ts.log 2>&1
rc=$?; tail -3 gpurun_out/r4g_ts.log; [ $rc -le 1 ] || exit $rc
log bench
timeout -k 10 300 python bench.py > gpurun_out/r4g_bench.log 2>&1 || { tail -20 gpurun_out/r4g_bench.log; exit 1; }
tail -1 gpurun_out/r4g_bench.log
log batch-1 latency A/B
for opt in "small_conv=0" "small_conv=1" "small_conv=0" "small_conv=1"; do
  timeout -k 10 200 python bench.py --steps 5 --warmup 2 --prime-steps 5 --latency-steps 5 --latency-queries 300 --e2e-queries 0 --engine-opt $opt > gpurun_out/r4g_b1lat_$opt.log 2>&1 || { tail -20 gpurun_out/r4g_b1lat_$opt.log; exit 1; }
  echo "$opt $(tail -1 gpurun_out/r4g_b1lat_$opt.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["gpu_batch1_latency_p50_ms"], d["gpu_batch1_latency_p95_ms"], d["value"])')"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4g_b1prof -o run -- python3 bench.py --steps 5 --warmup 2 --prime-steps 5 --latency-steps 5 --latency-queries 100 --e2e-queries 0 > gpurun_out/r4g_b1prof.log 2>&1 || { tail -5 gpurun_out/r4g_b1prof.log; exit 1; }
log block A/B
timeout -k 10 200 python tools/block_bench.py --dbg 0,16,0,16,0,16 > gpurun_out/r4g_blk.log 2>&1 || { tail -20 gpurun_out/r4g_blk.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r4g_blk.log
log r50 fused bottleneck_img A/B
R="python bench.py --model resnet50_fp8 --latency-queries 0 --e2e-queries 0 --latency-steps 10 --steps 100 --warmup 20"
for opt in 0 1 0 1; do
  timeout -k 10 300 $R --engine-opt fused_bottleneck_img=$opt > gpurun_out/r4g_r50_$opt.log 2>&1 || { tail -20 gpurun_out/r4g_r50_$opt.log; exit 1; }
  echo "fused_bottleneck_img=$opt $(tail -1 gpurun_out/r4g_r50_$opt.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
log tests
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r4g_t.log 2>&1
rc=$?; grep -E "passed|failed|FAILED" gpurun_out/r4g_t.log | tail -12; [ $rc -le 1 ] || exit $rc
