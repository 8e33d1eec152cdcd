#!/bin/bash
# round-4 combined session: block WS A/B, R50 fused head, batch-1 sweep, jobs bench, stem PMC
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
log() { echo "== $*"; }
log tests
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -k "conv3x3_block or fused_head or bench_path or batch1" -x -q --timeout 120 --timeout-method thread > gpurun_out/r4f_t.log 2>&1 || { tail -30 gpurun_out/r4f_t.log; exit 1; }
tail -1 gpurun_out/r4f_t.log
log block A/B
timeout -k 10 200 python tools/block_bench.py --dbg 0,16,0,16,0,16 > gpurun_out/r4f_blk.log 2>&1 || { tail -20 gpurun_out/r4f_blk.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r4f_blk.log
log r50 fused head A/B
R="python bench.py --model resnet50_fp8 --latency-queries 0 --e2e-queries 0 --latency-steps 10 --steps 100 --warmup 20"
for opt in 0 1 0 1; do
  timeout -k 10 300 $R --engine-opt fused_head=$opt > gpurun_out/r4f_r50_$opt.log 2>&1 || { tail -20 gpurun_out/r4f_r50_$opt.log; exit 1; }
  echo "fused_head=$opt $(tail -1 gpurun_out/r4f_r50_$opt.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
log batch-1 sweep
timeout -k 10 240 python tools/b1_sweep.py --tiles 0,2,3,5,6,7,8,9,10 --splits 1,2,4,8,16,32 > gpurun_out/r4f_b1.log 2>&1 || { tail -20 gpurun_out/r4f_b1.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r4f_b1.log | cut -c1-120
log batch-1 latency A/B
for opt in 0 1 0 1; do
  timeout -k 10 200 python bench.py --steps 5 --warmup 2 --prime-steps 5 --latency-steps 5 --latency-queries 300 --e2e-queries 0 --engine-opt igemm_small_m=$opt > gpurun_out/r4f_b1lat_$opt.log 2>&1 || { tail -20 gpurun_out/r4f_b1lat_$opt.log; exit 1; }
  echo "igemm_small_m=$opt $(tail -1 gpurun_out/r4f_b1lat_$opt.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["gpu_batch1_latency_p50_ms"], d["gpu_batch1_latency_p95_ms"], d["value"])')"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4f_b1prof -o run -- python3 bench.py --steps 5 --warmup 2 --prime-steps 5 --latency-steps 5 --latency-queries 100 --e2e-queries 0 > gpurun_out/r4f_b1prof.log 2>&1 || { tail -5 gpurun_out/r4f_b1prof.log; exit 1; }
log stem PMC
timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4f_pmc1 -o p --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY -- python3 bench.py --lanes 1 --steps 10 --warmup 2 --prime-steps 5 --latency-steps 2 --latency-queries 0 --e2e-queries 0 > gpurun_out/r4f_pmc1.log 2>&1 || { tail -5 gpurun_out/r4f_pmc1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4f_pmc2 -o p --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_WAVES -- python3 bench.py --lanes 1 --steps 10 --warmup 2 --prime-steps 5 --latency-steps 2 --latency-queries 0 --e2e-queries 0 > gpurun_out/r4f_pmc2.log 2>&1 || { tail -5 gpurun_out/r4f_pmc2.log; exit 1; }
log jobs
timeout -k 10 120 python tools/make_shards.py --synthetic 1000 --per 250 --out /tmp/shards > gpurun_out/r4f_mk.log 2>&1 || { tail -5 gpurun_out/r4f_mk.log; exit 1; }
for cfg in "64 4" "128 4"; do
  set -- $cfg
  timeout -k 10 300 python tools/bench_jobs.py --nodes 1 --executor gpu --shards /tmp/shards --job-limit 200000 \
      --batch $1 --adaptive-window $2 --fast-periods --out gpurun_out/r4f_jobs_b$1_w$2.json > gpurun_out/r4f_jobs_b$1_w$2.log 2>&1 \
      || { tail -20 gpurun_out/r4f_jobs_b$1_w$2.log; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r4f_jobs_b$1_w$2.json')); print('batch $1 window $2', [(j['model'], j['images_per_s'], j['steady_images_per_s'], j['steady_p50_ms'], j['steady_p95_ms']) for j in d['jobs']])"
done
