#!/bin/bash
# round-4: sustained two-job throughput (shard jobs), per-op profiles (ResNet18 b256 single lane,
# resnet50_fp8), stem PMC passes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
log() { echo "== $*"; }
log batch-1 latency and head
timeout -k 10 200 python bench.py --steps 5 --warmup 2 --prime-steps 5 --latency-steps 5 --latency-queries 300 --e2e-queries 0 > gpurun_out/r4h_b1.log 2>&1 || { tail -20 gpurun_out/r4h_b1.log; exit 1; }
tail -1 gpurun_out/r4h_b1.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("b1 p50/p95", d["gpu_batch1_latency_p50_ms"], d["gpu_batch1_latency_p95_ms"])'
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4h_b1prof -o run -- python3 bench.py --steps 5 --warmup 2 --prime-steps 5 --latency-steps 5 --latency-queries 100 --e2e-queries 0 > gpurun_out/r4h_b1prof.log 2>&1 || { tail -5 gpurun_out/r4h_b1prof.log; exit 1; }
python tools/lane_stats.py gpurun_out/r4h_b1prof/run_kernel_trace.csv --lat 10 2>&1 | sed -n '/batch-1/,$p'
log jobs
timeout -k 10 120 python tools/make_shards.py --synthetic 1000 --per 250 --out /tmp/shards > gpurun_out/r4h_mk.log 2>&1 || { tail -5 gpurun_out/r4h_mk.log; exit 1; }
for cfg in "64 4" "128 4"; do
  set -- $cfg
  timeout -k 10 300 python tools/bench_jobs.py --nodes 1 --executor gpu --shards /tmp/shards --job-limit 200000 \
      --batch $1 --adaptive-window $2 --fast-periods --out gpurun_out/r4h_jobs_b$1_w$2.json > gpurun_out/r4h_jobs_b$1_w$2.log 2>&1 \
      || { tail -20 gpurun_out/r4h_jobs_b$1_w$2.log; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r4h_jobs_b$1_w$2.json')); print('batch $1 window $2', [(j['model'], j['images_per_s'], j['steady_images_per_s'], j['steady_p50_ms'], j['steady_p95_ms']) for j in d['jobs']])"
done
log per-op profiles
timeout -k 10 300 python bench.py --lanes 1 --steps 10 --warmup 2 --prime-steps 5 --latency-queries 0 --e2e-queries 0 --profile-ops > gpurun_out/r4h_ops_r18.log 2>&1 || { tail -20 gpurun_out/r4h_ops_r18.log; exit 1; }
timeout -k 10 300 python bench.py --model resnet50_fp8 --steps 10 --warmup 2 --prime-steps 5 --latency-queries 0 --e2e-queries 0 --profile-ops > gpurun_out/r4h_ops_r50.log 2>&1 || { tail -20 gpurun_out/r4h_ops_r50.log; exit 1; }
tail -1 gpurun_out/r4h_ops_r50.log | cut -c1-300
log stem PMC
timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4h_pmc1 -o p --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY -- python3 bench.py --lanes 1 --steps 10 --warmup 2 --prime-steps 5 --latency-steps 2 --latency-queries 0 --e2e-queries 0 > gpurun_out/r4h_pmc1.log 2>&1 || { tail -5 gpurun_out/r4h_pmc1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4h_pmc2 -o p --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_WAVES -- python3 bench.py --lanes 1 --steps 10 --warmup 2 --prime-steps 5 --latency-steps 2 --latency-queries 0 --e2e-queries 0 > gpurun_out/r4h_pmc2.log 2>&1 || { tail -5 gpurun_out/r4h_pmc2.log; exit 1; }
echo done
