#!/bin/bash
# (1) batch-1 igemm tile x split sweep; (2) sustained two-job throughput over SDFS-staged shards (synthetic)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 python tools/b1_sweep.py --tiles 0,2,3,5,6,7,8,9,10 --splits 1,2,4,8,16,32 > gpurun_out/r4e_b1.log 2>&1 || { tail -20 gpurun_out/r4e_b1.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r4e_b1.log | cut -c1-200
timeout -k 10 120 python tools/make_shards.py --synthetic 1000 --per 250 --out /tmp/shards > gpurun_out/r4e_mk.log 2>&1 || { tail -5 gpurun_out/r4e_mk.log; exit 1; }
for cfg in "64 4" "128 4"; do
  set -- $cfg
  timeout -k 10 420 python tools/bench_jobs.py --nodes 1 --executor gpu --shards /tmp/shards --job-limit 200000 \
      --batch $1 --adaptive-window $2 --fast-periods --out gpurun_out/r4e_jobs_b$1_w$2.json > gpurun_out/r4e_jobs_b$1_w$2.log 2>&1 \
      || { tail -20 gpurun_out/r4e_jobs_b$1_w$2.log; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r4e_jobs_b$1_w$2.json')); print('batch $1 window $2', [(j['model'], j['images_per_s'], j['steady_images_per_s'], j['steady_p50_ms'], j['steady_p95_ms']) for j in d['jobs']])"
done
