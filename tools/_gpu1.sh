cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
for i in 1 2; do timeout -k 10 120 python bench.py --latency-queries 50 >> gpurun_out/ab.log 2>&1 || exit 1; done
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl10 -o run -- python3 bench.py --steps 20 --warmup 5 --latency-queries 0 > gpurun_out/tl10.log 2>&1 || exit 1
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|batch_latency_p50_ms": [0-9.]*' gpurun_out/ab.log
