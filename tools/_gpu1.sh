cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
bash tools/gpu_check.sh test || exit 1
for f in 1 0 1; do
DMLC_STREAM_WREG=$f timeout -k 10 120 python bench.py --latency-queries 50 >> gpurun_out/ab.log 2>&1 || exit 1
done
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl7 -o run -- python3 bench.py --steps 20 --warmup 5 --latency-queries 0 > gpurun_out/tl7.log 2>&1 || exit 1
grep -o '"value": [0-9.]*\|query_latency_p50_ms": [0-9.]*' gpurun_out/ab.log
