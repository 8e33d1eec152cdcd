cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "rows or stream or engine or fused or graph" > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
for f in 0 1; do
DMLC_STREAM_WREG=$f timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tw$f -o run -- python3 bench.py --steps 20 --warmup 5 --latency-queries 0 > gpurun_out/tw$f.log 2>&1 || exit 1
done
