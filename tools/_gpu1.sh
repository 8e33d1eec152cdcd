cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py tests/test_node_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
for f in 1 0 1; do DMLC_GRAPH_DIRECT=$f timeout -k 10 120 python bench.py --latency-queries 50 >> gpurun_out/ab.log 2>&1 || exit 1; done
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl9 -o run -- python3 bench.py --steps 20 --warmup 5 --latency-queries 0 > gpurun_out/tl9.log 2>&1 || exit 1
grep -o '"value": [0-9.]*\|query_latency_p50_ms": [0-9.]*' gpurun_out/ab.log
