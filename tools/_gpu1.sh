cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py tests/test_fp8_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
for m in resnet50_fp8 resnet50 resnet18; do timeout -k 10 200 python bench.py --model $m --latency-queries 20 >> gpurun_out/f8.log 2>&1 || exit 1; done
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/p_f8 -o run -- python3 bench.py --model resnet50_fp8 --steps 10 --warmup 3 --latency-queries 0 > gpurun_out/p_f8.log 2>&1 || exit 1
grep -ho '"metric": "[^"]*"\|"value": [0-9.]*' gpurun_out/f8.log
