#!/bin/bash
# pooled head for throughput batches: head / pool tests, resnet50_fp8 + resnet18 benches, R50 kernel trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py tests/test_kernels_gpu.py -k "head or avgpool or resnet50" -q --timeout 200 --timeout-method thread > gpurun_out/r4m_t.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" gpurun_out/r4m_t.log | tail -14; [ $rc -le 1 ] || exit $rc
R="python bench.py --model resnet50_fp8 --latency-queries 0 --e2e-queries 0 --latency-steps 10 --steps 100 --warmup 20"
for i in 1 2; do
  timeout -k 10 300 $R > gpurun_out/r4m_r50_$i.log 2>&1 || { tail -20 gpurun_out/r4m_r50_$i.log; exit 1; }
  echo "resnet50_fp8 $(tail -1 gpurun_out/r4m_r50_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
timeout -k 10 300 python bench.py --latency-queries 0 --e2e-queries 0 > gpurun_out/r4m_r18.log 2>&1 || { tail -20 gpurun_out/r4m_r18.log; exit 1; }
echo "resnet18 $(tail -1 gpurun_out/r4m_r18.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4m_prof -o run -- python3 bench.py --model resnet50_fp8 --steps 20 --warmup 5 --prime-steps 5 --latency-queries 0 --e2e-queries 0 --latency-steps 2 > gpurun_out/r4m_prof.log 2>&1 || { tail -5 gpurun_out/r4m_prof.log; exit 1; }
python tools/lane_stats.py gpurun_out/r4m_prof/run_kernel_trace.csv --lat 2 2>&1 | head -24
