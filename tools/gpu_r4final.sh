#!/bin/bash
# round-end check of the committed tree: the full GPU test suite, smoke(), the driver's
# bench command (N=1), the 200-step bench, ResNet50 e4m3, and a kernel trace of the bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== tests"
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/fin_t.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" gpurun_out/fin_t.log | tail -8; [ $rc -eq 0 ] || exit $rc
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin_smoke.log 2>&1; rc=$?; tail -3 gpurun_out/fin_smoke.log; [ $rc -eq 0 ] || exit $rc
echo "== bench (driver command)"
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/fin_bench_driver.log 2>&1; rc=$?; tail -1 gpurun_out/fin_bench_driver.log; [ $rc -eq 0 ] || exit $rc
echo "== bench 200 steps"
timeout -k 10 400 python bench.py --steps 200 --warmup 20 --latency-queries 0 --e2e-queries 0 > gpurun_out/fin_bench200.log 2>&1; rc=$?; tail -1 gpurun_out/fin_bench200.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
echo "== resnet50_fp8"
timeout -k 10 300 python bench.py --model resnet50_fp8 --latency-queries 0 --e2e-queries 0 --latency-steps 10 --steps 100 --warmup 20 > gpurun_out/fin_r50.log 2>&1; rc=$?; tail -1 gpurun_out/fin_r50.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
echo "== resnet50_fp8 strided e4m3 outputs (fp8_3x3_out_s2) A/B"
for o in 1 0; do
  timeout -k 10 300 python bench.py --model resnet50_fp8 --latency-queries 0 --e2e-queries 0 --latency-steps 10 --steps 100 --warmup 20 --engine-opt fp8_3x3_out_s2=$o > gpurun_out/fin_r50_s2_$o.log 2>&1 || { tail -5 gpurun_out/fin_r50_s2_$o.log; exit 1; }
  echo "fp8_3x3_out_s2=$o $(tail -1 gpurun_out/fin_r50_s2_$o.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
echo "== kernel trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fin_prof -o run -- python3 bench.py --steps 20 --warmup 5 --prime-steps 5 --latency-queries 0 --e2e-queries 0 --latency-steps 50 > gpurun_out/fin_prof.log 2>&1 || { tail -5 gpurun_out/fin_prof.log; exit 1; }
python tools/lane_stats.py gpurun_out/fin_prof/run_kernel_trace.csv --lat 50 > gpurun_out/fin_lane_stats.txt 2>&1; head -40 gpurun_out/fin_lane_stats.txt
