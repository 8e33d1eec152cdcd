#!/bin/bash
# ResNet50 layer2.0.conv2 row-streaming kernel (conv3x3_s2rows128) unit tests first, then the
# ResNet50 engine tests, then same-box bench A/B: s2rows128 on/off and the strided e4m3 outputs
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -k "s2rows128" -q --timeout 100 --timeout-method thread > gpurun_out/r4r_tk.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error|assert" gpurun_out/r4r_tk.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest tests/test_engine_gpu.py -k "resnet50" -q -s --timeout 300 --timeout-method thread > gpurun_out/r4r_t.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error|rel " gpurun_out/r4r_t.log | tail -12; [ $rc -eq 0 ] || exit $rc
R="python bench.py --model resnet50_fp8 --latency-queries 0 --e2e-queries 0 --latency-steps 10 --steps 100 --warmup 20"
for i in 1 2; do
  for o in "s2rows128=0" "s2rows128=1" "fp8_3x3_out=1"; do
    timeout -k 10 300 $R --engine-opt $o > gpurun_out/r4r_r50_$o$i.log 2>&1 || { tail -20 gpurun_out/r4r_r50_$o$i.log; exit 1; }
    echo "$o $(tail -1 gpurun_out/r4r_r50_$o$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4r_prof -o run -- python3 bench.py --model resnet50_fp8 --steps 20 --warmup 5 --prime-steps 5 --latency-queries 0 --e2e-queries 0 --latency-steps 2 > gpurun_out/r4r_prof.log 2>&1 || { tail -5 gpurun_out/r4r_prof.log; exit 1; }
python tools/lane_stats.py gpurun_out/r4r_prof/run_kernel_trace.csv --lat 2 2>&1 | head -30
