#!/bin/bash
# per-channel e4m3 scales for the 3x3 outputs (fp8_3x3_out): accuracy diagnostic, R50 tests, bench A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/r50_fp8_diag.py 64 > gpurun_out/r4t_64.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/r4t_64.log | grep -v "graph=True" | tail -14; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest tests/test_engine_gpu.py -k "resnet50" -q -s --timeout 300 --timeout-method thread > gpurun_out/r4t_t.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error|rel " gpurun_out/r4t_t.log | tail -12; [ $rc -eq 0 ] || exit $rc
R="python bench.py --model resnet50_fp8 --latency-queries 0 --e2e-queries 0 --latency-steps 10 --steps 100 --warmup 20"
for i in 1 2; do
  for o in 0 1; do
    timeout -k 10 300 $R --engine-opt fp8_3x3_out=$o > gpurun_out/r4t_r50_$o$i.log 2>&1 || { tail -20 gpurun_out/r4t_r50_$o$i.log; exit 1; }
    echo "fp8_3x3_out=$o $(tail -1 gpurun_out/r4t_r50_$o$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
