#!/bin/bash
# packed stem pooling (tests incl. bit-identity of the stem paths, engine vs fp32),
# stem knock-outs, then a same-box A/B of two builds: A = default, B = no SLP
# vectorisation (no packed f32 VALU next to the MFMAs) except conv3x3_rows28
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
LIB=distributed-machine-learning-cluster_amd/libdmlc_gpu.so
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -k "stem or b256 or batch1 or bench_path" -q --timeout 200 --timeout-method thread > gpurun_out/r4o_t.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" gpurun_out/r4o_t.log | tail -8; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/stem_roles_ab.py --rounds 3 --variants 0,16,52 > gpurun_out/r4o_ab.log 2>&1; rc=$?; tail -4 gpurun_out/r4o_ab.log; [ $rc -eq 0 ] || exit $rc
cp $LIB build/ab/libA_tree.so
for i in 1 2; do
  for v in A B; do
    cp build/ab/lib$v.so $LIB
    timeout -k 10 300 python bench.py --latency-queries 0 --e2e-queries 0 > gpurun_out/r4o_r18_$v$i.log 2>&1 || { tail -20 gpurun_out/r4o_r18_$v$i.log; cp build/ab/libA_tree.so $LIB; exit 1; }
    echo "resnet18 $v $(tail -1 gpurun_out/r4o_r18_$v$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
for v in A B; do
  cp build/ab/lib$v.so $LIB
  timeout -k 10 300 python bench.py --model resnet50_fp8 --latency-queries 0 --e2e-queries 0 --latency-steps 10 --steps 100 --warmup 20 > gpurun_out/r4o_r50_$v.log 2>&1 || { tail -20 gpurun_out/r4o_r50_$v.log; cp build/ab/libA_tree.so $LIB; exit 1; }
  echo "resnet50_fp8 $v $(tail -1 gpurun_out/r4o_r50_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
cp build/ab/libA_tree.so $LIB
