#!/bin/bash
# role-split stem variants: bit-identity + A/B timings, stem tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "stem" -q --timeout 120 --timeout-method thread > gpurun_out/r4n_t.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" gpurun_out/r4n_t.log | tail -8; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/stem_roles_ab.py --rounds 5 --variants 0,64,1,2 > gpurun_out/r4n_ab.log 2>&1; rc=$?; cat gpurun_out/r4n_ab.log | tail -12; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -k "head" -q --timeout 120 --timeout-method thread > gpurun_out/r4n_th.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" gpurun_out/r4n_th.log | tail -8; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -u tools/head_bench.py > gpurun_out/r4n_hb.log 2>&1; rc=$?; tail -6 gpurun_out/r4n_hb.log; [ $rc -eq 0 ] || exit $rc
