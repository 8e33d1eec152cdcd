#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/r50_fp8_diag.py 64 > gpurun_out/r4s_64.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/r4s_64.log | tail -22; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/r50_fp8_diag.py 256 > gpurun_out/r4s_256.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/r4s_256.log | tail -22; [ $rc -eq 0 ] || exit $rc
