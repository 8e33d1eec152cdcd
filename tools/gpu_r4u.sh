#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for b in 64 256; do
  timeout -k 10 300 python -u tools/r50_fp8_diag.py $b > gpurun_out/r4u_$b.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/r4u_$b.log | grep -v "graph=True" | tail -12; [ $rc -eq 0 ] || exit $rc
done
