#!/bin/bash
# stream-conv variants (PD 8, waves 4-7 at priority 1) + phase stamps
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/conv_bench.py --only l3,l4,l4.c1,l3.c1 --tiles none --variants 0,8,32,0,8,32 > gpurun_out/r4b_conv.log 2>&1 || { tail -20 gpurun_out/r4b_conv.log; exit 1; }
cat gpurun_out/r4b_conv.log | grep -v amdgpu.ids
DMLC_BT_DEBUG=32 timeout -k 10 300 python tools/conv_bench.py --only l3,l4,l4.c1,l3.c1 --tiles none --variants 0 > gpurun_out/r4b_stamps.log 2>&1 || { tail -20 gpurun_out/r4b_stamps.log; exit 1; }
cat gpurun_out/r4b_stamps.log | grep -v amdgpu.ids
