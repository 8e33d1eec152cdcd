#!/bin/bash
# fused R50 layer1 bottleneck (bottleneck56.hip v1) knock-outs on the release build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python tools/bottleneck_bench.py --dbg 0,1,2,4,3,7,0 > gpurun_out/bn_ko.log 2>&1 || { tail -20 gpurun_out/bn_ko.log; exit 1; }
cat gpurun_out/bn_ko.log | grep -v amdgpu.ids
