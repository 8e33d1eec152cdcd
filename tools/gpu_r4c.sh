#!/bin/bash
# weight-stationary layer1 block (variant 16) vs the streamed-weight block: test + A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "conv3x3_block" -x -q --timeout 120 --timeout-method thread > gpurun_out/r4c_t.log 2>&1 || { tail -30 gpurun_out/r4c_t.log; exit 1; }
tail -1 gpurun_out/r4c_t.log
timeout -k 10 200 python tools/block_bench.py --dbg 0,16,0,16,0,16 > gpurun_out/r4c_blk.log 2>&1 || { tail -20 gpurun_out/r4c_blk.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r4c_blk.log
