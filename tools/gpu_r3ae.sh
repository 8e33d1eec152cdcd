#!/bin/bash
# layer1 block kernel knock-outs (tools/block_bench.py) + block test
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "block" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_block.log 2>&1 || { tail -30 gpurun_out/t_block.log; exit 1; }
tail -1 gpurun_out/t_block.log
timeout -k 10 200 python tools/block_bench.py --dbg 0,1,2,4,7,0 > gpurun_out/blk_ko.log 2>&1 || { tail -20 gpurun_out/blk_ko.log; exit 1; }
grep -v amdgpu.ids gpurun_out/blk_ko.log
