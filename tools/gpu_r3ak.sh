#!/bin/bash
# ResNet18 block kernel with non-temporal y stores (blknt) vs HEAD (base)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "block" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_block.log 2>&1 || { tail -30 gpurun_out/t_block.log; exit 1; }
tail -1 gpurun_out/t_block.log
bash tools/ab_bench.sh "python tools/block_bench.py" base blknt base blknt || exit 1
bash tools/ab_bench.sh "python bench.py --latency-queries 0 --e2e-queries 0 --latency-steps 10 --steps 200 --warmup 20" base blknt base blknt
