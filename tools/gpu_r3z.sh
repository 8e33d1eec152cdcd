#!/bin/bash
# same-box A/B of the block-kernel epilogue change: base (HEAD build) vs blk1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "block" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_block.log 2>&1 || { tail -30 gpurun_out/t_block.log; exit 1; }
tail -2 gpurun_out/t_block.log
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -k "resnet18" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_eng.log 2>&1 || { tail -30 gpurun_out/t_eng.log; exit 1; }
tail -2 gpurun_out/t_eng.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
bash tools/ab_bench.sh "python tools/block_bench.py" base blk1 base blk1 || exit 1
bash tools/ab_bench.sh "python bench.py --latency-queries 0 --e2e-queries 0 --latency-steps 10 --steps 200 --warmup 20" base blk1 base blk1
