#!/bin/bash
# PMC pass: effective clock (GRBM_GUI_ACTIVE / 8 / wall) and MFMA busy per ResNet18 kernel, single lane
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R="python3 bench.py --steps 3 --warmup 1 --prime-steps 1 --latency-queries 0 --e2e-queries 0 --latency-steps 1 --lanes 1"
P3="GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY"
timeout -s KILL 120 rocprofv3 --pmc $P3 -d gpurun_out/pmc_r3 -o p --output-format csv -- $R > gpurun_out/pmc_r3.log 2>&1 || exit 1
head -2 gpurun_out/pmc_r3/p_counter_collection.csv
echo pmc done
