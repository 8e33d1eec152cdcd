#!/bin/bash
# PMC passes (kernel-trace-free, counters only) for the AlexNet stem and the ResNet18 stem / block
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
A="python3 bench.py --model alexnet --steps 3 --warmup 1 --prime-steps 1 --latency-queries 0 --e2e-queries 0 --latency-steps 1 --lanes 1"
R="python3 bench.py --steps 3 --warmup 1 --prime-steps 1 --latency-queries 0 --e2e-queries 0 --latency-steps 1 --lanes 1"
P1="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES"
timeout -s KILL 120 rocprofv3 --pmc $P1 -d gpurun_out/pmc_a1 -o p --output-format csv -- $A > gpurun_out/pmc_a1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc $P2 -d gpurun_out/pmc_a2 -o p --output-format csv -- $A > gpurun_out/pmc_a2.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc $P1 -d gpurun_out/pmc_r1 -o p --output-format csv -- $R > gpurun_out/pmc_r1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc $P2 -d gpurun_out/pmc_r2 -o p --output-format csv -- $R > gpurun_out/pmc_r2.log 2>&1 || exit 1
echo pmc done
