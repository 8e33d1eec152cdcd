#!/bin/bash
# Counter collection for the conv kernel (kernel-trace + pmc only, no sys/runtime trace).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/conv_bench.py --iters 10 > gpurun_out/conv_bench.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc -o pmc \
  --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU \
  -- python3 tools/conv_bench.py --iters 2 --tiles -1 > gpurun_out/pmc.log 2>&1
echo rc=$?
