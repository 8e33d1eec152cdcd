#!/bin/bash
# PMC passes over the fused bottleneck microbenchmark (one counter group per run)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
C="python3 tools/bottleneck_bench.py --dbg 0 --iters 3 --reps 2"
i=0
for pmc in "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY" \
           "GRBM_GUI_ACTIVE FETCH_SIZE" "GRBM_GUI_ACTIVE WRITE_SIZE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/bnpmc$i -o p --pmc $pmc -- $C > gpurun_out/bnpmc$i.log 2>&1 || { echo "pass $i rc=$?"; tail -5 gpurun_out/bnpmc$i.log; exit 1; }
  python3 tools/pmc_summary.py bottleneck56 gpurun_out/bnpmc$i
done
