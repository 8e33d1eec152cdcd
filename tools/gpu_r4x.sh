#!/bin/bash
# PMC (two passes, tools/pmc_derived.py) of the resnet50_fp8 b256 forward (final tree) and of the ResNet18 forward
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
P1="GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY"
P2="SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_WAVES"
for m in resnet50_fp8 resnet18; do
  i=1
  for P in "$P1" "$P2"; do
    timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4x_${m}_$i -o p --pmc $P -- python3 bench.py --model $m --lanes 1 --steps 10 --warmup 2 --prime-steps 5 --latency-steps 2 --latency-queries 0 --e2e-queries 0 > gpurun_out/r4x_${m}_$i.log 2>&1 || { tail -5 gpurun_out/r4x_${m}_$i.log; exit 1; }
    i=$((i+1))
  done
  python tools/pmc_derived.py gpurun_out/r4x_${m}_1 gpurun_out/r4x_${m}_2 > gpurun_out/r4x_${m}_derived.txt 2>&1; head -30 gpurun_out/r4x_${m}_derived.txt | cut -c1-230
done
