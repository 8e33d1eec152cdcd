#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python tools/bottleneck_img_bench.py --layers 3 --dbg 0,1,2,4,0 > gpurun_out/r4k_bi.log 2>&1 || { tail -20 gpurun_out/r4k_bi.log; exit 1; }
timeout -k 10 200 python tools/bottleneck_img_bench.py --layers 2,4 --dbg 0 >> gpurun_out/r4k_bi.log 2>&1 || { tail -20 gpurun_out/r4k_bi.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r4k_bi.log
timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4k_pmc1 -o p --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY -- python3 tools/bottleneck_img_bench.py --layers 3 --dbg 0 --iters 3 --reps 2 > gpurun_out/r4k_pmc1.log 2>&1 || { tail -5 gpurun_out/r4k_pmc1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4k_pmc2 -o p --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_WAVES -- python3 tools/bottleneck_img_bench.py --layers 3 --dbg 0 --iters 3 --reps 2 > gpurun_out/r4k_pmc2.log 2>&1 || { tail -5 gpurun_out/r4k_pmc2.log; exit 1; }
python tools/pmc_summary.py bottleneck_img gpurun_out/r4k_pmc1 gpurun_out/r4k_pmc2
