#!/bin/bash
# bottleneck non-temporal store A/B; kernel traces of the ResNet18 and resnet50_fp8 benches (final state)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python tools/bottleneck_bench.py --dbg 0,4,0,4 > gpurun_out/bn_nt.log 2>&1 || { tail -20 gpurun_out/bn_nt.log; exit 1; }
grep -v amdgpu.ids gpurun_out/bn_nt.log
B="bench.py --steps 20 --warmup 5 --latency-queries 0 --e2e-queries 0 --latency-steps 20"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt18 -o run -- python3 $B > gpurun_out/kt18.log 2>&1 || { tail -20 gpurun_out/kt18.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt50 -o run -- python3 $B --model resnet50_fp8 > gpurun_out/kt50.log 2>&1 || { tail -20 gpurun_out/kt50.log; exit 1; }
find gpurun_out/kt18 gpurun_out/kt50 -name "*kernel_trace.csv" | head
