cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/s3
for m in resnet50_fp8 resnet18; do
timeout -k 10 300 python bench.py --model $m --steps 10 --warmup 3 --latency-queries 0 --e2e-queries 0 --latency-steps 5 --profile-ops > gpurun_out/s3/ops_$m.log 2>&1 || { tail -5 gpurun_out/s3/ops_$m.log; exit 1; }
done
bash tools/gpu_session.sh s3 pmc:resnet18 pmc:resnet50_fp8 trace:resnet50_fp8
