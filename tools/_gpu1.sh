cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
for k in 0 1 2 3; do
DMLC_HEAD_KO=$k timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ko$k -o run -- python3 bench.py --steps 20 --warmup 5 --latency-queries 0 > gpurun_out/ko$k.log 2>&1 || exit 1
done
