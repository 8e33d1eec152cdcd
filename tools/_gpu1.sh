cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
bash tools/gpu_check.sh test && bash tools/gpu_check.sh bench && \
timeout -k 10 300 python tools/interference_probe.py > gpurun_out/interference.log 2>&1; echo rc=$?; cat gpurun_out/interference.log | tail -8
