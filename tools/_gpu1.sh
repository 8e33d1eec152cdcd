cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python tools/interference_probe.py > gpurun_out/interference.log 2>&1 || exit 1
tail -6 gpurun_out/interference.log
