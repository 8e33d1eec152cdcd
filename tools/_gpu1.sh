cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
for st in 0 14 8; do echo "strip $st"; DMLC_ROWS_STRIP=$st timeout -k 10 300 python tools/interference_probe.py --modes none,sleep1,sleep4,sleep16 2>&1 | grep forward || exit 1; done
