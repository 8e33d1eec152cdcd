cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 240 python -u tools/bench_jobs.py --out gpurun_out/jobs_none.json > gpurun_out/jobs_none.log 2>&1 || { tail -20 gpurun_out/jobs_none.log; exit 1; }
tail -3 gpurun_out/jobs_none.log
timeout -k 10 240 python -u tools/bench_jobs.py --kill member --port 22000 --out gpurun_out/jobs_member.json > gpurun_out/jobs_member.log 2>&1 || { tail -20 gpurun_out/jobs_member.log; exit 1; }
tail -3 gpurun_out/jobs_member.log
timeout -k 10 240 python -u tools/bench_jobs.py --kill leader --fast-periods --port 23000 --out gpurun_out/jobs_leader.json > gpurun_out/jobs_leader.log 2>&1 || { tail -20 gpurun_out/jobs_leader.log; exit 1; }
tail -3 gpurun_out/jobs_leader.log
