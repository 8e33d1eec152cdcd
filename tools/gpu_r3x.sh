#!/bin/bash
# same-box A/B: the previous commit's build (_ab_head/) vs the working tree
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ROOT=$(pwd)
step() {
  local name=$1 to=$2 dir=$3; shift 3
  echo "== $name" | tee -a gpurun_out/steps.log
  (cd "$dir" && timeout -k 10 "$to" "$@") > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc" | tee -a gpurun_out/steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
B="python bench.py --latency-queries 0 --e2e-queries 0 --latency-steps 10 --steps 200 --warmup 20"
step old1 200 "$ROOT/_ab_head" $B
step new1 200 "$ROOT" $B
step old2 200 "$ROOT/_ab_head" $B
step new2 200 "$ROOT" $B
step new_noroles 200 "$ROOT" $B --engine-opt stem_roles=0
