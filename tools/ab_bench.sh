#!/bin/bash
# Same-box A/B of libdmlc_gpu.so builds: for each variant under build/ab/<name>/
# (a libdmlc_gpu.so built from another revision, see tools/ab_snapshot.sh),
# swap it into the package, run the given command, restore the tree's own
# library. Boxes differ by several percent, so kernel changes are judged on
# one box, arms interleaved (A B A B).
#   tools/ab_bench.sh "<cmd>" name1 name2 ...
# Every run has its own time limit; a fault / abort / timeout ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
CMD=$1
shift
PKG=distributed-machine-learning-cluster_amd
mkdir -p gpurun_out
mkdir -p /tmp/ab_tree && cp "$PKG"/libdmlc_gpu.so "$PKG"/_C*.so /tmp/ab_tree/
restore() { cp /tmp/ab_tree/*.so "$PKG/"; }
trap restore EXIT
for name in "$@"; do
  cp "build/ab/$name/"*.so "$PKG/"
  echo "== $name"
  timeout -k 10 300 bash -c "$CMD" > "gpurun_out/ab_$name.log" 2>&1
  rc=$?
  grep -v "amdgpu.ids" "gpurun_out/ab_$name.log" | tail -4 | cut -c1-240
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
done
