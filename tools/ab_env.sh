#!/bin/bash
# Same-box A/B of bench.py under environment toggles, interleaved:
#   gpurun -- bash tools/ab_env.sh <tag> <rounds> "<envA>" "<envB>" [bench args...]
# env strings like "X=1 Y=2" or "-" for none; outputs in gpurun_out/<tag>/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=$1; rounds=$2; ea=$3; eb=$4; shift 4
OUT=gpurun_out/$tag
mkdir -p "$OUT"
args=("$@")
[ ${#args[@]} -eq 0 ] && args=(--steps 200 --warmup 20 --latency-queries 0 --e2e-queries 0)
for r in $(seq 1 "$rounds"); do
  for v in A B; do
    e=$ea; [ "$v" = B ] && e=$eb; [ "$e" = "-" ] && e=""
    env $e timeout -k 10 300 python bench.py "${args[@]}" > "$OUT/$v$r.log" 2>&1 || { echo "bench $v$r failed"; exit 1; }
    printf '%s round %s [%s]: ' "$v" "$r" "$e"
    grep -o '"value": [0-9.]*' "$OUT/$v$r.log"
  done
done
