#!/bin/bash
# One GPU session on a gpurun box, as a list of named steps run in order:
#
#   gpurun --timeout 1200 -- bash tools/gpu_session.sh <tag> <step> [<step> ...]
#
# steps:
#   tests            pytest -m gpu (the round-end suite)
#   smoke            __graft_entry__.smoke()
#   bench            the driver's command: bench.py --gpus 1 --steps 20 --warmup 5
#   bench200         bench.py --steps 200 --warmup 20 (ResNet18, no latency extras)
#   r50              bench.py --model resnet50_fp8 --steps 100 --warmup 20
#   trace:<model>    rocprofv3 kernel trace of a bench run (+ tools/lane_stats.py per-kernel medians
#                    of the single-lane forwards)
#   pmc:<model>      three rocprofv3 --pmc passes (SQ / FETCH_SIZE / WRITE_SIZE, kernel-trace only,
#                    each in its own run) of a short bench run; tools/roofline.py combines them
#   counters         rocprofv3 -L (the counters this box offers)
#   py:<script>      python tools/<script> (a probe or micro-bench); extra args after '--' in
#                    DMLC_PY_ARGS
#
# Every GPU step runs under its own time limit; the first step that faults,
# aborts or times out ends the session (never retried). Outputs land in
# gpurun_out/<tag>/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=$1
shift
OUT=gpurun_out/$tag
mkdir -p "$OUT"

step() {  # name timeout cmd...
  local name=$1 to=$2
  shift 2
  echo "== $name ($(date +%H:%M:%S))"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  tail -4 "$OUT/$name.log" | cut -c1-600
  echo "   rc=$rc"
  if [ $rc -ne 0 ]; then
    echo "stopping after $name (rc=$rc)"
    exit $rc
  fi
}

bench_short() {  # model: a short bench run whose dispatches are the model's b256 forward
  echo python3 bench.py --model "$1" --steps 4 --warmup 2 --prime-steps 2 --latency-steps 6 \
    --latency-queries 0 --e2e-queries 0
}

for s in "$@"; do
  case "$s" in
    tests)
      step tests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ;;
    smoke)
      step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" ;;
    bench)
      step bench 400 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    bench200)
      step bench200 400 python bench.py --steps 200 --warmup 20 --latency-queries 0 --e2e-queries 0 ;;
    r50)
      step r50 400 python bench.py --model resnet50_fp8 --steps 100 --warmup 20 --latency-queries 0 \
        --e2e-queries 0 --latency-steps 10 ;;
    trace:*)
      m=${s#trace:}
      step "trace_$m" 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_$m" -o run \
        -- python3 bench.py --model "$m" --steps 20 --warmup 5 --prime-steps 5 --latency-queries 0 \
        --e2e-queries 0 --latency-steps 50
      python tools/lane_stats.py "$OUT/trace_$m/run_kernel_trace.csv" --lat 50 > "$OUT/lane_stats_$m.txt" 2>&1
      head -30 "$OUT/lane_stats_$m.txt" ;;
    pmc:*)
      m=${s#pmc:}
      # shellcheck disable=SC2046
      step "pmc_sq_$m" 120 rocprofv3 --kernel-trace --output-format csv -d "$OUT/pmc_sq_$m" -o p --pmc \
        SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F8 SQ_INSTS_VALU_MFMA_MOPS_F6F4 SQ_INSTS_MFMA \
        SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -- $(bench_short "$m")
      step "pmc_fetch_$m" 120 rocprofv3 --kernel-trace --output-format csv -d "$OUT/pmc_fetch_$m" -o p --pmc \
        FETCH_SIZE -- $(bench_short "$m")
      step "pmc_write_$m" 120 rocprofv3 --kernel-trace --output-format csv -d "$OUT/pmc_write_$m" -o p --pmc \
        WRITE_SIZE -- $(bench_short "$m") ;;
    counters)
      step counters 120 rocprofv3 -L ;;
    py:*)
      # shellcheck disable=SC2086
      step "py_${s#py:}" 600 python -u "tools/${s#py:}" $DMLC_PY_ARGS ;;
    *)
      echo "unknown step $s"
      exit 2 ;;
  esac
done
echo "session done"
