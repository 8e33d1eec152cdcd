#!/bin/bash
# (tools/gpu_try.sh <out> <gpurun args...>)
# retry gpurun ACQUISITION only (nothing ran / nothing charged), never a failed command
out=$1; shift
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun "$@" > "$out" 2>&1
  rc=$?
  if grep -q "status=transient" "$out" && grep -qE "no free box|backing off|taken away|stopped responding while being prepared|slot\(s\) on this pod are busy" "$out"; then
    w=$(grep -oE "retry in [0-9]+s" "$out" | grep -oE "[0-9]+" | head -1); w=${w:-150}
    sleep $((w + 10)); continue
  fi
  exit $rc
done
