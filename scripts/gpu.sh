#!/bin/bash
# Run one gpurun call; re-submit ONLY when gpurun reports an uncharged
# infrastructure transient (the box never ran the command).  A command that
# ran and failed is never retried.
cmd="$1"; timeout_s="${2:-900}"
for attempt in $(seq 1 ${GPU_TRIES:-6}); do
  out=$(timeout $((timeout_s + 900)) /usr/local/graft/bin/gpurun --timeout "$timeout_s" -- "$cmd" 2>&1)
  echo "$out" | tail -6
  if echo "$out" | grep -q "status=transient" && echo "$out" | grep -qE "charged=(0\.0s|Nones)"; then
    sleep $((30 * (attempt < 4 ? attempt : 4))); continue
  fi
  exit 0
done
echo "[gpu.sh] giving up after repeated transients"
