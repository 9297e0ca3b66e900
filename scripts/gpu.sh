#!/bin/bash
# Run one gpurun call; re-submit ONLY when gpurun reports an uncharged
# infrastructure transient (the box never ran the command).  A command that
# ran and failed is never retried.
cmd="$1"; timeout_s="${2:-900}"
for attempt in 1 2 3 4 5 6; do
  out=$(timeout $((timeout_s + 900)) /usr/local/graft/bin/gpurun --timeout "$timeout_s" -- "$cmd" 2>&1)
  echo "$out" | tail -6
  if echo "$out" | grep -q "status=transient" && echo "$out" | grep -qE "charged=(0\.0s|Nones)"; then
    sleep $((30 * attempt)); continue
  fi
  exit 0
done
echo "[gpu.sh] giving up after repeated transients"
