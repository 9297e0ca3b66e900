#!/bin/bash
# A/B/C... in one gpurun call: bench (no extensions) once per env setting, the
# whole list twice (interleaved), one summary line each.
# Usage: bash scripts/abn.sh "ENV_A=1" "ENV_B=1" ... [-- bench args]
set -o pipefail
envs=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do envs+=("$1"); shift; done; [ "${1:-}" = "--" ] && shift
mkdir -p gpurun_out
for rep in ${ABN_REPS:-1 2}; do
  i=0
  for e in "${envs[@]}"; do
    i=$((i+1))
    env $e timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --cpu-n 0 --no-extensions "$@" > gpurun_out/abn_${i}_$rep.json 2>gpurun_out/abn_${i}_$rep.err || { tail -3 gpurun_out/abn_${i}_$rep.err; exit 1; }
    python3 scripts/showbench.py gpurun_out/abn_${i}_$rep.json | head -1 | sed "s|^|$rep [$e] |"
  done
done
