#!/bin/bash
# A/B in one gpurun call: bench (no extensions) with env A, then env B, then A again.
# Usage: bash scripts/ab.sh "ENV_A=1" "ENV_B=1" [bench args]
set -o pipefail
A=$1; B=$2; shift 2
mkdir -p gpurun_out
for tag in a1 b1 a2 b2; do
  case $tag in a*) e=$A;; b*) e=$B;; esac
  env $e timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --cpu-n 0 --no-extensions "$@" > gpurun_out/ab_$tag.json 2>/dev/null || exit 1
  python3 scripts/showbench.py gpurun_out/ab_$tag.json | head -1 | sed "s|^|$tag [$e] |"
done
