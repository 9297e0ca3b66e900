#!/bin/bash
# One GPU round trip: window-engine parity tests, then a short bench.
# Usage (inside gpurun): bash scripts/quick.sh [pytest -k expr] [bench args...]
set -o pipefail
k=${1:-window}; shift || true
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$k" > gpurun_out/t.log 2>&1
rc=$?; tail -3 gpurun_out/t.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --cpu-n 0 "$@" > gpurun_out/b.log 2>&1
rc=$?; tail -2 gpurun_out/b.log | cut -c1-300
exit $rc
