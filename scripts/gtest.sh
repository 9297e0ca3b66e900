#!/bin/bash
# One gpurun step: the given pytest targets (default: every -m gpu test), each
# test under a thread timeout, the whole step under `timeout`.  Log in
# gpurun_out/gtest.log.  Usage: bash scripts/gtest.sh [budget_s] [pytest args...]
set -o pipefail
budget=${1:-600}; shift || true
mkdir -p gpurun_out
timeout -k 10 "$budget" python -u -m pytest -m gpu -x -v --timeout 240 --timeout-method thread "${@:-tests}" \
  > gpurun_out/gtest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/gtest.log | tail -40
exit $rc
