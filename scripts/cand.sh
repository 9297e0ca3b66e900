#!/bin/bash
# Candidate build check in one gpurun call: window-engine parity tests on the
# candidate library ($1), then an A/B bench (default build vs candidate).
# Usage: bash scripts/cand.sh <lib.so> [pytest targets...]
set -o pipefail
lib=$1; shift
[ $# -gt 0 ] || set -- tests/test_gpu_parity.py tests/test_gpu_vs_port.py
GS_LIB_PATH=$lib bash scripts/gtest.sh 500 "$@" || exit 1
bash scripts/ab.sh "GS_AB=base" "GS_LIB_PATH=$lib"
