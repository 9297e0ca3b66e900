#!/bin/bash
# FETCH_SIZE per kernel of one N=1e9 flood broadcast for the default build and
# an experimental one (GS_LIB_PATH=$1), then A/B bench timing (scripts/ab.sh).
# Usage (inside gpurun): bash scripts/fetch_ab.sh <lib.so>
set -o pipefail
lib=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
args="--steps 1 --warmup 0 --no-roofline --no-extensions --cpu-n 0"
for tag in base exp; do
  if [ $tag = exp ]; then export GS_LIB_PATH=$lib; else unset GS_LIB_PATH; fi
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/fab_$tag -o run -- python3 bench.py $args > gpurun_out/fab_$tag.log 2>&1 || { echo "$tag pmc failed"; tail -5 gpurun_out/fab_$tag.log; exit 1; }
  python3 scripts/pmc_summary.py gpurun_out/fab_$tag > gpurun_out/fab_$tag.csv && rm -rf gpurun_out/fab_$tag/
  echo "== $tag"; head -6 gpurun_out/fab_$tag.csv
done
unset GS_LIB_PATH
bash scripts/ab.sh "GS_AB=a" "GS_LIB_PATH=$lib"
