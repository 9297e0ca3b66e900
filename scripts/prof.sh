#!/bin/bash
# rocprofv3 kernel trace of a short C5 bench (no extensions): per-kernel
# summary, per-window split and GPU idle gaps of the last broadcast.
# Usage (inside gpurun): bash scripts/prof.sh <tag> [bench args...]
tag=${1:-prof}; shift || true
o=gpurun_out/$tag; mkdir -p $o
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $o/prof -o run -- python3 bench.py --steps 2 --warmup 1 --cpu-n 0 --no-extensions --no-roofline "$@" > $o/prof.log 2>&1 || { tail -20 $o/prof.log; exit 1; }
f=$(find $o/prof -name '*.db' | head -1)
python3 tools_profsummary.py "$f" 25 > $o/kernel_summary.txt && python3 scripts/perwindow.py "$f" 28 > $o/perwindow.txt && python3 scripts/gaps.py "$f" > $o/gaps.txt
cat $o/kernel_summary.txt | head -30; tail -1 $o/perwindow.txt; cat $o/gaps.txt
find $o/prof -name '*.db' -delete
