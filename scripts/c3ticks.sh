#!/bin/bash
# rocprofv3 kernel trace of one warm C3 batch overlay build (scripts/c3_ticks.py)
# and its per-tick split (scripts/ov_ticks.py).  Usage (inside gpurun): bash scripts/c3ticks.sh <tag> [trials]
set -o pipefail
o=gpurun_out/${1:-c3ticks}; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 rocprofv3 --kernel-trace -d $o/prof -o run -- python3 scripts/c3_ticks.py ${2:-5000} > $o/prof.log 2>&1 || { tail -20 $o/prof.log; exit 1; }
f=$(find $o/prof -name '*.db' | head -1)
python3 scripts/ov_ticks.py "$f" > $o/ov_ticks.txt && python3 tools_profsummary.py "$f" 16 > $o/kernel_summary.txt
find $o/prof -name '*.db' -delete
cat $o/prof.log | grep build; tail -3 $o/ov_ticks.txt; head -12 $o/kernel_summary.txt
