#!/bin/bash
# rocprofv3 kernel trace of one warm C3 batch broadcast (scripts/c3_bcast.py) and
# its kernel totals (scripts/c3_bcast_summary.py).  Usage (inside gpurun): bash scripts/c3bcast.sh <tag> [trials]
set -o pipefail
o=gpurun_out/${1:-c3bcast}; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 rocprofv3 --kernel-trace -d $o/prof -o run -- python3 scripts/c3_bcast.py ${2:-5000} > $o/prof.log 2>&1 || { tail -20 $o/prof.log; exit 1; }
f=$(find $o/prof -name '*.db' | head -1)
python3 scripts/c3_bcast_summary.py "$f" > $o/summary.txt
find $o/prof -name '*.db' -delete
grep broadcast $o/prof.log; cat $o/summary.txt
