#!/bin/bash
# rocprofv3 kernel trace of one python script, then an analysis script over
# the trace database (the .db is deleted afterwards; the summaries stay).
# Usage (inside gpurun): bash scripts/kprof.sh <tag> <secs> <analysis.py|-> <script.py> [args...]
tag=$1; secs=$2; ana=$3; shift 3
o=gpurun_out/$tag; mkdir -p $o
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 "$secs" rocprofv3 --kernel-trace --stats -d $o/prof -o run -- python3 "$@" > $o/run.log 2>&1 || { tail -20 $o/run.log; exit 1; }
f=$(find $o/prof -name '*.db' | head -1)
python3 tools_profsummary.py "$f" 25 > $o/kernel_summary.txt
[ "$ana" != "-" ] && python3 "$ana" "$f" $ANA_ARGS > $o/analysis.txt
grep -v "^\s*$" $o/run.log | tail -12; head -16 $o/kernel_summary.txt; [ "$ana" != "-" ] && tail -30 $o/analysis.txt
find $o/prof -name '*.db' -delete
exit 0
