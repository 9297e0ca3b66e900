#!/bin/bash
# One GPU iteration (inside gpurun): all gpu tests, a short bench, a rocprof
# kernel trace with the per-window split.  Usage: bash scripts/iter.sh <tag> [bench args]
tag=${1:-it}; shift || true
o=gpurun_out/$tag; mkdir -p $o
set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --cpu-n 0 "$@" > $o/bench.json 2> $o/bench.err || { tail -20 $o/bench.err; exit 1; }
python3 scripts/showbench.py $o/bench.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prof -o run -- python3 bench.py --steps 1 --warmup 0 --cpu-n 0 --no-roofline --no-extensions "$@" > $o/prof.log 2>&1 || { tail -20 $o/prof.log; exit 1; }
f=$(find $o/prof -name '*.db' | head -1)
python3 tools_profsummary.py "$f" 12 > $o/kernel_summary.txt && python3 scripts/perwindow.py "$f" 40 > $o/perwindow.txt && tail -1 $o/perwindow.txt && head -8 $o/kernel_summary.txt
