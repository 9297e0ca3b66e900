#!/bin/bash
# Full GPU evidence pass (inside gpurun): gpu tests, smoke, bench, rocprof stats.
# Usage: bash scripts/round.sh <tag>
tag=${1:-r02}
o=gpurun_out/$tag; mkdir -p $o
set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { tail -20 $o/smoke.log; exit 1; }
tail -1 $o/smoke.log
timeout -k 10 900 python -u bench.py > $o/bench.json 2> $o/bench.err || { tail -20 $o/bench.err; exit 1; }
cut -c1-300 $o/bench.json; grep "\[bench\]" $o/bench.err
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $o/prof -o run -- python3 bench.py --steps 2 --warmup 1 --cpu-n 0 --no-c3 > $o/prof.log 2>&1 || { tail -20 $o/prof.log; exit 1; }
f=$(find $o/prof -name '*.db' | head -1)
python3 tools_profsummary.py "$f" 30 > $o/kernel_summary.txt && python3 scripts/perwindow.py "$f" 28 > $o/perwindow.txt && python3 scripts/gaps.py "$f" > $o/gaps.txt
find $o/prof -name '*stats*.csv' -exec cp {} $o/ \;
find $o/prof -name '*.db' -delete
head -25 $o/kernel_summary.txt; cat $o/gaps.txt
