#!/bin/bash
# Round-3 GPU call V: the default bench line and smoke at HEAD (k_part2 tiles
# dealt by XCD), then a kernel trace of one C5 flood broadcast.
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r03v; mkdir -p $o
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { tail -20 $o/smoke.log; exit 1; }
tail -1 $o/smoke.log
timeout -k 10 900 python -u bench.py > $o/bench.json 2> $o/bench.err || { tail -20 $o/bench.err; exit 1; }
cut -c1-300 $o/bench.json; grep "\[bench\]" $o/bench.err
bash scripts/pw.sh r03v/pw > /dev/null && tail -1 $o/pw/perwindow.txt
