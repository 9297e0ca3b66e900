#!/bin/bash
# Round-3 GPU call Y: k_units / k_unitscan issue their L loads before the first use,
# k_cut no longer spills (launch bounds 256), window checks are selects, the
# small resolve loads its bucket before the check: -m gpu suite, smoke, trace, bench.
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r03y; mkdir -p $o
bash scripts/gtest.sh 600 > /dev/null || { tail -30 gpurun_out/gtest.log; exit 1; }
tail -1 gpurun_out/gtest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { tail -20 $o/smoke.log; exit 1; }
tail -1 $o/smoke.log
bash scripts/pw.sh r03y/pw > /dev/null && tail -1 $o/pw/perwindow.txt && head -14 $o/pw/kernel_summary.txt
timeout -k 10 900 python -u bench.py > $o/bench.json 2> $o/bench.err || { tail -20 $o/bench.err; exit 1; }
cut -c1-300 $o/bench.json; grep "\[bench\]" $o/bench.err
