#!/bin/bash
# Round-3 GPU call X: k_cut's coarse-bin scan on wave shuffles (was an 8-step
# LDS scan, 16 barriers): full -m gpu suite, smoke, then a kernel trace.
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r03x; mkdir -p $o
bash scripts/gtest.sh 600 > /dev/null || { tail -30 gpurun_out/gtest.log; exit 1; }
tail -1 gpurun_out/gtest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { tail -20 $o/smoke.log; exit 1; }
tail -1 $o/smoke.log
bash scripts/pw.sh r03x/pw > /dev/null && tail -1 $o/pw/perwindow.txt && head -14 $o/pw/kernel_summary.txt
