#!/bin/bash
# Round-3 GPU call Q: PMC passes of one C5 flood broadcast at HEAD
# (scripts/pmc.sh -> calibrated traffic per kernel), then a kernel trace with
# the per-window split (scripts/pw.sh).
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r03q; mkdir -p $o
bash scripts/pmc.sh $o/pmc > $o/pmc.log 2>&1 || { tail -12 $o/pmc.log; exit 1; }
tail -9 $o/pmc.log; head -c 1500 $o/pmc/pmc_traffic.json
bash scripts/pw.sh r03q/pw > /dev/null && tail -1 $o/pw/perwindow.txt
