#!/bin/bash
# Round-3 GPU call A: the GPU test suite, smoke, FETCH/WRITE_SIZE calibration.
o=gpurun_out/r03a; mkdir -p $o
cd "$GRAFT_REPO_ROOT"
(nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)))") > $o/cpu.txt 2>&1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $o/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 $o/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $o/smoke.log; exit 1; }
tail -1 $o/smoke.log
bash scripts/calib.sh $o/calib > $o/calib.log 2>&1; echo "calib rc=$?"; tail -3 $o/calib.log
