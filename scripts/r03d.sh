#!/bin/bash
# Round-3 GPU call D: push-pull parity (with the pull-answer rounds), the full bench line (with
# the in-process shard scaling legs) and a kernel trace.
o=gpurun_out/r03d; mkdir -p $o
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python3 -u -m pytest tests/test_pushpull.py tests/test_full_size.py -m gpu -x -q --timeout 300 --timeout-method thread -k "pushpull" > $o/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $o/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python3 -u bench.py --steps 20 --warmup 5 --shard-scaling > $o/bench.json 2> $o/bench.err
rc=$?; echo "bench rc=$rc"; tail -c 600 $o/bench.json; grep -E "failed|Error" $o/bench.err | head -5
[ $rc -eq 0 ] || { tail -20 $o/bench.err; exit $rc; }
bash scripts/prof.sh r03d/prof > $o/prof.log 2>&1; echo "prof rc=$?"; head -25 gpurun_out/r03d/prof/kernel_summary.txt 2>/dev/null
