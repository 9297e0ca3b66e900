#!/bin/bash
# Round-3 GPU call C: shard rework (flood partition, push-pull shards, two-rank exchange), then the expand A/B.
o=gpurun_out/r03c; mkdir -p $o
cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python3 -u -m pytest tests/test_pushpull.py tests/test_rank_exchange.py tests/test_gpu_multi.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "not ks and not native_rng" > $o/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "FAILED|ERROR" $o/tests.log | tail -20; tail -2 $o/tests.log
[ $rc -eq 0 ] || exit $rc
bash scripts/abn.sh "GS_XH=0" "GS_XH=8" "GS_XH=4"
