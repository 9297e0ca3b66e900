#!/bin/bash
# Round-3 GPU call L: push-pull shards with pull-answer sharded rounds: parity
# (in-process shards vs the oracle and the unsharded run, two gloo ranks),
# then 8 in-process shards at N = 1e9.
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r03l; mkdir -p $o
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_pushpull.py tests/test_rank_exchange.py -k "shard or rank" > $o/tests.log 2>&1
rc=$?; tail -22 $o/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import torch; print(torch.cuda.is_available())" && \
timeout -k 10 600 python -u scripts/pp_shard_probe.py 8 > $o/pp8.log 2>&1
rc=$?; tail -3 $o/pp8.log; exit $rc
