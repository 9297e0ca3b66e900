#!/bin/bash
# Round-3 GPU call H: flood shards read same-device blocks in place (no pack):
# shard parity tests, then the in-process scaling probe.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03h
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_multi.py tests/test_pushpull.py tests/test_rank_exchange.py -k "shard or rank" > gpurun_out/r03h/tests.log 2>&1
rc=$?; tail -25 gpurun_out/r03h/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u scripts/shard_probe.py > gpurun_out/r03h/probe.log 2>&1
rc=$?; tail -8 gpurun_out/r03h/probe.log; exit $rc
