#!/bin/bash
# Round-3 GPU call G: owner-expand flood shards (all-to-all of messages):
# shard parity tests (in-process G = 1..8, RCCL rank of one, two gloo ranks),
# the PMC passes of one C5 broadcast at HEAD, then the in-process scaling probe.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03g
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_multi.py -k "shard or rank" tests/test_rank_exchange.py > gpurun_out/r03g/tests.log 2>&1
trc=$?; tail -25 gpurun_out/r03g/tests.log
# a failed assertion (1) still leaves the GPU usable; anything else ends the call
[ $trc -eq 0 ] || [ $trc -eq 1 ] || exit $trc
bash scripts/pmc.sh gpurun_out/r03g/pmc > gpurun_out/r03g/pmc.log 2>&1; prc=$?; tail -12 gpurun_out/r03g/pmc.log
[ $prc -eq 0 ] || exit $prc
[ $trc -eq 0 ] || exit $trc
timeout -k 10 600 python -u scripts/shard_probe.py > gpurun_out/r03g/probe.log 2>&1
rc=$?; tail -12 gpurun_out/r03g/probe.log; exit $rc
