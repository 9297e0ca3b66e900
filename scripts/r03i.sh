#!/bin/bash
# Round-3 GPU call I: 16-B aligned long rows (C4) and the 20-slot expand:
# window-engine parity (incl. shards, C4 1e8 vs the port), the in-process
# scaling probe, then an A/B of the k_part2 tile (8192 x 512 vs 16384 x 1024).
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r03i; mkdir -p $o
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_vs_port.py tests/test_gpu_multi.py tests/test_rank_exchange.py \
  -k "not ks and not native_rng" > $o/tests.log 2>&1
rc=$?; tail -5 $o/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u scripts/shard_probe.py > $o/probe.log 2>&1
rc=$?; tail -6 $o/probe.log; [ $rc -eq 0 ] || exit $rc
bash scripts/abn.sh "GS_LIB_PATH=gossip_simulator_amd/_build_ab/libgossip_hip_p8k.so" "GS_AB=base"
