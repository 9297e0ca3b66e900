#!/bin/bash
# Round-3 GPU call J: push-pull shards with the replica's early rounds at
# N = 1e9 (8 and 2 in-process shards), per-run wall time.
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r03j; mkdir -p $o
timeout -k 10 120 python -u -c "import torch; print(torch.cuda.is_available(), torch.cuda.device_count())" && timeout -k 10 600 python -u scripts/pp_shard_probe.py 8 > $o/pp8.log 2>&1
rc=$?; tail -4 $o/pp8.log; [ $rc -eq 0 ] || exit $rc
GS_PP_NO_REPLICA=1 timeout -k 10 600 python -u scripts/pp_shard_probe.py 8 > $o/pp8_norep.log 2>&1
rc=$?; tail -4 $o/pp8_norep.log; exit $rc
