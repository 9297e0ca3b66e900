#!/bin/bash
# Round-3 GPU call B: the lane-pair expand (k_expand2): window parity tests, then A/B timing.
o=gpurun_out/r03b; mkdir -p $o
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_vs_port.py tests/test_full_size.py tests/test_gpu_multi.py -m gpu -x -q --timeout 300 --timeout-method thread -k "not ks and not native_rng" > $o/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $o/tests.log
[ $rc -eq 0 ] || exit $rc
bash scripts/abn.sh "GS_XH=0" "GS_XH=8" "GS_XH=4"
