#!/bin/bash
# Round-3 GPU call E: window-engine parity after the k_resolve prefetch change, then A/B vs the previous library.
o=gpurun_out/r03e; mkdir -p $o
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_vs_port.py tests/test_gpu_multi.py tests/test_full_size.py -m gpu -x -q --timeout 300 --timeout-method thread -k "not ks and not native_rng and not pushpull" > $o/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $o/tests.log
[ $rc -eq 0 ] || exit $rc
bash scripts/abn.sh "GS_LIB_PATH=gossip_simulator_amd/_build_ab/libgossip_hip_a.so" "GS_AB=b"
