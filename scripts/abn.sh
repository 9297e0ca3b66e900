#!/bin/bash
# A/B/C... in one gpurun call: the C5 flood bench (no extensions) once per
# library build, twice round-robin.  Usage: bash scripts/abn.sh lib1.so lib2.so ...
# ("main" = gossip_simulator_amd/libgossip_hip.so)
set -o pipefail
mkdir -p gpurun_out/abn
for pass in 1 2; do
  for lib in "$@"; do
    tag=$(basename "$lib" .so)
    if [ "$lib" = main ]; then unset GS_LIB_PATH; else export GS_LIB_PATH=$PWD/gossip_simulator_amd/$lib; fi
    timeout -k 10 300 python -u bench.py --steps 6 --warmup 1 --cpu-n 0 --no-extensions --no-c3 --no-c4 \
      > gpurun_out/abn/${tag}_$pass.json 2>/dev/null || exit 1
    python3 scripts/showbench.py gpurun_out/abn/${tag}_$pass.json | head -2 | sed "s/^/$pass $tag /"
  done
done
unset GS_LIB_PATH
