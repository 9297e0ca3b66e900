#!/bin/bash
# k_expand phase stamps (GS_XSTAMPS build at $1, GS_STAMPS=1): one N=1e9 C5
# flood broadcast; the per-phase means print at context teardown.
set -o pipefail
lib=${1:-gossip_simulator_amd/_build_xs/libgossip_hip.so}
mkdir -p gpurun_out
GS_STAMPS=1 GS_LIB_PATH=$lib timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --cpu-n 0 --no-roofline --no-extensions --no-c3 --no-c4 > gpurun_out/xstamps.json 2> gpurun_out/xstamps.err || { tail -5 gpurun_out/xstamps.err; exit 1; }
grep stamps gpurun_out/xstamps.err
