"""One C3 batch's overlay builds (5,000 trials of N = 1e5, bench.py's batch)
for a rocprofv3 kernel trace: the context is built, renumbered with
gs_set_trial and built again, so scripts/ov_ticks.py's "last build" is a warm
one.  Usage (inside gpurun):
  rocprofv3 --kernel-trace -d <dir> -o run -- python3 scripts/c3_ticks.py [trials]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gossip_simulator_amd as gs  # noqa: E402

T = int(sys.argv[1]) if len(sys.argv) > 1 else 5000
with gs.Simulator(gs.Config(n=100_000, seed=0x5EED, trial=0, trials=T)) as sim:
    for b in (0, T):
        if b:
            sim.reset()
            sim.set_trial(b)
        t0 = time.perf_counter()
        sim.build_overlay()
        tm = sim.timing()
        print(f"build at trial {b}: {(time.perf_counter() - t0) * 1e3:.0f} ms wall, overlay_ms {tm['overlay_ms']:.0f}, "
              f"ticks partitioned {tm['ov_part_ticks']} sorted {tm['ov_sort_ticks']}", flush=True)
