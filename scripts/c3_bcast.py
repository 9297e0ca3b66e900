"""One C3 batch's broadcast (5,000 trials of N = 1e5) for a rocprofv3 kernel
trace: overlay, a warm broadcast, then a marker kernel-free gap and the
measured broadcast.  Prints the wall of each broadcast.  The trace's last
broadcast starts at the last k_schedule* kernel (scripts/c3_bcast_summary.py).
Usage: rocprofv3 --kernel-trace -d <dir> -o run -- python3 scripts/c3_bcast.py [trials]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gossip_simulator_amd as gs  # noqa: E402

T = int(sys.argv[1]) if len(sys.argv) > 1 else 5000
with gs.Simulator(gs.Config(n=100_000, seed=0x5EED, trial=0, trials=T)) as sim:
    sim.build_overlay()
    for i in range(2):
        sim.reset()
        time.sleep(0.05)
        t0 = time.perf_counter()
        sim.broadcast_begin(-1)
        polls, st = sim.run(poll=10)
        print(f"broadcast {i}: {(time.perf_counter() - t0) * 1e3:.1f} ms, {len(polls)} polls, status {st}, "
              f"exact fine redos so far {sim.timing()['exact_redos']}", flush=True)
