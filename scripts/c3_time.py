"""Config C3 timing detail: per batch, context + overlay + broadcast wall time."""
import sys
import time
from dataclasses import replace

sys.path.insert(0, ".")
import gossip_simulator_amd as gs

total = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
batch = int(sys.argv[2]) if len(sys.argv) > 2 else 2500
cfg = gs.Config(n=100_000, seed=0x5EED)
for rep in range(2):
    t0 = time.perf_counter()
    sim = gs.Simulator(replace(cfg, trials=batch))
    for b in range(0, total, batch):
        a = time.perf_counter()
        if True:
            sim.reset()
            sim.set_trial(b)
            c = time.perf_counter()
            sim.build_overlay()
            o = time.perf_counter()
            sim.broadcast_begin(-1)
            polls, st = sim.run(poll=10)
            r = time.perf_counter()
            res = sim.trial_results()
        e = time.perf_counter()
        print(f"rep {rep} batch {b}: create {c - a:.3f} overlay {o - c:.3f} run {r - o:.3f} ({len(polls)} polls) "
              f"close {e - r:.3f}", flush=True)
    print(f"rep {rep}: {total} trials in {time.perf_counter() - t0:.2f} s", flush=True)
