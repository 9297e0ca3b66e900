"""Config C3 probe: per-trial wall time of independent trials at N = 1e5
(overlay build + broadcast to 99 %), one GPU, through dist.run_one_trial."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gossip_simulator_amd as gs  # noqa: E402
from gossip_simulator_amd import dist  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
CONC = [int(x) for x in sys.argv[2:]] or [16]
cfg = gs.Config(n=100_000, crashrate=0.001, seed=0x5EED)
t_ov = t_bc = 0.0
for t in range(K):
    sim = gs.Simulator(gs.Config(**{**cfg.__dict__, "trial": t}))
    t0 = time.perf_counter()
    sim.build_overlay()
    t1 = time.perf_counter()
    sim.broadcast_begin(-1)
    sim.run(poll=10)
    t2 = time.perf_counter()
    sim.close()
    if t:  # first trial warms up
        t_ov += t1 - t0
        t_bc += t2 - t1
print(f"C3 probe: {K - 1} trials, overlay {t_ov / (K - 1) * 1e3:.2f} ms/trial, "
      f"broadcast {t_bc / (K - 1) * 1e3:.2f} ms/trial")
for conc in CONC:
    cfg1 = gs.Config(n=100_000, seed=0x5EED)
    dist.run_trials(gs.Simulator, cfg1, total=conc, concurrency=conc)
    t0 = time.perf_counter()
    dist.run_trials(gs.Simulator, cfg1, total=4 * conc, concurrency=conc)
    dt = time.perf_counter() - t0
    print(f"C3 probe: concurrency {conc}: {4 * conc / dt:.1f} trials/s")
