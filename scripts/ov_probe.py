"""Overlay build timing at N (default 1e9, C5's fanout 5 / fanin 6): builds
twice and prints the wall time and the per-10-tick makeup / breakup counts of
the last build (OV_BUILDS builds, default 2).  Run under rocprofv3 --kernel-trace for the per-tick split
(scripts/ov_ticks.py).  Usage: python scripts/ov_probe.py [n]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import gossip_simulator_amd as gs  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_000_000_000
gs.load()
cfg = gs.Config(n=n, fanout=5, fanin=6, crashrate=0.01, droprate=0.1, seed=0x5EED, device=0)
with gs.Simulator(cfg) as sim:
    for rep in range(int(os.environ.get("OV_BUILDS", "2"))):
        t0 = time.perf_counter()
        ws, ft = sim.build_overlay()
        print(f"build {rep}: {time.perf_counter() - t0:.3f} s  final tick {ft}", flush=True)
    for w in ws[:12]:
        print("  window", w, flush=True)
