"""One N = 1e9 C5 overlay build (GS_OV_DEBUG=2 prints per-tick event counts)."""
import os, sys, time
sys.path.insert(0, "/root/repo" if os.path.exists("/root/repo") else ".")
import gossip_simulator_amd as gs
gs.load()
cfg = gs.Config(n=1_000_000_000, fanout=5, fanin=6, delaylow=10, delayhigh=20, droprate=0.1, crashrate=0.01, seed=12345)
with gs.Simulator(cfg) as sim:
    t0 = time.perf_counter(); sim.build_overlay(); print(f"overlay {time.perf_counter()-t0:.2f} s", flush=True)
