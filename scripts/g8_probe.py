"""In-process shards of one broadcast, device-driven (bench.py's
shards_inproc without the serial timing run): G shards on one GPU, one
overlay, a warm-up broadcast and REPS timed ones.  Run under rocprofv3
--kernel-trace with scripts/ddgaps.py for the last broadcast's per-kernel
busy and idle time.  Usage: python scripts/g8_probe.py [G] [n] [reps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import gossip_simulator_amd as gs  # noqa: E402

G = int(sys.argv[1]) if len(sys.argv) > 1 else 8
n = int(float(sys.argv[2])) if len(sys.argv) > 2 else 1_000_000_000
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 2
gs.load()
cfg = gs.Config(n=n, fanout=5, fanin=6, crashrate=0.01, droprate=0.1, seed=0x5EED, device=0)
with gs.Simulator(cfg, devices=[0] * G) as sim:
    sim.build_overlay()
    sim.broadcast_begin(-1)
    sim.run(poll=10)
    for r in range(reps):
        sim.reset()
        sim.broadcast_begin(-1)
        t0 = time.perf_counter()
        sim.run(poll=10)
        print(f"G={G} n={n} rep {r}: run {1e3 * (time.perf_counter() - t0):.2f} ms", flush=True)
