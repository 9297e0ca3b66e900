"""C4 at one shard (bench.py's flood_sharded at --gpus 1): where the wall time
over the kernels' time goes.  Times reset + broadcast_begin and run() apart
(a synchronise between them), then the GS_FLAG_TIMING run's kernel time.
Run under rocprofv3 --kernel-trace to see the gaps (scripts/gaps.py).
Usage: [C4_NO_TIMING=1] python scripts/c4_probe.py [reps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import gossip_simulator_amd as gs  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
gs.load()
cfg = gs.Config(n=100_000_000, fanout=18, fanin=19, crashrate=0.001, droprate=0.1, seed=0x5EED, device=0)
sim = gs.Simulator(cfg, devices=[0])
try:
    sim.build_overlay()
    for r in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sim.reset()
        sim.broadcast_begin(-1)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        polls, status = sim.run(poll=10)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"rep {r}: reset+begin {1e3 * (t1 - t0):.3f} ms  run {1e3 * (t2 - t1):.3f} ms  "
              f"ticks {sim.totals()['tick']} status {status}", flush=True)
    if os.environ.get("C4_NO_TIMING"):  # the trace's last broadcast is then a device-driven one
        raise SystemExit(0)
    sim.set_flags(True)
    sim.reset()
    sim.broadcast_begin(-1)
    sim.run(poll=10)
    tm = sim.timing()
    print(f"timing run: deliver {tm['deliver_ms']:.3f} ms  resolve {tm['resolve_ms']:.3f} ms  "
          f"launches {tm['resolve_launches']}", flush=True)
finally:
    sim.close()
