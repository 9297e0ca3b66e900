"""C3 (bench.py's c3_trials leg) after a preceding heavy phase, in a fresh
process: does a large device allocation + free before it slow the batched
builds down?  Usage: python scripts/c3_after.py none|pp|alloc [GiB]
  none   C3 alone
  pp     an N = 1e9 push-pull context first (overlay + reverse table), closed
  alloc  a torch allocation of GiB (default 94) first, touched, freed, cache emptied"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
import gossip_simulator_amd as gs  # noqa: E402

mode = sys.argv[1]
gib = float(sys.argv[2]) if len(sys.argv) > 2 else 94.0
gs.load()
sys.argv = [sys.argv[0]]
a = bench.parse()
t0 = time.perf_counter()
if mode == "pp":
    cfg = gs.Config(n=a.n, fanout=a.fanout, fanin=a.fanin, delaylow=a.delaylow, delayhigh=a.delayhigh,
                    droprate=a.droprate, crashrate=a.crashrate, seed=a.seed, model="pushpull")
    with gs.Simulator(cfg) as sim:
        sim.build_overlay()
        sim.broadcast_begin(-1)
        torch.cuda.synchronize()
        tm = sim.timing()
        print(f"pp: overlay {tm['overlay_ms']:.0f} ms, prep {tm['prep_ms']:.0f} ms, rev_part {tm['pp_rev_part']}",
              flush=True)
elif mode == "alloc":
    x = torch.empty(int(gib * (1 << 30)), dtype=torch.uint8, device="cuda")
    x.fill_(1)
    torch.cuda.synchronize()
    del x
    torch.cuda.empty_cache()
    print(f"alloc: {gib} GiB touched and freed", flush=True)
torch.cuda.synchronize()
print(f"{mode}: first phase {time.perf_counter() - t0:.2f} s", flush=True)
r = bench.c3_trials(a, gs, 0, 1, 0, None)
print(f"{mode}: C3 {r['s_total']} s ({r['covered']} covered)", flush=True)
