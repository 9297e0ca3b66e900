#!/usr/bin/env python3
"""Per-window (10-tick poll) workload of the C5 flood broadcast: fires, delivered
sends, infections, and the mean receipts per 16384-node bucket -- the numbers
the per-window kernel split (scripts/perwindow.py) is read against."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gossip_simulator_amd as gs  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000_000
cfg = gs.Config(n=n, fanout=5, fanin=6, delaylow=10, delayhigh=20, droprate=0.1,
                crashrate=0.01, seed=0x5EED, trial=0, device=0)
nb = (n + 16383) // 16384
with gs.Simulator(cfg) as sim:
    sim.build_overlay()
    sim.broadcast_begin(-1)
    w = 0
    print("win  ticks      fired         sent     received  recv/bucket  infected/bucket")
    prev = 0
    while True:
        a = sim.step(10)
        fired, sent, recv = int(a[:, 1].sum()), int(a[:, 2].sum()), int(a[-1][4])
        print(f"{w:3d} {int(a[0][0]):4d}-{int(a[-1][0]):<4d} {fired:11d} {sent:12d} {recv:12d} "
              f"{sent / nb:11.1f} {(recv - prev) / nb:11.1f}")
        prev = recv
        w += 1
        if gs.covered(recv, n) or int(a[-1][6]) == 0 or w > 60:
            break
