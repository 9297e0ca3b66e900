"""C3 (10,000 trials of N = 1e5) on one GPU three ways, in one process:
  seq   bench.py's round-5 form: one 5,000-trial context, renumbered batch after batch
  mM    ONE gs_create_multi context of all 10,000 trials over M members on the same
        device (M = 2, 4): the members build their overlays and run their
        broadcasts concurrently, each on its own stream (par_members)
Each is created and run once untimed, then timed end to end for one pass over
all trials (overlay + broadcast + results); the trial tables must be equal.
  mMp   the same with the batched overlay ticks partitioned (GS_OV_PART_BATCHED=1)
Usage: python scripts/c3_members.py [total] [modes...]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gossip_simulator_amd as gs  # noqa: E402
from gossip_simulator_amd import _lib  # noqa: E402

total = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000
modes = sys.argv[2:] or ["seq", "m2", "m4"]
gs.load()
hip = _lib.load()
want = None
for mode in modes:
    # a trailing "p": batched overlay ticks by the destination partition
    # (GS_OV_PART_BATCHED=1, read per build) instead of the radix sort
    if mode.endswith("p"):
        os.environ["GS_OV_PART_BATCHED"] = "1"
    else:
        os.environ.pop("GS_OV_PART_BATCHED", None)
    members = int(mode[1:].rstrip("p")) if mode[0] == "m" else 1
    cfg = gs.Config(n=100_000, seed=0x5EED, trial=0, trials=total if mode != "seq" else 5000)
    t0 = time.perf_counter()
    sim = gs.Simulator(cfg, devices=[0] * members) if mode != "seq" else gs.Simulator(cfg)
    create = time.perf_counter() - t0

    split = [0.0, 0.0]

    def one_pass():
        rows = []
        split[0] = split[1] = 0.0
        for b in ((0,) if mode != "seq" else range(0, total, 5000)):
            sim.reset()
            sim.set_trial(b)
            a0 = time.perf_counter()
            sim.build_overlay()
            a1 = time.perf_counter()
            sim.broadcast_begin(-1)
            sim.run(poll=10)
            rows.append(sim.trial_results())
            split[0] += a1 - a0
            split[1] += time.perf_counter() - a1
        return np.concatenate(rows)

    w0 = time.perf_counter()
    one_pass()
    warm = time.perf_counter() - w0
    best, splits = [], []
    for _ in range(2):
        s0 = time.perf_counter()
        res = one_pass()
        best.append(time.perf_counter() - s0)
        splits.append(f"overlay {split[0]:.3f} + broadcast {split[1]:.3f}")
    sim.close()
    same = "n/a" if want is None else bool(np.array_equal(res, want))
    if want is None:
        want = res
    print(f"C3 {mode}: {len(res)} trials, create {create:.3f} s, first pass {warm:.3f} s, "
          f"timed passes {', '.join(f'{x:.3f}' for x in best)} s ({'; '.join(splits)}), equal to first mode: {same}",
          flush=True)
