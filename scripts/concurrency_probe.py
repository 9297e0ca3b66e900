"""Do two window pipelines overlap on one MI355X?  Two flood contexts of
N = n each (own streams), broadcast alone and then both at once from two
host threads: if A||B takes about max(A, B), the kernels (k_expand's gather,
k_resolve's LDS atomics) share the chip well and overlapping window w's
expand with window w-1's resolve would pay; if A + B, it would not.
Usage: python scripts/concurrency_probe.py [n] [reps]"""
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import gossip_simulator_amd as gs  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 400_000_000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
gs.load()
sims = []
for t in range(2):
    cfg = gs.Config(n=n, fanout=5, fanin=6, delaylow=10, delayhigh=20, droprate=0.1, crashrate=0.01,
                    seed=12345, trial=t)
    s = gs.Simulator(cfg)
    t0 = time.perf_counter()
    s.build_overlay()
    print(f"context {t}: overlay {time.perf_counter() - t0:.2f} s", flush=True)
    sims.append(s)


def one(s):
    s.reset()
    s.broadcast_begin(-1)
    s.run(poll=10)


for s in sims:  # warmup (packed rows, code objects)
    one(s)
torch.cuda.synchronize()
for r in range(reps):
    ta = []
    for s in sims:
        t0 = time.perf_counter()
        one(s)
        torch.cuda.synchronize()
        ta.append((time.perf_counter() - t0) * 1e3)
    th = [threading.Thread(target=one, args=(s,)) for s in sims]
    t0 = time.perf_counter()
    for x in th:
        x.start()
    for x in th:
        x.join()
    torch.cuda.synchronize()
    tab = (time.perf_counter() - t0) * 1e3
    print(f"rep {r}: A {ta[0]:.1f} ms, B {ta[1]:.1f} ms, sum {sum(ta):.1f}; A||B {tab:.1f} ms "
          f"({tab / sum(ta):.2f} of the sum, {tab / max(ta):.2f} of the max)", flush=True)
for s in sims:
    s.close()
