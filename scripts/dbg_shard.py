"""Debug: first tick where oracle / unsharded / sharded(G) runs diverge."""
import sys
import numpy as np
sys.path.insert(0, ".")
import gossip_simulator_amd as gs
from oracle import pyoracle as O

n, stride = int(sys.argv[1]), int(sys.argv[2])
crash = float(sys.argv[3])
rng = np.random.default_rng(1)
deg = rng.integers(stride - 1, stride + 1, size=n).astype(np.uint8)
ids = rng.integers(0, n, size=(n, stride)).astype(np.uint32)
p = O.make_params(n=n, fanout=stride - 1, fanin=stride, crash_rate=crash, drop_rate=0.1, seed=0x5EED)
e = O.Engine(p, deg, ids)
e.begin(-1)
c = gs.Config(n=n, fanout=stride - 1, fanin=stride, crashrate=crash, droprate=0.1, seed=0x5EED)
sims = {"unsharded": gs.Simulator(c), "G1": gs.Simulator(c, devices=[0]), "G2": gs.Simulator(c, devices=[0, 0])}
for s in sims.values():
    s.load_peers(deg, ids)
    s.broadcast_begin(-1)
for t in range(1, 400):
    a = e.step(1)[0]
    out = {k: s.step(1)[0] for k, s in sims.items()}
    bad = [k for k, b in out.items() if not np.array_equal(a, b)]
    if bad:
        print("tick", t, "oracle", a)
        for k, b in out.items():
            print("  ", k, b)
        break
    if int(a[6]) == 0:
        print("all agree to the end, tick", t)
        break
