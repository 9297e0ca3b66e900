"""One C5 push-pull broadcast (N = 1e9 default, fanout 5 / fanin 6, droprate
0.1, no failed nodes) over a GPU-built overlay, for PMC passes
(scripts/pmc_pp.sh): the overlay, one broadcast (its begin builds the
reverse table), nothing else.  Prints the broadcast's rounds and messages.
Usage: python scripts/pp_once.py [n] [failed_fraction]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import gossip_simulator_amd as gs  # noqa: E402


def failed_mask(n, frac, seed):  # as bench.py's
    rng = np.random.default_rng(seed)
    idx = rng.integers(0, n, size=int(round(frac * n)), dtype=np.int64)
    w = np.zeros((n + 63) // 64, dtype=np.uint64)
    np.bitwise_or.at(w, idx >> 6, np.left_shift(np.uint64(1), (idx & 63).astype(np.uint64)))
    return w


def main():
    n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_000_000_000
    frac = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
    cfg = gs.Config(n=n, fanout=5, fanin=6, droprate=0.1, crashrate=0.0, seed=0x5EED, model="pushpull")
    with gs.Simulator(cfg) as sim:
        sim.build_overlay()
        if frac > 0:
            sim.set_failed(failed_mask(n, frac, 0x5EED + 1))
        t0 = time.perf_counter()
        sim.broadcast_begin(-1)
        _, status = sim.run(poll=10)
        dt = time.perf_counter() - t0
        tot = sim.totals()
        print(f"push-pull n={n} failed={frac}: rounds={tot['tick']} messages={tot['messages']} "
              f"calls={tot['fired']} status={status} {dt * 1e3:.1f} ms (incl. reverse-table build)", flush=True)


if __name__ == "__main__":
    main()
