"""Push-pull timing probe (config C5 extension): one N-node GPU overlay, then
timed gs_broadcast_begin + gs_run for each round mode, without and with 1 %
failed nodes.  Usage (on the GPU box): python scripts/pp_time.py [n] [modes] [nofail|onlyfail]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gossip_simulator_amd as gs  # noqa: E402


def failed_mask(n, frac, seed):  # as bench.py's
    rng = np.random.default_rng(seed)
    idx = rng.integers(0, n, size=int(round(frac * n)), dtype=np.int64)
    w = np.zeros((n + 63) // 64, dtype=np.uint64)
    np.bitwise_or.at(w, idx >> 6, np.left_shift(np.uint64(1), (idx & 63).astype(np.uint64)))
    return w


def run(sim):
    t0 = time.perf_counter()
    sim.broadcast_begin(-1)
    polls, status = sim.run(poll=10)
    dt = time.perf_counter() - t0
    tot = sim.totals()
    sim.reset()
    return dt, tot, status


def main():
    n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_000_000_000
    modes = sys.argv[2].split(",") if len(sys.argv) > 2 else ["auto", "dense"]
    which = sys.argv[3] if len(sys.argv) > 3 else ""
    cfg = gs.Config(n=n, fanout=5, fanin=6, droprate=0.1, crashrate=0.01, seed=0x5EED, model="pushpull")
    with gs.Simulator(cfg) as sim:
        t0 = time.perf_counter()
        sim.build_overlay()
        print(f"overlay {time.perf_counter() - t0:.2f} s", flush=True)
        ref = None
        for m in modes if which != "onlyfail" else []:
            sim.cfg.pp_rounds = m
            sim.set_flags(False)
            run(sim)  # warmup (and the reverse-table build)
            prep = sim.timing()["prep_ms"]
            res = [run(sim) for _ in range(3)]
            dt = min(r[0] for r in res)
            tot, status = res[-1][1], res[-1][2]
            key = (tot["tick"], tot["received"], tot["messages"], tot["sent"])
            same = "" if ref is None else (" same" if key == ref else " DIFFERENT")
            ref = ref or key
            print(f"{m:6s} {dt * 1e3:8.1f} ms  rounds={tot['tick']} recv={tot['received']} msgs={tot['messages']} "
                  f"status={status} prep={prep:.1f} ms{same}", flush=True)
        if which == "nofail":
            return
        sim.set_failed(failed_mask(n, 0.01, 0x5EED + 1))
        ref = None
        for m in modes:
            sim.cfg.pp_rounds = m
            sim.set_flags(False)
            res = [run(sim) for _ in range(2)]
            prep = sim.timing()["prep_ms"]
            dt = min(r[0] for r in res)
            tot, status = res[-1][1], res[-1][2]
            key = (tot["tick"], tot["received"], tot["messages"], tot["sent"])
            same = "" if ref is None else (" same" if key == ref else " DIFFERENT")
            ref = ref or key
            print(f"failed {m:6s} {dt * 1e3:8.1f} ms  rounds={tot['tick']} recv={tot['received']} "
                  f"msgs={tot['messages']} status={status} prep={prep:.1f} ms{same}", flush=True)


if __name__ == "__main__":
    main()
