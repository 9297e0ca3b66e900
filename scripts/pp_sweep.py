"""Push-pull bottom-up threshold sweep at N (default 1e9): for each
GS_PP_BOTTOM256 value k (dense rounds bottom-up once |I| >= n*k/256), the best
of 3 broadcasts, without and with 1 % failed nodes; results must not change.
Usage (on the GPU box): python scripts/pp_sweep.py [n] [k,k,...]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gossip_simulator_amd as gs  # noqa: E402
from pp_time import failed_mask, run  # noqa: E402


def main():
    n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_000_000_000
    ks = [int(k) for k in sys.argv[2].split(",")] if len(sys.argv) > 2 else [32, 64, 96, 128, 160, 256]
    cfg = gs.Config(n=n, fanout=5, fanin=6, droprate=0.1, crashrate=0.01, seed=0x5EED, model="pushpull")
    with gs.Simulator(cfg) as sim:
        sim.build_overlay()
        for failed in (False, True):
            if failed:
                sim.set_failed(failed_mask(n, 0.01, 0x5EED + 1))
            ref = None
            for k in ks:
                os.environ["GS_PP_BOTTOM256"] = str(k)
                res = [run(sim) for _ in range(3)]
                tm = sim.timing()
                dt = min(r[0] for r in res)
                tot = res[-1][1]
                key = (tot["tick"], tot["received"], tot["messages"], tot["sent"])
                same = "" if ref is None else (" same" if key == ref else " DIFFERENT")
                ref = ref or key
                print(f"{'failed ' if failed else ''}k={k:3d} {dt * 1e3:8.1f} ms rounds={tot['tick']} "
                      f"recv={tot['received']}{same}", flush=True)


if __name__ == "__main__":
    main()
