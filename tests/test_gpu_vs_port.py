"""The window engine on the GPU against the CPU oracle at a size the
single-thread restatement would take minutes on: the all-core OpenMP port of
the same tick model (oracle/gsomp.c, bit-exact to the restatement for every
thread count, tests/test_omp_port.py) runs the broadcast over the table the GPU
overlay built.  Per-tick counters (fired, sent, TotalMessage, received,
crashed, pending) and the final received / crashed bitsets must be identical.

Config C5's parameters (fanout 5, fanin 6, delays 10-20, drop 0.1, crash 0.01)
at N = 1e8, and config C4 as BASELINE.json names it (N = 1e8, fanout 18 =
floor(ln 1e8), fanin 19; plus N = 2e7 of the same shape): dense windows
with tens of thousands of receipts per 16384-node bucket, crashed and
crash-rolled nodes in every bucket -- the k_resolve paths the small fixtures
only touch lightly."""
from __future__ import annotations

import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,fanout,fanin", [(100_000_000, 5, 6), (20_000_000, 18, 19),
                                            (100_000_000, 18, 19)])
def test_window_engine_matches_port(oracle, n, fanout, fanin):
    import gossip_simulator_amd as gs
    gs.load()
    kw = dict(fanout=fanout, fanin=fanin, delaylow=10, delayhigh=20, droprate=0.1, crashrate=0.01,
              seed=0x5EED, trial=3)
    cfg = gs.Config(n=n, device=0, **kw)
    p = oracle.make_params(n=n, fanout=fanout, fanin=fanin, delay_low=10, delay_high=20, drop_rate=0.1,
                           crash_rate=0.01, seed=0x5EED, trial=3)
    try:
        threads = min(64, len(os.sched_getaffinity(0)))
    except (AttributeError, OSError):
        threads = min(16, os.cpu_count() or 1)
    with gs.Simulator(cfg) as sim:
        sim.build_overlay()
        deg, ids = sim.read_peers()
        port = oracle.OmpEngine(p, deg, ids, threads=threads)
        del deg, ids
        sim.broadcast_begin(-1)
        port.begin(-1)
        polls = 0
        while True:
            a, b = port.step(10), sim.step(10)
            assert np.array_equal(a, b), f"poll {polls}: tick stats differ\n{a}\n{b}"
            polls += 1
            if gs.covered(int(a[-1][4]), n) or int(a[-1][6]) == 0:
                break
        assert polls > 10
        assert int(a[-1][5]) > 0, "some nodes crashed (the crashed / rolled paths ran)"
        assert np.array_equal(port.received(), sim.received())
        assert np.array_equal(port.crashed(), sim.crashed())
