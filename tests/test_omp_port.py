"""The all-core CPU port (oracle/gsomp.c, bench.py's cpu_baseline) against the
single-thread restatement: identical per-tick counters and bitsets for every
thread count (keyed draws + rule A6 make the result order-free)."""
from __future__ import annotations

import numpy as np
import pytest


@pytest.mark.parametrize("kw,threads", [
    (dict(n=20000, crash_rate=0.02), 4),
    (dict(n=30000, drop_rate=0.29, crash_rate=0.57), 8),
    (dict(n=5000, delay_low=1, delay_high=2, crash_rate=0.05), 3),
    (dict(n=12345, fanout=18, fanin=19, crash_rate=0.01), 2),
])
def test_omp_port_matches_restatement(oracle, kw, threads):
    base = dict(fanout=5, fanin=6, delay_low=10, delay_high=20, drop_rate=0.1, crash_rate=0.001, seed=7, trial=1)
    base.update(kw)
    p = oracle.make_params(**base)
    deg, ids, _, _ = oracle.overlay(p)
    a = oracle.Engine(p, deg, ids)
    b = oracle.OmpEngine(p, deg, ids, threads=threads)
    assert b.threads == threads
    a.begin(-1)
    b.begin(-1)
    for _ in range(40):
        x, y = a.step(10), b.step(10)
        assert np.array_equal(x, y)
        if int(x[-1][6]) == 0:
            break
    assert np.array_equal(a.received(), b.received()) and np.array_equal(a.crashed(), b.crashed())


def test_omp_port_failed_sender(oracle):
    p = oracle.make_params(n=4000, seed=3)
    deg, ids, _, _ = oracle.overlay(p)
    s = oracle.pick_sender(p)
    w = np.zeros((4000 + 63) // 64, np.uint64)
    w[s // 64] |= np.uint64(1) << np.uint64(s % 64)
    for E in (oracle.Engine(p, deg, ids), oracle.OmpEngine(p, deg, ids, threads=2)):
        E.set_failed(w)
        E.begin(-1)
        r = E.step(50)
        assert int(r[-1][4]) == 0 and int(r[0][6]) == 0
