"""Native-RNG check (BASELINE.json north star): the rounds-to-coverage
distribution of the keyed tick model must agree, under a two-sample KS test at
p > 0.01, with or_refsim -- an event-driven restatement of simulator.go that
consumes ONE sequential random stream in processing order (as math/rand's
global source does) and keeps its events in a time-ordered FIFO.

CPU: tick-model oracle vs or_refsim.  GPU: the HIP engine (overlay + broadcast,
keyed Philox, trial = sample index) vs or_refsim.
"""
from __future__ import annotations

import numpy as np
import pytest
from scipy.stats import ks_2samp

KW = dict(n=2000, fanout=5, fanin=6, delay_low=10, delay_high=20, drop_rate=0.1,
          crash_rate=0.0, seed=0x5EED)
SAMPLES = 300


def first_cover_tick(rows, n, covered):
    for r in rows:
        if covered(int(r[4]), n):
            return int(r[0])
    return None


def tick_model_sample(oracle, kw, trials):
    out = []
    for t in range(trials):
        p = oracle.make_params(**dict(kw, trial=t))
        deg, ids, _, _ = oracle.overlay(p)
        e = oracle.Engine(p, deg, ids)
        e.begin(-1)
        rows = e.step(400)
        out.append(first_cover_tick(rows, p.n, oracle.covered))
    return np.array([x for x in out if x is not None])


def refsim_sample(oracle, kw, trials, base=10_000):
    p = oracle.make_params(**dict(kw, trial=0))
    out = []
    for s in range(trials):
        r = oracle.refsim(p, base + s)
        if r.reached:
            out.append(int(r.tick_99))
    return np.array(out)


def test_tick_model_vs_refsim_rounds_to_99(oracle):
    a = tick_model_sample(oracle, KW, SAMPLES)
    b = refsim_sample(oracle, KW, SAMPLES)
    assert len(a) > 0.9 * SAMPLES and len(b) > 0.9 * SAMPLES
    res = ks_2samp(a, b)
    assert res.pvalue > 0.01, (res, a.mean(), b.mean())


def test_tick_model_vs_refsim_with_crash(oracle):
    kw = dict(KW, crash_rate=0.01, drop_rate=0.2)
    a = tick_model_sample(oracle, kw, SAMPLES)
    b = refsim_sample(oracle, kw, SAMPLES)
    res = ks_2samp(a, b)
    assert res.pvalue > 0.01, (res, a.mean(), b.mean())


def test_overlay_degree_histograms_agree(oracle):
    p = oracle.make_params(**dict(KW, n=20000))
    deg, _, _, _ = oracle.overlay(p)
    r = oracle.refsim(p, 77)
    h_tick = np.bincount(deg, minlength=256)[:8] / p.n
    h_ref = np.array(r.deg_hist[:8], dtype=float) / p.n
    assert np.abs(h_tick - h_ref).max() < 0.02, (h_tick, h_ref)


def test_overlay_degrees_ks(oracle):
    """SURVEY.md 8(c)4 on CPU: KS (p > 0.01) on overlay degrees, the tick-model
    overlay (what the GPU builds, bit-exact) vs or_refsim, 40 overlays each at
    N = 1e4; fanin 7 is rejected (power)."""
    n, runs = 10_000, 40
    a = np.concatenate([oracle.overlay(oracle.make_params(**dict(KW, n=n, trial=t)))[0]
                        for t in range(runs)]).astype(np.int64)
    p = oracle.make_params(**dict(KW, n=n))
    h = np.zeros(256, dtype=np.int64)
    for s in range(runs):
        h += np.array(oracle.refsim(p, 60_000 + s).deg_hist[:256], dtype=np.int64)
    b = np.repeat(np.arange(256), h)
    assert ks_2samp(a, b).pvalue > 0.01
    c = np.concatenate([oracle.overlay(oracle.make_params(**dict(KW, n=n, fanin=7, trial=t)))[0]
                        for t in range(2)]).astype(np.int64)
    assert ks_2samp(c, b).pvalue < 0.01


def test_ks_detects_a_real_difference(oracle):
    """Power check: a changed delay range must be rejected."""
    a = tick_model_sample(oracle, KW, 150)
    b = refsim_sample(oracle, dict(KW, delay_low=11, delay_high=21), 150)
    assert ks_2samp(a, b).pvalue < 0.01


@pytest.mark.gpu
def test_gpu_native_vs_refsim_rounds_to_99(oracle):
    import gossip_simulator_amd as gs
    kw = dict(KW, crash_rate=0.01)
    a = []
    for t in range(SAMPLES):
        cfg = gs.Config(n=kw["n"], fanout=5, fanin=6, delaylow=10, delayhigh=20,
                        droprate=kw["drop_rate"], crashrate=kw["crash_rate"], seed=kw["seed"],
                        trial=t)
        with gs.Simulator(cfg) as sim:
            sim.build_overlay()
            sim.broadcast_begin(-1)
            x = first_cover_tick(sim.step(400), kw["n"], gs.covered)
            if x is not None:
                a.append(x)
    b = refsim_sample(oracle, kw, SAMPLES)
    res = ks_2samp(np.array(a), b)
    assert res.pvalue > 0.01, (res, np.mean(a), b.mean())
