"""Multi-shard and batched-trial contexts against the one-device engine and
the oracle (bit-exact), on one GPU.

* Node-range shards (config C4): G shards of one
  broadcast -- gs_create_multi with device 0 repeated, and gs_create_rank
  with one rank (the RCCL path) -- must reproduce the unsharded run per poll
  and in the final bitsets.
* Batched trials (config C3): T trials in one context must reproduce T
  one-trial contexts trial by trial (overlay tables, stopping polls,
  counters), and match the oracle at N = 1e5.
* The native-RNG KS check of SURVEY.md section 8(c)4 at 1000 trials, N = 1e4.
"""
from __future__ import annotations

import concurrent.futures as cf

import numpy as np
import pytest
from scipy.stats import ks_2samp

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gs():
    import gossip_simulator_amd as mod
    mod.load()
    return mod


def cfg(gs, **kw):
    base = dict(n=50000, fanout=5, fanin=6, delaylow=10, delayhigh=20, droprate=0.1, crashrate=0.001,
                seed=0x5EED, trial=0)
    base.update(kw)
    return gs.Config(**base)


def run_polls(sim, polls=200):
    """Polls of 10 ticks until covered / nothing pending; returns the rows."""
    out = []
    for _ in range(polls):
        rows = sim.step(10)
        out.append(rows)
        last = rows[-1]
        if int(last[6]) == 0 or np.float32(int(last[4])) / np.float32(sim.n) >= np.float32(0.99):
            break
    return np.concatenate(out)


@pytest.fixture(scope="module")
def c4_table(gs):
    """Config C4's row shape (fanout 18 = floor(ln 1e8), fanin 19) at N = 1e6,
    GPU overlay, and the unsharded run over it."""
    c = cfg(gs, n=1_000_000, fanout=18, fanin=19, crashrate=0.02)
    with gs.Simulator(c) as sim:
        sim.build_overlay()
        deg, ids = sim.read_peers()
        sim.broadcast_begin(-1)
        rows = run_polls(sim)
        return c, deg, ids, rows, sim.received(), sim.crashed()


@pytest.mark.parametrize("G,mode", [(1, "dd"), (2, "dd"), (4, "dd"), (8, "dd"), (2, "host"), (8, "host")])
def test_shards_match_unsharded_c4_shape(gs, c4_table, G, mode, monkeypatch):
    """mode dd: device-driven shard windows (one device's shards on one
    stream; the first windows overflow the empty message buffers and are
    redone host-driven, which grows them); host: GS_SYNC_WINDOWS=1, every
    window host-driven."""
    if mode == "host":
        monkeypatch.setenv("GS_SYNC_WINDOWS", "1")
    c, deg, ids, rows, recv, crash = c4_table
    with gs.Simulator(c, devices=[0] * G) as sim:
        assert len(sim.shard_info()) == G and sim.shard_info()[-1][1] == c.n
        sim.load_peers(deg, ids)
        sim.broadcast_begin(-1)
        got = run_polls(sim)
        assert np.array_equal(got, rows)
        assert np.array_equal(sim.received(), recv)
        assert np.array_equal(sim.crashed(), crash)


@pytest.mark.parametrize("G", [1, 3, 8])
def test_shards_run_polls_like_unsharded(gs, c4_table, G):
    """gs_run over device-driven shard windows (the poll rule on the device,
    k_close_dd) gives the unsharded run's polls and status, three times.  The
    first broadcast's overflowing windows are redone host-driven, which grows
    the buffers to what those windows need; the later broadcasts run every
    window device-driven (dd_fallbacks stays: r04z found the fine buffer grown
    to exactly the bound k_rtab checks against its 16-element-short capacity,
    so the peak window was redone in every broadcast)."""
    c, deg, ids, _, recv, crash = c4_table
    with gs.Simulator(c) as one:
        one.load_peers(deg, ids)
        one.broadcast_begin(-1)
        ref, ref_status = one.run(poll=10)
    with gs.Simulator(c, devices=[0] * G) as sim:
        sim.load_peers(deg, ids)
        fb = []
        for _ in range(3):
            sim.reset()
            sim.broadcast_begin(-1)
            got, status = sim.run(poll=10)
            assert status == ref_status
            assert np.array_equal(got, ref)
            assert np.array_equal(sim.received(), recv) and np.array_equal(sim.crashed(), crash)
            fb.append(sim.timing()["dd_fallbacks"])
        assert fb[0] > 0 and fb[2] == fb[1] == fb[0], fb


def skewed_table(n, stride, frac, seed):
    """Random rows whose targets crowd into the first fine bucket: region
    estimates overflow (the coarse ones make a device-driven window stop and
    be redone host-driven; the fine ones are re-partitioned in the window, or,
    with one in-process shard (G = 1, no receive layout), stop it too)."""
    rng = np.random.default_rng(seed)
    deg = rng.integers(stride // 2, stride + 1, size=n).astype(np.uint8)
    hot = rng.random((n, stride)) < frac
    ids = np.where(hot, rng.integers(0, min(n, 16384), size=(n, stride)),
                   rng.integers(0, n, size=(n, stride))).astype(np.uint32)
    return deg, ids


@pytest.mark.parametrize("G,frac,n", [(1, 0.8, 60000), (2, 0.8, 60000), (3, 0.6, 100000)])
def test_shards_skewed_targets_match_oracle(gs, oracle, G, frac, n):
    stride = 6
    deg, ids = skewed_table(n, stride, frac, seed=G)
    c = cfg(gs, n=n, crashrate=0.03, droprate=0.05)
    p = oracle.make_params(n=n, fanout=c.fanout, fanin=c.fanin, delay_low=c.delaylow, delay_high=c.delayhigh,
                           drop_rate=c.droprate, crash_rate=c.crashrate, seed=c.seed, trial=0)
    for rep in range(2):  # the second broadcast runs on the grown buffers
        e = oracle.Engine(p, deg, ids)
        e.begin(-1)
        if rep == 0:
            sim = gs.Simulator(c, devices=[0] * G)
            sim.load_peers(deg, ids)
        else:
            sim.reset()
        sim.broadcast_begin(-1)
        for i in range(40):
            a, b = e.step(10), sim.step(10)
            assert np.array_equal(a, b), f"rep {rep} poll {i}"
            if int(a[-1][6]) == 0:
                break
        assert np.array_equal(e.received(), sim.received())
        assert np.array_equal(e.crashed(), sim.crashed())
    assert sim.timing()["exact_redos"] > 0  # an overflowed estimate was redone exactly
    sim.close()


def test_shard_overlay_matches(gs, c4_table):
    """Shards building the overlay themselves (replicated build, then each keeps
    its partition) give the same broadcast."""
    c, _, _, rows, recv, _ = c4_table
    with gs.Simulator(c, devices=[0, 0, 0]) as sim:
        sim.build_overlay()
        with pytest.raises(gs.GossipError):
            sim.read_peers()
        sim.broadcast_begin(-1)
        assert np.array_equal(run_polls(sim), rows)
        assert np.array_equal(sim.received(), recv)


def test_rank_of_one_uses_rccl_and_matches(gs, c4_table):
    """gs_create_rank with one rank: the RCCL all-gather / all-reduce path."""
    from gossip_simulator_amd import engine
    c, deg, ids, rows, recv, crash = c4_table
    sim = gs.Simulator.rank(c, 1, 0, engine.comm_unique_id())
    try:
        sim.load_peers(deg, ids)
        sim.broadcast_begin(-1)
        assert np.array_equal(run_polls(sim), rows)
        assert np.array_equal(sim.received(), recv) and np.array_equal(sim.crashed(), crash)
    finally:
        sim.close()


@pytest.mark.parametrize("kw,stride,G", [
    (dict(n=70001, droprate=0.29, crashrate=0.57), 6, 3),      # heavy crash, ragged last shard
    (dict(n=40000, delaylow=1, delayhigh=2, crashrate=0.05), 8, 2),  # hop mode: 1-tick windows
    (dict(n=50000, delaylow=0, delayhigh=3, droprate=0.0), 4, 2),    # 0-ms delays
])
def test_shards_match_oracle_injected(gs, oracle, kw, stride, G):
    rng = np.random.default_rng(kw["n"])
    n = kw["n"]
    deg = rng.integers(0, stride + 1, size=n).astype(np.uint8)
    ids = rng.integers(0, n, size=(n, stride)).astype(np.uint32)
    c = cfg(gs, **kw)
    p = oracle.make_params(n=n, fanout=c.fanout, fanin=c.fanin, delay_low=c.delaylow, delay_high=c.delayhigh,
                           drop_rate=c.droprate, crash_rate=c.crashrate, seed=c.seed, trial=0)
    e = oracle.Engine(p, deg, ids)
    e.begin(-1)
    with gs.Simulator(c, devices=[0] * G) as sim:
        sim.load_peers(deg, ids)
        sim.broadcast_begin(-1)
        for i in range(60):
            a, b = e.step(7), sim.step(7)
            assert np.array_equal(a, b), f"chunk {i}"
            assert np.array_equal(e.received(), sim.received())
            if int(a[-1][6]) == 0:
                break
        assert np.array_equal(e.crashed(), sim.crashed())


def test_shard_failed_mask_and_failed_sender(gs, oracle):
    n = 40000
    rng = np.random.default_rng(9)
    deg = np.full(n, 6, np.uint8)
    ids = rng.integers(0, n, size=(n, 6)).astype(np.uint32)
    bits = rng.random(n) < 0.05
    p = oracle.make_params(n=n, drop_rate=0.1, crash_rate=0.0, seed=3)
    sender = oracle.pick_sender(p)
    bits[sender] = False
    words = np.packbits(bits, bitorder="little").view(np.uint8)
    words = np.concatenate([words, np.zeros((-len(words)) % 8, np.uint8)]).view(np.uint64)
    for failed_sender in (False, True):
        b = bits.copy()
        b[sender] = failed_sender
        w = np.packbits(b, bitorder="little")
        w = np.concatenate([w, np.zeros((-len(w)) % 8, np.uint8)]).view(np.uint64)
        e = oracle.Engine(p, deg, ids)
        e.set_failed(w)
        e.begin(-1)
        with gs.Simulator(cfg(gs, n=n, crashrate=0.0, seed=3), devices=[0, 0]) as sim:
            sim.load_peers(deg, ids)
            sim.set_failed(w)
            sim.broadcast_begin(-1)
            a, bb = e.step(300), sim.step(300)
            assert np.array_equal(a, bb)
            assert np.array_equal(e.received(), sim.received())
            if failed_sender:
                assert int(a[-1][4]) == 0 and int(a[0][6]) == 0


# ---- batched trials (config C3) ---------------------------------------------
def single_trials(gs, c, T):
    """T one-trial contexts: tables, per-trial results, per-tick rows."""
    tabs, res, rows = [], [], []
    for t in range(T):
        with gs.Simulator(cfg(gs, **dict(c.__dict__, trial=c.trial + t, trials=1))) as sim:
            sim.build_overlay()
            tabs.append(sim.read_peers())
            sim.broadcast_begin(-1)
            sim.run(poll=10)
            res.append(sim.trial_results()[0])
    return tabs, np.array(res)


@pytest.mark.parametrize("n,T,crash", [(20000, 12, 0.01), (100_000, 4, 0.001), (16384, 5, 0.3)])
def test_batched_trials_match_single(gs, n, T, crash):
    c = cfg(gs, n=n, crashrate=crash, trial=3)
    tabs, want = single_trials(gs, c, T)
    with gs.Simulator(cfg(gs, n=n, crashrate=crash, trial=3, trials=T)) as sim:
        sim.build_overlay()
        deg, ids = sim.read_peers()
        for t in range(T):
            d0, i0 = tabs[t]
            assert np.array_equal(deg[t * n:(t + 1) * n], d0), f"trial {t} degrees"
            m = np.arange(i0.shape[1])[None, :] < d0[:, None]
            assert np.array_equal(np.where(m, ids[t * n:(t + 1) * n], 0), np.where(m, i0, 0)), f"trial {t} rows"
        sim.broadcast_begin(-1)
        polls, status = sim.run(poll=10)
        got = sim.trial_results()
    assert np.array_equal(got, want), f"\n{got}\n{want}"


def batch_run(sim):
    sim.build_overlay()
    sim.broadcast_begin(-1)
    sim.run(poll=10)
    return sim.trial_results()


def test_set_trial_renumbered_batches_match_fresh(gs):
    """bench.py's C3 loop (verdict r05 item 3a): a batched context renumbered
    with gs_set_trial after gs_reset, its overlay rebuilt in the kept
    workspace, equals a fresh context of the same trials, for two successive
    renumberings."""
    n, T = 100_000, 24
    with gs.Simulator(cfg(gs, n=n, crashrate=0.01, trial=0, trials=T)) as sim:
        first = batch_run(sim)
        for b in (T, 2 * T):
            sim.reset()
            sim.set_trial(b)
            got = batch_run(sim)
            with gs.Simulator(cfg(gs, n=n, crashrate=0.01, trial=b, trials=T)) as fresh:
                want = batch_run(fresh)
            assert list(got[:, 0]) == list(range(b, b + T))
            assert np.array_equal(got, want), f"batch at trial {b}:\n{got}\n{want}"
    with gs.Simulator(cfg(gs, n=n, crashrate=0.01, trial=0, trials=T)) as fresh:
        assert np.array_equal(batch_run(fresh), first)


def test_c3_batch_of_5000_matches_single_trials(gs):
    """One 5,000-trial batch at N = 1e5 (bench.py's C3 batch, 5e8 ids in one
    context) and its renumbering to trials 5000..9999 (the bench's second
    batch) equal fresh one-trial contexts at both ends and in the middle;
    single trials at 1e5 are oracle-pinned by the test below."""
    n, T = 100_000, 5000
    picks = (0, 1, 2499, 4999)
    with gs.Simulator(gs.Config(n=n, seed=0x5EED, trial=0, trials=T)) as sim:
        got = [batch_run(sim)]
        sim.reset()
        sim.set_trial(T)
        got.append(batch_run(sim))
    for b, res in zip((0, T), got):
        assert res.shape[0] == T and list(res[[0, -1], 0]) == [b, b + T - 1]
        for t in picks:
            with gs.Simulator(gs.Config(n=n, seed=0x5EED, trial=b + t)) as one:
                want = batch_run(one)[0]
            assert np.array_equal(res[t], want), f"trial {b + t}: {res[t]} vs {want}"


def test_batched_trial_windows_never_redo_their_coarse_plan(gs):
    """Round 6: a batched context's messages stay in
    their sender's trial, so each (coarse bin, XCD) region gets an exact
    upper bound from the window's firing nodes and never overflows -- the
    node-share estimate sent most windows of a C3 batch through an exact
    recount and a second expand.  400 trials of N = 1e5 (50 coarse bins,
    trials at different phases in every window)."""
    with gs.Simulator(cfg(gs, n=100_000, trials=400)) as sim:
        sim.build_overlay()
        sim.broadcast_begin(-1)
        sim.run(poll=10)
        res = sim.trial_results()
        tm = sim.timing()
    assert tm["coarse_redos"] == 0, tm["coarse_redos"]
    assert len(res) == 400 and int((res[:, 8] == 0).sum()) > 0


def test_batched_trials_injected_match_oracle_1e5(gs, oracle):
    """Config C3 size (N = 1e5), three trials: oracle overlay and oracle
    broadcast per trial vs one batched context fed the oracle's tables."""
    n, T = 100_000, 3
    tabs, want = [], []
    for t in range(T):
        p = oracle.make_params(n=n, seed=0x5EED, trial=t)
        deg, ids, _, _ = oracle.overlay(p)
        tabs.append((deg, ids))
        rows, _ = oracle.run_to_coverage(p, deg, ids)
        tick99 = next((int(r[0]) for r in rows if oracle.covered(int(r[4]), n)), 0)
        last = rows[-1]
        st = 0 if oracle.covered(int(last[4]), n) else 1
        want.append([t, tick99, int(last[0]), *[int(x) for x in rows[:, 1:4].sum(0)], int(last[4]),
                     int(last[5]), st])
    deg = np.concatenate([d for d, _ in tabs])
    ids = np.concatenate([i for _, i in tabs])
    with gs.Simulator(cfg(gs, n=n, trials=T)) as sim:
        sim.load_peers(deg, ids)
        sim.broadcast_begin(-1)
        sim.run(poll=10)
        got = sim.trial_results()
    assert np.array_equal(got, np.array(want)), f"\n{got}\n{np.array(want)}"
    with gs.Simulator(cfg(gs, n=n, trials=T)) as sim:  # and the GPU overlay is the oracle's
        sim.build_overlay()
        gdeg, gids = sim.read_peers()
        for t in range(T):
            d0, i0 = tabs[t]
            assert np.array_equal(gdeg[t * n:(t + 1) * n], d0)
            m = np.arange(i0.shape[1])[None, :] < d0[:, None]
            assert np.array_equal(np.where(m, gids[t * n:(t + 1) * n, :i0.shape[1]], 0), np.where(m, i0, 0))


def test_batched_per_tick_sums_and_bitsets(gs):
    """gs_step on a batch = the sum of the trials' per-tick rows; the batch's
    bitsets = the trials' bitsets."""
    n, T, ticks = 30000, 6, 150
    singles, recvs = [], []
    for t in range(T):
        with gs.Simulator(cfg(gs, n=n, crashrate=0.02, trial=t)) as sim:
            sim.build_overlay()
            sim.broadcast_begin(-1)
            singles.append(sim.step(ticks).astype(np.int64))
            recvs.append(sim.received())
    with gs.Simulator(cfg(gs, n=n, crashrate=0.02, trials=T)) as sim:
        sim.build_overlay()
        sim.broadcast_begin(-1)
        rows = sim.step(ticks).astype(np.int64)
        got = sim.received()
    want = np.sum(singles, axis=0)
    want[:, 0] = singles[0][:, 0]
    assert np.array_equal(rows, want)
    assert np.array_equal(got, np.stack(recvs))


def test_trials_split_over_members(gs):
    """gs_create_multi with trials: two batches on device 0 == one batch."""
    c = cfg(gs, n=20000, crashrate=0.01, trials=9)
    with gs.Simulator(c) as one:
        one.build_overlay()
        one.broadcast_begin(-1)
        one.run(poll=10)
        a = one.trial_results()
    with gs.Simulator(c, devices=[0, 0]) as two:
        two.build_overlay()
        two.broadcast_begin(-1)
        two.run(poll=10)
        b = two.trial_results()
    assert np.array_equal(a, b)
    assert list(b[:, 0]) == list(range(9))


# ---- native RNG vs the Go-like event model -----------
KS_KW = dict(n=10000, fanout=5, fanin=6, delay_low=10, delay_high=20, drop_rate=0.1, crash_rate=0.001,
             seed=0x5EED)  # the reference's defaults (simulator.go:187-193), N = 1e4
KS_TRIALS = 1000


def refsim_ticks(oracle, kw, trials, base=20_000):
    p = oracle.make_params(**dict(kw, trial=0))

    def one(s):
        r = oracle.refsim(p, base + s)
        return int(r.tick_99) if r.reached else None

    with cf.ThreadPoolExecutor(8) as ex:  # ctypes drops the GIL
        out = list(ex.map(one, range(trials)))
    return np.array([x for x in out if x is not None])


def gpu_ticks(gs, kw, trials):
    c = gs.Config(n=kw["n"], fanout=kw["fanout"], fanin=kw["fanin"], delaylow=kw["delay_low"],
                  delayhigh=kw["delay_high"], droprate=kw["drop_rate"], crashrate=kw["crash_rate"],
                  seed=kw["seed"], trials=trials)
    with gs.Simulator(c) as sim:
        sim.build_overlay()
        sim.broadcast_begin(-1)
        sim.run(poll=10)
        r = sim.trial_results()
    return r[r[:, 1] > 0, 1]  # first covered tick of the trials that got there


def test_gpu_native_rng_ks_1000_trials(gs, oracle):
    a = gpu_ticks(gs, KS_KW, KS_TRIALS)
    b = refsim_ticks(oracle, KS_KW, KS_TRIALS)
    assert len(a) > 0.9 * KS_TRIALS and len(b) > 0.9 * KS_TRIALS
    res = ks_2samp(a, b)
    assert res.pvalue > 0.01, (res, a.mean(), b.mean())
    # power: a one-tick shift of the delay range is rejected at this size
    c = refsim_ticks(oracle, dict(KS_KW, delay_low=11, delay_high=21), KS_TRIALS, base=40_000)
    assert ks_2samp(a, c).pvalue < 0.01


def refsim_degrees(oracle, n, runs, base=60_000):
    """Friends-list lengths of `runs` or_refsim overlays (the Go-like event
    model: one sequential stream, FIFO events), as a sample."""
    p = oracle.make_params(n=n, seed=0x5EED)
    ref = np.zeros(256, dtype=np.int64)
    for s in range(runs):
        ref += np.array(oracle.refsim(p, base + s).deg_hist[:256], dtype=np.int64)
    return np.repeat(np.arange(256), ref)


@pytest.mark.parametrize("n,trials", [(10_000, 40), (100_000, 8)])
def test_gpu_overlay_degree_ks(gs, oracle, n, trials):
    """KS (ks_2samp, p > 0.01) on overlay degrees, batched GPU
    overlays (simulator.go:66-106 restated tick-synchronously) vs or_refsim, at
    N = 1e4 and at C3's N = 1e5; a power check rejects fanin 7."""
    with gs.Simulator(gs.Config(n=n, seed=0x5EED, trials=trials)) as sim:
        sim.build_overlay()
        deg, _ = sim.read_peers()
    ref = refsim_degrees(oracle, n, trials)
    res = ks_2samp(deg.astype(np.int64), ref)
    assert res.pvalue > 0.01, (res, np.bincount(deg, minlength=8)[:8] / deg.size)
    alt = np.concatenate([oracle.overlay(oracle.make_params(n=n, seed=0x5EED, fanin=7, trial=t))[0]
                          for t in range(2)]).astype(np.int64)
    assert ks_2samp(deg.astype(np.int64), alt).pvalue < 0.01


def test_gpu_overlay_degree_histogram(gs, oracle):
    """Overlay degree histogram of 200 batched GPU trials vs or_refsim's
    Go-like overlay (one sequential stream, FIFO events): within 0.02 per bin."""
    n, T = 10000, 200
    with gs.Simulator(gs.Config(n=n, seed=0x5EED, trials=T)) as sim:
        sim.build_overlay()
        deg, _ = sim.read_peers()
    p = oracle.make_params(n=n, seed=0x5EED)
    ref = np.zeros(256)
    for s in range(20):
        ref += np.array(oracle.refsim(p, 60_000 + s).deg_hist[:256], dtype=float)
    h_gpu = np.bincount(deg, minlength=256)[:8] / deg.size
    h_ref = ref[:8] / ref.sum()
    assert np.abs(h_gpu - h_ref).max() < 0.02, (h_gpu, h_ref)
