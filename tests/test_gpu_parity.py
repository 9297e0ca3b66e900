"""Parity of the HIP engine (through the C ABI) against the CPU restatement.

Bar: bit-exact -- per-tick counters and the per-tick received bitset (and the
crashed bitset) must equal the oracle's on the same injected peer table and
keyed Philox decisions; the GPU overlay must produce the oracle's table.
"""
from __future__ import annotations

import hashlib
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = ["a_n100_tick", "b_n1000_default", "c_n4133_hop", "d_n10000_crash"]


class _Engine:
    """The package, plus which broadcast engine the Configs should select."""

    def __init__(self, mod, engine):
        self.mod, self.engine = mod, engine

    def __getattr__(self, k):
        return getattr(self.mod, k)


@pytest.fixture(scope="module", params=["window", "tick"])
def gs(request):
    import gossip_simulator_amd as mod
    mod.load()  # fails loudly if the in-tree library is missing
    return _Engine(mod, request.param)


def cfg_from(gs, kw):
    return gs.Config(n=kw["n"], fanout=kw["fanout"], fanin=kw["fanin"], delaylow=kw["delay_low"],
                     delayhigh=kw["delay_high"], droprate=kw["drop_rate"],
                     crashrate=kw["crash_rate"], seed=kw["seed"], trial=kw["trial"],
                     engine=getattr(gs, "engine", "window"))


def sha(words):
    return hashlib.sha256(np.ascontiguousarray(words, dtype="<u8").tobytes()).hexdigest()


def masked(deg, ids):
    m = np.arange(ids.shape[1])[None, :] < deg[:, None]
    return np.where(m, ids, 0).astype(np.uint32)


def load_case(name):
    with open(os.path.join(GOLDEN, f"{name}.json")) as f:
        doc = json.load(f)
    z = np.load(os.path.join(GOLDEN, f"{name}_peers.npz"))
    return doc, z["deg"], z["ids"]


@pytest.mark.parametrize("name", CASES)
def test_golden_broadcast_per_tick(gs, name):
    doc, deg, ids = load_case(name)
    with gs.Simulator(cfg_from(gs, doc["params"])) as sim:
        sim.load_peers(deg, ids)
        sim.broadcast_begin(-1)
        for i, tk in enumerate(doc["ticks"]):
            s = sim.step(1)[0]
            assert [int(x) for x in s] == tk["stats"], f"tick {i + 1} stats differ"
            assert sha(sim.received()) == tk["received_sha256"], f"tick {i + 1} received set differs"
        assert sha(sim.crashed()) == doc["crashed_sha256_final"]


@pytest.mark.parametrize("name", CASES)
def test_golden_overlay(gs, name):
    doc, deg, ids = load_case(name)
    with gs.Simulator(cfg_from(gs, doc["params"])) as sim:
        wins, final = sim.build_overlay()
        assert final == doc["overlay_final_tick"]
        assert [list(w) for w in wins] == doc["overlay_windows"]
        gdeg, gids = sim.read_peers()
        assert np.array_equal(gdeg, deg)
        assert np.array_equal(masked(gdeg, gids)[:, :ids.shape[1]], ids)


def random_table(n, stride, deg_lo, deg_hi, seed):
    rng = np.random.default_rng(seed)
    deg = rng.integers(deg_lo, deg_hi + 1, size=n).astype(np.uint8)
    ids = rng.integers(0, n, size=(n, stride)).astype(np.uint32)
    return deg, ids


def run_both(gs, oracle, kw, deg, ids, sender=-1, ticks=400, failed=None, chunk=1):
    p = oracle.make_params(**kw)
    e = oracle.Engine(p, deg, ids)
    if failed is not None:
        e.set_failed(failed)
    e.begin(sender)
    with gs.Simulator(cfg_from(gs, kw)) as sim:
        sim.load_peers(deg, ids)
        if failed is not None:
            sim.set_failed(failed)
        sim.broadcast_begin(sender)
        done = 0
        while done < ticks:
            a = e.step(chunk)
            b = sim.step(chunk)
            assert np.array_equal(a, b), f"stats differ after tick {done + chunk}:\n{a}\n{b}"
            assert np.array_equal(e.received(), sim.received()), f"received differs at {done + chunk}"
            done += chunk
            if int(a[-1][6]) == 0:
                break
        assert np.array_equal(e.crashed(), sim.crashed())
        return a[-1]


BASE = dict(fanout=5, fanin=6, delay_low=10, delay_high=20, drop_rate=0.1, crash_rate=0.001,
            seed=11, trial=0)


@pytest.mark.parametrize("kw,stride,dlo,dhi", [
    (dict(BASE, n=1), 2, 1, 2),                                   # self-friend
    (dict(BASE, n=2, crash_rate=0.3), 3, 0, 3),                   # tiny, zero-degree nodes
    (dict(BASE, n=777, delay_low=1, delay_high=2), 6, 0, 6),      # hop mode, ragged words
    (dict(BASE, n=5000, fanout=18, fanin=19), 19, 18, 19),        # C4-like wide rows
    (dict(BASE, n=9000, drop_rate=0.0, crash_rate=0.0), 6, 5, 6), # flood, no loss
    (dict(BASE, n=9000, drop_rate=0.29, crash_rate=0.57), 6, 5, 6),  # heavy crash (kc=56)
    (dict(BASE, n=4097, delay_low=0, delay_high=3), 4, 1, 4),     # 0-ms delays clamp to 1 tick
    (dict(BASE, n=20000, drop_rate=1.0), 6, 5, 6),                # every send dropped
    (dict(BASE, n=12345, delay_low=3, delay_high=40, trial=9), 8, 2, 8),  # long ring
])
def test_random_tables_bit_exact(gs, oracle, kw, stride, dlo, dhi):
    deg, ids = random_table(kw["n"], stride, dlo, dhi, seed=kw["n"])
    run_both(gs, oracle, kw, deg, ids)


def test_skewed_targets_force_exact_partition(gs, oracle):
    """Every friend of every node lies in [0, 16384): the window engine's
    estimated coarse/fine regions overflow and the window is redone with exact
    counts; the one hot bucket also takes k_resolve's global-streaming path."""
    n = 5_000_000
    rng = np.random.default_rng(7)
    deg = np.full(n, 6, np.uint8)
    ids = rng.integers(0, 16384, size=(n, 6)).astype(np.uint32)
    kw = dict(BASE, n=n, delay_low=1, delay_high=2, drop_rate=0.0, crash_rate=0.02)
    run_both(gs, oracle, kw, deg, ids, sender=10, ticks=8)


def test_sender_argument_and_multi_tick_steps(gs, oracle):
    kw = dict(BASE, n=3000, crash_rate=0.02)
    deg, ids = random_table(3000, 6, 5, 6, seed=5)
    run_both(gs, oracle, kw, deg, ids, sender=1234, chunk=7)


def test_failed_mask_flood_and_crash(gs, oracle):
    n = 6000
    rng = np.random.default_rng(2)
    bits = rng.random(n) < 0.05
    words = np.zeros((n + 63) // 64, dtype=np.uint64)
    for v in np.nonzero(bits)[0]:
        words[v >> 6] |= np.uint64(1) << np.uint64(v & 63)
    deg, ids = random_table(n, 6, 5, 6, seed=3)
    run_both(gs, oracle, dict(BASE, n=n, crash_rate=0.0), deg, ids, failed=words)
    run_both(gs, oracle, dict(BASE, n=n, crash_rate=0.03), deg, ids, failed=words)


def test_ring_graph_bfs_layers(gs):
    """drop 0, crash 0, constant delay d: hop h reaches exactly ring distance h."""
    n, d = 1001, 3
    deg = np.full(n, 2, np.uint8)
    ids = np.stack([(np.arange(n) - 1) % n, (np.arange(n) + 1) % n], 1).astype(np.uint32)
    kw = dict(BASE, n=n, delay_low=d, delay_high=d + 1, drop_rate=0.0, crash_rate=0.0)
    with gs.Simulator(cfg_from(gs, kw)) as sim:
        sim.load_peers(deg, ids)
        s0 = 17
        sim.broadcast_begin(s0)
        for h in range(1, 30):
            sim.step(d)
            recv = np.unpackbits(sim.received().view(np.uint8), bitorder="little")[:n]
            dist = np.minimum((np.arange(n) - s0) % n, (s0 - np.arange(n)) % n)
            # the sender itself is received only via the echo at hop 2
            want = (dist <= h) & (dist >= 1) | ((dist == 0) & (h >= 2))
            assert np.array_equal(recv.astype(bool), want), f"hop {h}"


def test_overlay_c2_size_matches_oracle(gs, oracle):
    """Config C2 shape (fanout 3, fanin 6) at n=2e5: GPU overlay == oracle overlay."""
    kw = dict(n=200000, fanout=3, fanin=6, delay_low=10, delay_high=20, drop_rate=0.1,
              crash_rate=0.001, seed=1, trial=0)
    deg, ids, wins, final = oracle.overlay(oracle.make_params(**kw))
    with gs.Simulator(cfg_from(gs, kw)) as sim:
        gw, gf = sim.build_overlay()
        assert gf == final
        assert [tuple(w) for w in gw] == [tuple(w) for w in wins]
        gdeg, gids = sim.read_peers()
        assert np.array_equal(gdeg, deg)
        assert np.array_equal(masked(gdeg, gids), masked(deg, ids))
        # invariant simulator.go:68,80,96: fanout <= len(friends) <= fanin
        assert gdeg.min() >= 3 and gdeg.max() <= 6


@pytest.mark.parametrize("block,dlow,dhigh", [("1", 10, 20), ("2", 10, 20), ("5", 10, 20), ("10", 10, 20),
                                             (None, 10, 20), ("10", 5, 9), ("10", 2, 7), ("10", 1, 4)])
def test_overlay_tick_blocks_match_oracle(gs, oracle, monkeypatch, block, dlow, dhigh):
    """The overlay can process blocks of L ticks at once (L | 10, L <=
    delaylow; GS_OV_BLOCK caps L, default 1): every block length gives the
    oracle's per-tick overlay -- windows, final tick, rows."""
    if block is None:
        monkeypatch.delenv("GS_OV_BLOCK", raising=False)
    else:
        monkeypatch.setenv("GS_OV_BLOCK", block)
    kw = dict(n=50000, fanout=3, fanin=6, delay_low=dlow, delay_high=dhigh, drop_rate=0.1,
              crash_rate=0.001, seed=7, trial=0)
    deg, ids, wins, final = oracle.overlay(oracle.make_params(**kw))
    with gs.Simulator(cfg_from(gs, kw)) as sim:
        gw, gf = sim.build_overlay()
        assert gf == final
        assert [tuple(w) for w in gw] == [tuple(w) for w in wins]
        gdeg, gids = sim.read_peers()
        assert np.array_equal(gdeg, deg)
        assert np.array_equal(masked(gdeg, gids), masked(deg, ids))


@pytest.mark.parametrize("n,trials", [(6_000_000, 1), (60_000, 120)])
def test_overlay_partition_equals_sort_at_scale(gs, monkeypatch, n, trials):
    """Past the oracle's reach: at n = 6e6 (367 fine regions, 2 coarse
    regions, C5's fanout 5 / fanin 6) and at 120 batched trials (the opt-in
    batched plans), the overlay built with the destination partition is the
    one built with the radix sort -- table, degrees, windows, final tick --
    and every tick is grouped (no fallback)."""
    from dataclasses import replace
    if gs.engine == "tick":
        pytest.skip("one engine is enough: the overlay is the same code")
    kw = dict(n=n, fanout=5, fanin=6, delay_low=10, delay_high=20, drop_rate=0.1, crash_rate=0.01,
              seed=17, trial=2)
    out = {}
    for mode in ("sort", "partition"):
        for var in ("GS_OV_SORT", "GS_OV_PART_BATCHED"):
            monkeypatch.delenv(var, raising=False)
        if mode == "sort":
            monkeypatch.setenv("GS_OV_SORT", "1")
        elif trials > 1:
            monkeypatch.setenv("GS_OV_PART_BATCHED", "1")
        with gs.Simulator(replace(cfg_from(gs, kw), trials=trials)) as sim:
            wins, final = sim.build_overlay()
            tm = sim.timing()
            deg, ids = sim.read_peers()
        out[mode] = (hashlib.sha256(deg.tobytes()).hexdigest(), hashlib.sha256(masked(deg, ids).tobytes()).hexdigest(),
                     [tuple(w) for w in wins], final)
        if mode == "partition":
            assert tm["ov_part_ticks"] >= 10 and tm["ov_part_fallbacks"] == 0, tm
    assert out["sort"] == out["partition"]


@pytest.mark.parametrize("mode", ["partition", "sort", "fallback", "batched", "pick-count", "pick-overflow",
                                  "staged-rows", "unstaged"])
def test_overlay_destination_partition(gs, oracle, monkeypatch, mode):
    """Verdict r04 item 6: dense overlay ticks are grouped by destination with
    the hand-written partition (k_ov_part x2 + k_ov_fine) instead of the
    radix sort.  partition: the default (dense ticks partitioned, sparse ticks
    sorted); sort: GS_OV_SORT=1, every tick sorted; fallback: plans at half
    the expected counts, so every dense tick's regions overflow and the tick
    is sorted from its intact bucket; batched: 12 trials in one id space
    (plans from each trial's own count of the tick's events);
    pick-count / pick-overflow: tick 0's picks counted before they are written
    (instead of one pass into planned buckets), or the plan too small so the
    planned pass overflows and falls back to that; staged-rows / unstaged:
    k_process with a thread's rows loaded together (GS_OV_STAGED=1) / with
    every key read from global memory (GS_OV_STAGED=0).
    Every mode builds the oracle's overlay -- windows, final tick, rows -- and
    a window context's rows come out sealed (slots past the degree empty)."""
    from dataclasses import replace
    if mode == "batched" and gs.engine == "tick":
        pytest.skip("batched trials run on the window engine")
    for var in ("GS_OV_SORT", "GS_OV_PART_SCALE", "GS_OV_PICK_COUNT", "GS_OV_PICK_SCALE", "GS_OV_PART_BATCHED",
                "GS_OV_STAGED"):
        monkeypatch.delenv(var, raising=False)
    if mode in ("staged-rows", "unstaged"):
        monkeypatch.setenv("GS_OV_STAGED", "1" if mode == "staged-rows" else "0")
    if mode == "pick-count":  # tick 0 counted, then written (the planned single pass off)
        monkeypatch.setenv("GS_OV_PICK_COUNT", "1")
    if mode == "pick-overflow":  # tick 0's planned buckets too small: the count-and-write fallback
        monkeypatch.setenv("GS_OV_PICK_SCALE", "0.5")
    if mode == "batched":  # (batched builds sort by default: not faster for C3, see gs_overlay.hip)
        monkeypatch.setenv("GS_OV_PART_BATCHED", "1")
    if mode == "sort":
        monkeypatch.setenv("GS_OV_SORT", "1")
    if mode == "fallback":
        monkeypatch.setenv("GS_OV_PART_SCALE", "0.5")
    kw = dict(n=150000 if mode != "batched" else 20000, fanout=5, fanin=6, delay_low=10, delay_high=20,
              drop_rate=0.1, crash_rate=0.01, seed=5, trial=3)
    trials = 12 if mode == "batched" else 1
    with gs.Simulator(replace(cfg_from(gs, kw), trials=trials)) as sim:
        gw, gf = sim.build_overlay()
        tm = sim.timing()
        gdeg, gids = sim.read_peers()
        n = kw["n"]
        res = [(gdeg[t * n:(t + 1) * n], gids[t * n:(t + 1) * n]) for t in range(trials)]
    if gs.engine != "tick":  # sealed: every slot past a node's degree holds the empty id
        pad = np.arange(gids.shape[1])[None, :] >= gdeg.astype(np.int64)[:, None]
        assert np.all(gids[pad] == 0xFFFFFFFF)
    if mode in ("partition", "pick-count", "pick-overflow", "batched", "staged-rows", "unstaged"):
        assert tm["ov_part_ticks"] >= 10 and tm["ov_part_fallbacks"] == 0, tm
    elif mode == "sort":
        assert tm["ov_part_ticks"] == 0 and tm["ov_sort_ticks"] > 0, tm
    else:
        assert tm["ov_part_ticks"] == 0 and tm["ov_part_fallbacks"] >= 10, tm
    for t, (gdeg, gids) in enumerate(res):
        deg, ids, wins, final = oracle.overlay(oracle.make_params(**dict(kw, trial=kw["trial"] + t)))
        if trials == 1:
            assert gf == final
            assert [tuple(w) for w in gw] == [tuple(w) for w in wins]
        assert np.array_equal(gdeg, deg), f"trial {t}"
        assert np.array_equal(masked(gdeg, gids)[:, :ids.shape[1]], masked(deg, ids)), f"trial {t}"


def test_overlay_longest_ring_and_its_limit(gs, oracle):
    """the overlay's ring of blocks holds ceil(R / L) + 2 buckets,
    and its LDS histograms kMaxRing = 1026 of them.  delayhigh = 1024 (the
    longest ring, 1026 buckets) must build the oracle's overlay; 1025 must be
    refused (GS_EINVAL) instead of overrunning the histograms."""
    from gossip_simulator_amd import _lib
    kw = dict(n=3000, fanout=3, fanin=6, delay_low=10, delay_high=1024, drop_rate=0.1,
              crash_rate=0.001, seed=11, trial=0)
    deg, ids, wins, final = oracle.overlay(oracle.make_params(**kw))
    with gs.Simulator(cfg_from(gs, kw)) as sim:
        gw, gf = sim.build_overlay()
        assert gf == final
        assert [tuple(w) for w in gw] == [tuple(w) for w in wins]
        gdeg, gids = sim.read_peers()
        assert np.array_equal(gdeg, deg)
        assert np.array_equal(masked(gdeg, gids), masked(deg, ids))
    kw["delay_high"] = 1025
    with gs.Simulator(cfg_from(gs, kw)) as sim:
        with pytest.raises(_lib.GossipError) as e:
            sim.build_overlay()
        assert e.value.code == _lib.GS_EINVAL and "ring limit" in str(e.value)


@pytest.mark.parametrize("mode", ["tick", "hop"])
def test_c2_full_size_bit_exact(gs, oracle, mode):
    """Config C2: N=1e6, fanout 3 (fanin 6); GPU overlay + broadcast vs oracle, per poll."""
    kw = dict(n=1_000_000, fanout=3, fanin=6, delay_low=10, delay_high=20 if mode == "tick" else 11,
              drop_rate=0.1, crash_rate=0.001, seed=1, trial=0)
    p = oracle.make_params(**kw)
    deg, ids, _, _ = oracle.overlay(p)
    e = oracle.Engine(p, deg, ids)
    e.begin(-1)
    with gs.Simulator(cfg_from(gs, kw)) as sim:
        sim.build_overlay()
        gdeg, gids = sim.read_peers()
        assert np.array_equal(gdeg, deg) and np.array_equal(masked(gdeg, gids), masked(deg, ids))
        sim.broadcast_begin(-1)
        while True:
            a = e.step(10)
            b = sim.step(10)
            assert np.array_equal(a, b)
            if gs.covered(int(a[-1][4]), p.n) or int(a[-1][6]) == 0:
                break
        assert np.array_equal(e.received(), sim.received())
        assert np.array_equal(e.crashed(), sim.crashed())


def test_run_polls_like_reference(gs, oracle):
    kw = dict(BASE, n=50000, seed=1)
    p = oracle.make_params(**kw)
    deg, ids, _, _ = oracle.overlay(p)
    rows, _ = oracle.run_to_coverage(p, deg, ids)
    with gs.Simulator(cfg_from(gs, kw)) as sim:
        sim.load_peers(deg, ids)
        sim.broadcast_begin(-1)
        polls, status = sim.run(poll=10)
        assert status == 0  # GS_RUN_COVERED
        assert int(polls[-1][0]) == int(rows[-1][0])
        assert int(polls[-1][4]) == int(rows[-1][4])
        assert int(polls[:, 3].sum()) == int(rows[:, 3].sum())
