"""Pins for the CPU restatement (oracle/).  The reference ships no tests or
vectors and cannot run here (no Go toolchain), so the oracle is pinned by
hand-derived known answers and published Philox KATs, and by its own frozen
fixtures (tests/golden, regenerated only deliberately)."""
from __future__ import annotations

import hashlib
import json
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def sha(words):
    return hashlib.sha256(np.ascontiguousarray(words, dtype="<u8").tobytes()).hexdigest()


# ---- Philox4x32-10 -----------------------------------------------------------
RANDOM123_KAT = [  # Random123 kat_vectors, philox4x32 10 rounds
    ([0, 0, 0, 0], [0, 0], [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]),
    ([0xffffffff] * 4, [0xffffffff] * 2, [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]),
    ([0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344], [0xa4093822, 0x299f31d0],
     [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]),
]


@pytest.mark.parametrize("ctr,key,out", RANDOM123_KAT)
def test_philox_random123_kat(oracle, ctr, key, out):
    assert oracle.philox(ctr, key) == out


def test_philox_matches_rocrand_engine(oracle):
    with open(os.path.join(GOLDEN, "philox_kat.json")) as f:
        kat = json.load(f)
    assert len(kat) >= 150
    for v in kat:
        assert oracle.philox(v["ctr"], v["key"]) == v["out"]


# ---- Go quantisation and float32 rules --------------------------------------
@pytest.mark.parametrize("rate,k", [(0.001, 0), (0.1, 10), (0.29, 28), (0.57, 56), (0.58, 57),
                                    (0.01, 1), (1.0, 100), (0.0, 0), (-0.3, 0), (5.0, 100),
                                    (0.999, 99), (0.07, 7)])
def test_threshold_int_rate_times_100(oracle, rate, k):
    # simulator.go:172,180: int(rate*100), float64 product then truncation
    assert oracle.threshold(rate) == k
    assert int(rate * 100) == k or rate < 0 or rate > 1


@pytest.mark.parametrize("n,need", [(50000, 49500), (100000, 99000), (1000000, 990000),
                                    (100000000, 98999996), (1000000000, 989999968)])
def test_float32_99_percent_threshold(oracle, n, need):
    # simulator.go:246-248: float32(TotalReceived)/float32(N) >= 0.99
    assert oracle.covered(need, n)
    assert not oracle.covered(need - 1, n)


def test_uniform_map(oracle):
    assert oracle.lib().or_uniform(0, 100) == 0
    assert oracle.lib().or_uniform(0xFFFFFFFF, 100) == 99
    assert oracle.lib().or_uniform(0x80000000, 10) == 5


def test_drop_and_crash_are_the_first_two_base100_digits(oracle):
    """RandomDrop (simulator.go:172) and the message's crash roll (:180) come
    from one draw r: (drop, crash) = divmod(floor(10^4 r / 2^32), 100), so each
    of the 10^4 pairs is taken by 429496 or 429497 of the 2^32 words -- the two
    draws are independent uniforms to within 2.4e-6 relative."""
    import ctypes as C
    L = oracle.lib()
    rng = np.random.default_rng(11)
    rs = np.concatenate([rng.integers(0, 2**32, 20000, dtype=np.uint64),
                         np.array([0, 1, 42949672, 42949673, 2**31, 2**32 - 1], np.uint64)])
    d, c = C.c_uint32(), C.c_uint32()
    for r in rs.tolist():
        L.or_drop_crash(r, C.byref(d), C.byref(c))
        assert divmod((r * 10000) >> 32, 100) == (d.value, c.value)
    # exact pair counts over all 2^32 words
    m = np.arange(10000, dtype=np.uint64)
    first = (m * 2**32 + 9999) // 10000           # smallest r with floor(10^4 r / 2^32) >= m
    counts = np.diff(np.append(first, 2**32))
    assert counts.min() == 2**32 // 10000 and counts.max() == 2**32 // 10000 + 1
    # the law on Philox output: chi-square of the 10^4 pairs over 2e6 draws
    ws = np.array([oracle.philox([i, 7, 0, 3 << 24], [1, 2]) for i in range(500_000)], np.uint64).ravel()
    pair = (ws * 10000) >> np.uint64(32)
    obs = np.bincount(pair.astype(np.int64), minlength=10000)
    chi2 = float(((obs - len(ws) / 1e4) ** 2 / (len(ws) / 1e4)).sum())
    assert chi2 < 10000 + 6 * np.sqrt(2 * 10000)  # 9999 dof: mean 9999, sd 141


# ---- broadcast known answers -------------------------------------------------
def ring(n):
    deg = np.full(n, 2, np.uint8)
    ids = np.stack([(np.arange(n) - 1) % n, (np.arange(n) + 1) % n], 1).astype(np.uint32)
    return deg, ids


def bits(words, n):
    return np.unpackbits(words.view(np.uint8), bitorder="little")[:n].astype(bool)


def test_ring_bfs_layers(oracle):
    n, d, s0 = 257, 4, 100
    deg, ids = ring(n)
    p = oracle.make_params(n=n, delay_low=d, delay_high=d + 1, drop_rate=0, crash_rate=0)
    e = oracle.Engine(p, deg, ids)
    e.begin(s0)
    dist = np.minimum((np.arange(n) - s0) % n, (s0 - np.arange(n)) % n)
    for h in range(1, 20):
        st = e.step(d)
        want = ((dist >= 1) & (dist <= h)) | ((dist == 0) & (h >= 2))
        assert np.array_equal(bits(e.received(), n), want)
        # every tick between hops is silent
        assert st[:-1, 1].sum() == 0


def test_complete_graph_two_hops(oracle):
    n = 40
    deg = np.full(n, n - 1, np.uint8)
    ids = np.array([[u for u in range(n) if u != v] for v in range(n)], np.uint32)
    p = oracle.make_params(n=n, fanout=n - 1, fanin=n - 1, delay_low=5, delay_high=6,
                           drop_rate=0, crash_rate=0)
    e = oracle.Engine(p, deg, ids)
    e.begin(3)
    st = e.step(5)[-1]
    assert st[4] == n - 1 and st[3] == n - 1          # all but the sender after one hop
    st = e.step(5)[-1]
    assert st[4] == n                                  # the echo reaches the sender
    assert st[3] == (n - 1) * (n - 1)                  # everyone re-broadcast to n-1 friends


def test_drop_everything(oracle):
    deg, ids = ring(100)
    p = oracle.make_params(n=100, drop_rate=1.0, crash_rate=0)
    e = oracle.Engine(p, deg, ids)
    e.begin(0)
    st = e.step(40)
    assert st[:, 1].sum() == 1 and st[:, 2].sum() == 0 and st[-1, 4] == 0 and st[-1, 6] == 0


def test_sender_echo_broadcasts_twice(oracle):
    # two nodes, each the other's friend: s fires, t receives and fires, s is
    # received on the echo and fires again (simulator.go:117-122, :240-241)
    deg = np.array([1, 1], np.uint8)
    ids = np.array([[1], [0]], np.uint32)
    p = oracle.make_params(n=2, delay_low=2, delay_high=3, drop_rate=0, crash_rate=0)
    e = oracle.Engine(p, deg, ids)
    e.begin(0)
    st = e.step(10)
    assert st[:, 1].sum() == 3            # 0, then 1, then 0 again
    assert st[-1, 4] == 2 and st[:, 3].sum() == 3


def test_crash_on_first_receipt(oracle):
    # crashrate 1.0: every receipt crashes a live node; nobody is ever received
    deg, ids = ring(50)
    p = oracle.make_params(n=50, delay_low=1, delay_high=2, drop_rate=0, crash_rate=1.0)
    e = oracle.Engine(p, deg, ids)
    e.begin(7)
    st = e.step(5)
    assert st[-1, 4] == 0 and st[-1, 5] == 2 and st[:, 3].sum() == 2


def test_first_crash_restates_the_sequential_draws(oracle):
    """or_first_crash: draws U_(k-g+1)(lane (g-1)%4 of Philox{u, t, (g-1)/4,
    ORDER << 24 | trial}) < ones, g = 1, 2, ...; position 1 without a draw
    when k == 1 or every receipt carries a roll."""
    key = [0x1234, 0x5678]
    for (u, t, k, ones) in [(3, 17, 5, 2), (99, 4, 7, 1), (12, 250, 19, 5), (0, 1, 3, 2)]:
        g = 1
        while True:
            r = oracle.philox([u, t, (g - 1) // 4, (10 << 24) | 7], key)[(g - 1) % 4]
            if (r * (k - g + 1)) >> 32 < ones:
                break
            g += 1
        assert oracle.first_crash(key, 7, u, t, k, ones) == g
    assert oracle.first_crash(key, 7, 5, 5, 1, 1) == 1
    assert oracle.first_crash(key, 7, 5, 5, 6, 6) == 1


@pytest.mark.parametrize("k,ones", [(2, 1), (5, 2), (6, 3)])
def test_first_crash_law_is_a_uniform_order(oracle, k, ones):
    """The reference takes a tick's receipts in a random order and stops at the
    first crash: P(first crash at g) = C(k-g, ones-1) / C(k, ones).  The keyed
    draw has that law (chi-square over 40,000 (u, t) keys)."""
    from math import comb
    from scipy.stats import chisquare
    key = [0x5EED, 0]
    n = 40_000
    obs = np.zeros(k - ones + 1)
    for i in range(n):
        obs[oracle.first_crash(key, 0, i, 1 + i % 97, k, ones) - 1] += 1
    exp = np.array([comb(k - g, ones - 1) / comb(k, ones) for g in range(1, k - ones + 2)]) * n
    assert abs(exp.sum() - n) < 1e-6
    assert chisquare(obs, exp).pvalue > 0.001


def test_default_crashrate_quantises_to_zero(oracle):
    deg, ids, _, _ = oracle.overlay(oracle.make_params(n=3000))
    rows, e = oracle.run_to_coverage(oracle.make_params(n=3000), deg, ids)
    assert rows[-1, 5] == 0  # crashrate 0.001 -> int(0.1) = 0 (simulator.go:180)
    assert rows[:, 3].sum() == rows[:, 2].sum()  # no crash -> every delivered send counted


# ---- overlay -------------------------------------------------------------------
def test_overlay_invariants_and_symmetry(oracle):
    p = oracle.make_params(n=20000, fanout=5, fanin=6)
    deg, ids, wins, final = oracle.overlay(p)
    assert deg.min() >= 5 and deg.max() <= 6
    # edges form in pairs (simulator.go:69, 73-74): in-degree tracks out-degree
    indeg = np.bincount(np.concatenate([ids[v, :deg[v]] for v in range(p.n)]), minlength=p.n)
    assert abs(int(indeg.sum()) - int(deg.sum())) == 0
    assert np.mean(np.abs(indeg.astype(int) - deg.astype(int))) < 0.5
    assert final % 10 == 0 and final > 0
    assert sum(w[1] for w in wins) >= p.n * 5


def test_overlay_deterministic_and_trial_keyed(oracle):
    a = oracle.overlay(oracle.make_params(n=3000, trial=0))
    b = oracle.overlay(oracle.make_params(n=3000, trial=0))
    c = oracle.overlay(oracle.make_params(n=3000, trial=1))
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) and a[2] == b[2]
    assert not np.array_equal(a[1], c[1])


def test_overlay_livelock_detected(oracle):
    with pytest.raises(oracle.OverlayError):
        oracle.overlay(oracle.make_params(n=200, fanout=5, fanin=5), max_ticks=3000)


def test_overlay_no_friends(oracle):
    deg, ids, wins, final = oracle.overlay(oracle.make_params(n=10, fanout=0, fanin=6))
    assert final == 10 and wins == [] and deg.sum() == 0


def test_self_pick_maps_to_next(oracle):
    # n=1: every pick is the node itself, mapped to (id+1)%1 = 0 (simulator.go:98-100).
    # The run either stabilises or hits the reference's endless rejection loop
    # (simulator.go:87-89), which the oracle reports instead of hanging.
    try:
        deg, ids, _, _ = oracle.overlay(oracle.make_params(n=1, fanout=5, fanin=6))
        assert (ids[0, :deg[0]] == 0).all() and 5 <= deg[0] <= 6
    except oracle.OverlayError as e:
        assert "-3" in str(e)


# ---- frozen fixtures ---------------------------------------------------------
@pytest.mark.parametrize("name", ["a_n100_tick", "b_n1000_default", "c_n4133_hop",
                                  "d_n10000_crash"])
def test_oracle_reproduces_golden(oracle, name):
    with open(os.path.join(GOLDEN, f"{name}.json")) as f:
        doc = json.load(f)
    z = np.load(os.path.join(GOLDEN, f"{name}_peers.npz"))
    p = oracle.make_params(**doc["params"])
    deg, ids, wins, final = oracle.overlay(p)
    m = np.arange(ids.shape[1])[None, :] < deg[:, None]
    assert np.array_equal(deg, z["deg"])
    assert np.array_equal(np.where(m, ids, 0), z["ids"])
    assert [list(w) for w in wins] == doc["overlay_windows"] and final == doc["overlay_final_tick"]
    assert oracle.pick_sender(p) == doc["sender"]
    e = oracle.Engine(p, z["deg"], z["ids"])
    e.begin(-1)
    for tk in doc["ticks"]:
        s = e.step(1)[0]
        assert [int(x) for x in s] == tk["stats"]
        assert sha(e.received()) == tk["received_sha256"]
    assert sha(e.crashed()) == doc["crashed_sha256_final"]
