"""Push-pull extension (config C5): no reference semantics exist
(simulator.go only floods, :140-149), so the CPU restatement in
oracle/gsoracle.c (pushpull_step) is pinned here by a second, independent
pure-Python restatement and by hand-derived answers, and the HIP rounds
(gs_pushpull.hip) must match it bit-exactly per round.
"""
from __future__ import annotations

import numpy as np
import pytest

from test_gpu_parity import masked, random_table, sha

PP = dict(fanout=5, fanin=6, delay_low=10, delay_high=20, drop_rate=0.1, crash_rate=0.0,
          seed=0x5EED, trial=0, model=1)


def py_pushpull(oracle, p, deg, ids, sender, rounds, failed=None):
    """Independent restatement: one synchronous round per tick, all draws keyed
    Philox{v, t, 0, kind 9 << 24 | trial}."""
    n = int(p.n)
    key = [int(p.seed) & 0xFFFFFFFF, int(p.seed) >> 32]
    kd = oracle.threshold(p.drop_rate)
    dead = np.zeros(n, bool) if failed is None else failed
    inf = np.zeros(n, bool)
    recv = 0
    if not dead[sender]:
        inf[sender] = True
        recv = 1
    out = []
    for t in range(1, rounds + 1):
        nxt = inf.copy()
        fired = sent = msgs = 0
        for v in range(n):
            d = int(deg[v])
            if dead[v] or d == 0:
                continue
            r = oracle.philox([v, t, 0, (9 << 24) | int(p.trial)], key)
            u = int(ids[v, (r[0] * d) >> 32])
            kept = ((r[1] * 100) >> 32) >= kd
            fired += 1
            if inf[v]:
                if kept:
                    sent += 1
                    if not dead[u]:
                        msgs += 1
                        nxt[u] = True
            elif inf[u] and kept:
                sent += 1
                msgs += 1
                nxt[v] = True
        recv += int((nxt & ~inf).sum())
        inf = nxt
        out.append([t, fired, sent, msgs, recv, 0, recv])
    return np.array(out, dtype=np.uint64), inf


def words_of(bits):
    n = bits.size
    w = np.zeros((n + 63) // 64, dtype=np.uint64)
    idx = np.nonzero(bits)[0]
    np.bitwise_or.at(w, idx // 64, np.left_shift(np.uint64(1), (idx % 64).astype(np.uint64)))
    return w


@pytest.mark.parametrize("n,drop,fail_frac", [(1, 0.1, 0.0), (2, 0.0, 0.0), (300, 0.1, 0.0),
                                              (257, 0.3, 0.05), (500, 1.0, 0.0)])
def test_oracle_matches_python_restatement(oracle, n, drop, fail_frac):
    deg, ids = random_table(n, 6, 0 if n > 2 else 1, 6, seed=n + 1)
    p = oracle.make_params(**dict(PP, n=n, drop_rate=drop))
    rng = np.random.default_rng(n)
    dead = rng.random(n) < fail_frac
    sender = int(oracle.pick_sender(p))
    rounds = 25
    ref, inf = py_pushpull(oracle, p, deg, masked(deg, ids), sender, rounds, dead)
    e = oracle.Engine(p, deg, ids)
    if fail_frac:
        e.set_failed(words_of(dead))
    e.begin(-1)
    got = e.step(rounds)
    assert np.array_equal(got, ref)
    assert np.array_equal(e.received(), words_of(inf))


def test_oracle_known_answers(oracle):
    n = 4000
    deg, ids = random_table(n, 6, 5, 6, seed=3)
    # every call lost: only the sender is ever informed, nothing is sent
    e = oracle.Engine(oracle.make_params(**dict(PP, n=n, drop_rate=1.0)), deg, ids)
    e.begin(7)
    s = e.step(10)
    assert (s[:, 4] == 1).all() and (s[:, 2] == 0).all() and (s[:, 1] == n).all()
    # a failed sender informs nobody, and a failed node is never informed
    failed = np.zeros(n, bool)
    failed[[7, 100, 2000]] = True
    e = oracle.Engine(oracle.make_params(**dict(PP, n=n)), deg, ids)
    e.set_failed(words_of(failed))
    e.begin(7)
    assert (e.step(5)[:, 4] == 0).all()
    e = oracle.Engine(oracle.make_params(**dict(PP, n=n, drop_rate=0.0)), deg, ids)
    e.set_failed(words_of(failed))
    e.begin(8)
    s = e.step(40)
    rec = e.received()
    for v in (7, 100, 2000):
        assert not (int(rec[v // 64]) >> (v % 64)) & 1
    assert (np.diff(s[:, 4].astype(np.int64)) >= 0).all() and (s[:, 6] == s[:, 4]).all()
    assert int(s[-1, 4]) == n - 3  # a connected table: everyone live is reached
    # complete graph, no loss: round 1 informs the sender's pick and every
    # node that picked the sender
    n = 64
    deg = np.full(n, n - 1, np.uint8)
    ids = np.array([[u for u in range(n) if u != v] for v in range(n)], np.uint32)
    p = oracle.make_params(**dict(PP, n=n, fanout=n - 1, fanin=n - 1, drop_rate=0.0))
    e = oracle.Engine(p, deg, ids)
    e.begin(0)
    s = e.step(1)[0]
    key = [int(p.seed) & 0xFFFFFFFF, int(p.seed) >> 32]
    picks = [int(ids[v, (oracle.philox([v, 1, 0, 9 << 24], key)[0] * (n - 1)) >> 32]) for v in range(n)]
    expect = {0, picks[0]} | {v for v in range(n) if picks[v] == 0}
    assert int(s[4]) == len(expect)
    assert int(s[2]) == 1 + sum(1 for v in range(1, n) if picks[v] == 0)


@pytest.mark.gpu
@pytest.mark.parametrize("rounds", ["auto", "early", "dense", "topdown", "bottom", "answer"])
@pytest.mark.parametrize("kw,stride,dlo,dhi,fail_frac", [
    (dict(PP, n=1), 2, 1, 2, 0.0),
    (dict(PP, n=2, drop_rate=0.0), 3, 0, 3, 0.0),
    (dict(PP, n=777), 6, 0, 6, 0.0),                        # ragged words, zero degrees
    (dict(PP, n=20000), 6, 5, 6, 0.01),                     # C5 shape, 1 % failed
    (dict(PP, n=20000, drop_rate=1.0), 6, 5, 6, 0.0),       # every call lost
    (dict(PP, n=9000, drop_rate=0.05), 16, 1, 16, 0.0),     # widest packed slot bytes (j, deg <= 16)
    (dict(PP, n=65536 + 77, drop_rate=0.29, trial=5), 19, 18, 19, 0.03),  # wide rows
])
def test_gpu_pushpull_bit_exact(oracle, kw, stride, dlo, dhi, fail_frac, rounds, l2_only=False):
    """Per round bit-exact to the oracle: with the default round selection,
    with sparse early rounds forced for the whole run (informed list +
    reverse table), with dense rounds only (no reverse table, and the
    failed-word gather instead of the failed-slot mask), and with the dense
    rounds forced top-down (atomic pushes) or bottom-up (in-edge scans)."""
    import gossip_simulator_amd as gs
    gs.load()
    n = kw["n"]
    deg, ids = random_table(n, stride, dlo, dhi, seed=n)
    p = oracle.make_params(**kw)
    e = oracle.Engine(p, deg, ids)
    failed = words_of(np.random.default_rng(1).random(n) < fail_frac) if fail_frac else None
    if failed is not None:
        e.set_failed(failed)
    e.begin(-1)
    cfg = gs.Config(n=n, fanout=kw["fanout"], fanin=kw["fanin"], delaylow=kw["delay_low"],
                    delayhigh=kw["delay_high"], droprate=kw["drop_rate"], crashrate=kw["crash_rate"],
                    seed=kw["seed"], trial=kw["trial"], model="pushpull", pp_l2_only=l2_only,
                    timing=l2_only, pp_rounds=rounds)
    with gs.Simulator(cfg) as sim:
        sim.load_peers(deg, ids)
        if failed is not None:
            sim.set_failed(failed)
        sim.broadcast_begin(-1)
        # the sparse rounds' reverse table is built at begin unless dense-only
        assert (sim.timing()["prep_ms"] > 0) == (rounds != "dense")
        for r in range(60):
            a, b = e.step(1), sim.step(1)
            assert np.array_equal(a, b), f"round {r + 1}:\n{a}\n{b}"
            assert sha(e.received()) == sha(sim.received()), f"informed set differs at round {r + 1}"
            if oracle.covered(int(a[0, 4]), n) or int(a[0, 4]) == 0:
                break
        tm = sim.timing()
        # bottom-up needs packed slot bytes (stride <= 16) and, with failed
        # nodes, the failed-slot mask (stride <= 8)
        can_bottom = stride <= 16 and (fail_frac == 0 or stride <= 8)
        if rounds in ("dense", "topdown") or not can_bottom:
            assert tm["pp_bottom_rounds"] == 0 and tm["pp_answer_rounds"] == 0
        elif rounds == "bottom":
            assert tm["pp_bottom_rounds"] == r + 1 - tm["pp_early_rounds"]
        elif rounds == "answer":
            assert tm["pp_answer_rounds"] + tm["pp_bottom_rounds"] == r + 1 - tm["pp_early_rounds"]
        if rounds == "early":
            assert tm["pp_early_rounds"] >= 1
        if rounds != "dense" and n > 100:
            # the reverse table came from the edge partition (k_rv_*), not the atomic fill
            assert tm["pp_rev_part"] >= 1


@pytest.mark.gpu
@pytest.mark.parametrize("rounds", ["answer", "bottom"])
def test_gpu_pushpull_hub_past_the_compact_view(oracle, rounds):
    """A hub: every node's slot 0 names node 1, so node 1 has ~70,000
    in-edges and its 64-node block passes the 65,535 the dense rounds'
    compact view of the in-edge ends holds (u16 per node, PPSparse::rend16):
    that context reads the 8-B ends instead (and a fine region of the
    partition build overflows, so the reverse table may come from the atomic
    fill).  Per round bit-exact to the oracle through pull-answer or
    bottom-up rounds."""
    import gossip_simulator_amd as gs
    gs.load()
    n = 70_000
    deg, ids = random_table(n, 6, 5, 6, seed=11)
    ids[:, 0] = 1
    ids[1, 0] = 2
    kw = dict(PP, n=n)
    e = oracle.Engine(oracle.make_params(**kw), deg, ids)
    e.begin(-1)
    cfg = gs.Config(n=n, fanout=kw["fanout"], fanin=kw["fanin"], delaylow=kw["delay_low"],
                    delayhigh=kw["delay_high"], droprate=kw["drop_rate"], crashrate=kw["crash_rate"],
                    seed=kw["seed"], trial=kw["trial"], model="pushpull", pp_rounds=rounds)
    with gs.Simulator(cfg) as sim:
        sim.load_peers(deg, ids)
        sim.broadcast_begin(-1)
        for r in range(60):
            a, b = e.step(1), sim.step(1)
            assert np.array_equal(a, b), f"round {r + 1}:\n{a}\n{b}"
            assert sha(e.received()) == sha(sim.received()), f"informed set differs at round {r + 1}"
            if oracle.covered(int(a[0, 4]), n) or int(a[0, 4]) == 0:
                break
        tm = sim.timing()
        assert tm["pp_answer_rounds"] + tm["pp_bottom_rounds"] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("rounds", ["answer", "bottom", "auto"])
def test_gpu_pushpull_new_mask_and_table_on_one_context(oracle, rounds):
    """the per-(table, failure mask) caches (live-caller counts,
    the has-failed-friend bits, the failed-caller bit per in-edge) must follow
    a new mask and a new table on the SAME context: three broadcasts -- mask A,
    then mask B, then a new table with mask B -- each bit-exact per round.
    Both tables carry a hub (friend 0 of every node) whose in-list is longer
    than the per-caller scan bound, so the failed-caller bits of its in-edges
    come from the hub pass (a quadratic scan before)."""
    import gossip_simulator_amd as gs
    gs.load()
    kw = dict(PP, n=20000)
    n = kw["n"]
    rng = np.random.default_rng(9)
    tables = []
    for seed, hub in ((3, 0), (4, 5)):
        deg, ids = random_table(n, 6, 5, 6, seed=seed)
        ids = ids.copy()
        ids[np.arange(n) != hub, 0] = hub
        tables.append((deg, ids))
    masks = [words_of(rng.random(n) < 0.01), words_of(rng.random(n) < 0.03)]
    cfg = gs.Config(n=n, fanout=kw["fanout"], fanin=kw["fanin"], delaylow=kw["delay_low"],
                    delayhigh=kw["delay_high"], droprate=kw["drop_rate"], crashrate=kw["crash_rate"],
                    seed=kw["seed"], trial=kw["trial"], model="pushpull", pp_rounds=rounds)
    with gs.Simulator(cfg) as sim:
        for case, (ti, mi) in enumerate(((0, 0), (0, 1), (1, 1))):
            deg, ids = tables[ti]
            if case:
                sim.reset()
            if case == 0 or ti != 0:
                sim.load_peers(deg, ids)
            sim.set_failed(masks[mi])
            e = oracle.Engine(oracle.make_params(**kw), deg, ids)
            e.set_failed(masks[mi])
            e.begin(-1)
            sim.broadcast_begin(-1)
            for r in range(80):
                a, b = e.step(1), sim.step(1)
                assert np.array_equal(a, b), f"broadcast {case}, round {r + 1}:\n{a}\n{b}"
                if oracle.covered(int(a[0, 4]), n) or int(a[0, 4]) == 0:
                    break
            assert sha(e.received()) == sha(sim.received()), f"broadcast {case}"


@pytest.mark.gpu
def test_gpu_pushpull_reverse_table_builds_agree(monkeypatch):
    """The reverse table built by the edge partition in one pass, in three
    passes over the coarse bins (GS_PP_REV_PASSES: the bounded-temporaries
    build a context takes when the device allocator's largest block is small),
    and by the atomic count + fill (GS_PP_REV_ATOMIC, the fallback) drive the
    same rounds: every pull-answer and bottom-up round scans it, so per-round
    counters and the informed set must be identical, with and without a
    failure mask (whose failed-caller bits are built from it).  The dense
    rounds' compact view of the in-edge ends (rend16 / rbase, the default)
    must also equal reading the 8-B ends (GS_PP_REND16=0).  The switches are
    read per build (per broadcast for GS_PP_REND16).  N = 1e7 spans three
    2^22-node coarse bins."""
    import gossip_simulator_amd as gs
    gs.load()
    n = 10_000_000
    failed = words_of(np.random.default_rng(2).random(n) < 0.01)
    runs = {}
    for mode in ("one", "three", "atomic", "rend64"):
        for var in ("GS_PP_REV_PASSES", "GS_PP_REV_ATOMIC", "GS_PP_REND16"):
            monkeypatch.delenv(var, raising=False)
        if mode == "rend64":
            monkeypatch.setenv("GS_PP_REND16", "0")
        if mode == "three":
            monkeypatch.setenv("GS_PP_REV_PASSES", "3")
        if mode == "atomic":
            monkeypatch.setenv("GS_PP_REV_ATOMIC", "1")
        cfg = gs.Config(n=n, fanout=5, fanin=6, droprate=0.1, crashrate=0.0, seed=0x5EED, model="pushpull",
                        pp_rounds="auto")
        with gs.Simulator(cfg) as sim:
            sim.build_overlay()
            out = []
            for mask in (None, failed):
                sim.reset()
                if mask is not None:
                    sim.set_failed(mask)
                sim.broadcast_begin(-1)
                rows = sim.step(60)
                out.append((rows, sha(sim.received())))
                if mask is None:
                    tm = sim.timing()
                    assert tm["pp_rev_part"] == {"one": 1, "three": 3, "atomic": 0, "rend64": 1}[mode], \
                        tm["pp_rev_part"]
                    assert tm["pp_bottom_rounds"] > 0 and tm["pp_answer_rounds"] > 0
            runs[mode] = out
    for mode in ("three", "atomic", "rend64"):
        for (a, ha), (b, hb) in zip(runs["one"], runs[mode]):
            assert np.array_equal(a, b), f"{mode}: per-round counters differ"
            assert ha == hb, f"{mode}: informed sets differ"


@pytest.mark.gpu
def test_gpu_pushpull_bit_exact_l2_only(oracle):
    """The round kernel without its LDS summary level (the N > ~1.02e9 path),
    forced by GS_FLAG_PP_L2_ONLY: bit-exact to the oracle like the default path."""
    test_gpu_pushpull_bit_exact(oracle, dict(PP, n=65536 + 77, drop_rate=0.29, trial=5), 19, 18, 19, 0.03,
                                "dense", l2_only=True)
    test_gpu_pushpull_bit_exact(oracle, dict(PP, n=20000), 6, 5, 6, 0.0, "auto", l2_only=True)


@pytest.mark.gpu
def test_gpu_pushpull_c5_shape_1e6(oracle):
    """N = 1e6 over the GPU-built overlay (fanout 5, fanin 6), 0.5 % failed nodes:
    bit-exact to the oracle at every round until 99 % coverage."""
    import gossip_simulator_amd as gs
    gs.load()
    n = 1_000_000
    cfg = gs.Config(n=n, fanout=5, fanin=6, droprate=0.1, crashrate=0.0, seed=0x5EED,
                    model="pushpull")
    with gs.Simulator(cfg) as sim:
        sim.build_overlay()
        deg, ids = sim.read_peers()
        failed = words_of(np.random.default_rng(2).random(n) < 0.005)
        sim.set_failed(failed)
        p = oracle.make_params(n=n, drop_rate=0.1, crash_rate=0.0, model=1)
        e = oracle.Engine(p, deg, ids)
        e.set_failed(failed)
        e.begin(-1)
        sim.broadcast_begin(-1)
        for r in range(200):
            a, b = e.step(1), sim.step(1)
            assert np.array_equal(a, b), f"round {r + 1}"
            if oracle.covered(int(a[0, 4]), n):
                break
        assert oracle.covered(int(a[0, 4]), n)
        assert sha(e.received()) == sha(sim.received())


@pytest.mark.gpu
@pytest.mark.parametrize("rounds", ["auto", "early"])
@pytest.mark.parametrize("fail_frac", [0.0, 0.02])
def test_gpu_pushpull_run_polls_like_oracle(oracle, fail_frac, rounds):
    """gs_run: 10-round polls, stop at 99 % (float32 rule) or after a poll
    window that informed nobody new (2 % failed nodes cannot reach 99 %)."""
    import gossip_simulator_amd as gs
    gs.load()
    n = 30000
    deg, ids = random_table(n, 6, 5, 6, seed=4)
    kw = dict(PP, n=n)
    p = oracle.make_params(**kw)
    failed = words_of(np.random.default_rng(3).random(n) < fail_frac) if fail_frac else None
    rows, e = oracle.run_to_coverage(p, deg, ids, failed=failed)
    cfg = gs.Config(n=n, droprate=kw["drop_rate"], crashrate=0.0, seed=kw["seed"], model="pushpull",
                    pp_rounds=rounds)
    with gs.Simulator(cfg) as sim:
        sim.load_peers(deg, ids)
        if failed is not None:
            sim.set_failed(failed)
        sim.broadcast_begin(-1)
        polls, status = sim.run(poll=10)
        assert int(polls[-1][0]) == int(rows[-1][0])
        assert int(polls[-1][4]) == int(rows[-1][4])
        assert int(sim.totals()["messages"]) == int(rows[:, 3].sum())
        assert status == (gs.GS_RUN_COVERED if oracle.covered(int(rows[-1][4]), n) else gs.GS_RUN_QUIESCENT)
        assert sha(sim.received()) == sha(e.received())


# ---- node-range shards (SURVEY.md 8(e)2 for config C5) ------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("replica", [True, False])
@pytest.mark.parametrize("kw,stride,dlo,dhi,fail_frac,G", [
    (dict(PP, n=20000), 6, 5, 6, 0.01, 2),                                  # C5 shape, 1 % failed
    (dict(PP, n=65536 + 77, drop_rate=0.29, trial=5), 16, 1, 16, 0.0, 3),   # widest packed rows, 77-node shard
    (dict(PP, n=50000, drop_rate=0.05), 8, 0, 8, 0.02, 2),                  # zero degrees, 8-slot fmask
])
def test_gpu_pushpull_shards_bit_exact(oracle, monkeypatch, kw, stride, dlo, dhi, fail_frac, G, replica):
    """G node-range shards of one push-pull run on one GPU (gs_create_multi):
    the sparse early rounds on the device's replica (the full table, the
    replicated sets; replica=False: GS_PP_NO_REPLICA=1, none), then
    pull-answer rounds (each shard's informed nodes answer the pulls among
    their in-edges, into one shared set) and bottom-up rounds on each shard's
    own nodes against the replicated informed set, exchanged after the round;
    per round bit-exact to the oracle's pushpull_step (oracle/gsoracle.c), as
    the unsharded engine is."""
    import gossip_simulator_amd as gs
    gs.load()
    if not replica:
        monkeypatch.setenv("GS_PP_NO_REPLICA", "1")
    n = kw["n"]
    deg, ids = random_table(n, stride, dlo, dhi, seed=n)
    e = oracle.Engine(oracle.make_params(**kw), deg, ids)
    failed = words_of(np.random.default_rng(1).random(n) < fail_frac) if fail_frac else None
    if failed is not None:
        e.set_failed(failed)
    e.begin(-1)
    cfg = gs.Config(n=n, fanout=kw["fanout"], fanin=kw["fanin"], delaylow=kw["delay_low"],
                    delayhigh=kw["delay_high"], droprate=kw["drop_rate"], crashrate=kw["crash_rate"],
                    seed=kw["seed"], trial=kw["trial"], model="pushpull")
    with gs.Simulator(cfg, devices=[0] * G) as sim:
        assert len(sim.shard_info()) == G
        sim.load_peers(deg, ids)
        if failed is not None:
            sim.set_failed(failed)
        sim.broadcast_begin(-1)
        for r in range(60):
            a, b = e.step(1), sim.step(1)
            assert np.array_equal(a, b), f"round {r + 1}:\n{a}\n{b}"
            assert sha(e.received()) == sha(sim.received()), f"informed set differs at round {r + 1}"
            if oracle.covered(int(a[0, 4]), n) or int(a[0, 4]) == 0:
                break
        tm = sim.timing()
        assert tm["pp_bottom_rounds"] + tm["pp_early_rounds"] + tm["pp_answer_rounds"] == r + 1
        assert (tm["pp_early_rounds"] >= 1) == replica


@pytest.fixture(scope="module")
def pp_1e6():
    """Push-pull at N = 1e6 over the GPU overlay, 1 % failed: the unsharded run."""
    import gossip_simulator_amd as gs
    gs.load()
    n = 1_000_000
    cfg = gs.Config(n=n, fanout=5, fanin=6, droprate=0.1, crashrate=0.0, seed=0x5EED, model="pushpull")
    failed = words_of(np.random.default_rng(7).random(n) < 0.01)
    with gs.Simulator(cfg) as sim:
        sim.build_overlay()
        deg, ids = sim.read_peers()
        sim.set_failed(failed)
        sim.broadcast_begin(-1)
        rows = sim.step(45)
        polls = None
        rec = sim.received()
        sim.reset()
        sim.broadcast_begin(-1)
        polls, status = sim.run(poll=5)
    return cfg, deg, ids, failed, rows, rec, polls, status


@pytest.mark.gpu
@pytest.mark.parametrize("G,answer", [(2, True), (4, True), (8, True), (4, False)])
def test_gpu_pushpull_shards_match_unsharded_1e6(pp_1e6, monkeypatch, G, answer):
    """N = 1e6 (C5 shape, 1 % failed) in G shards, per round and through
    gs_run's poll and stop rule: identical to the unsharded run (answer=False:
    GS_PP_SHARD_BOTTOM=1, bottom-up sharded rounds only)."""
    import gossip_simulator_amd as gs
    if not answer:
        monkeypatch.setenv("GS_PP_SHARD_BOTTOM", "1")
    cfg, deg, ids, failed, rows, rec, polls, status = pp_1e6
    with gs.Simulator(cfg, devices=[0] * G) as sim:
        sim.load_peers(deg, ids)
        sim.set_failed(failed)
        sim.broadcast_begin(-1)
        assert np.array_equal(sim.step(45), rows)
        assert sha(sim.received()) == sha(rec)
        sim.reset()
        sim.broadcast_begin(-1)
        p2, s2 = sim.run(poll=5)
        assert s2 == status and np.array_equal(p2, polls)
        assert (sim.timing()["pp_answer_rounds"] > 0) == answer
