"""BASELINE.json's full size (config C5: N = 1e9, fanout 5, fanin 6, drop 0.1,
crash 0.01) on one MI355X.  The CPU oracle cannot finish at this size, so the
checks are size-independent properties plus a cross-check between the two
independent HIP engines (window pipeline vs per-tick atomic engine), which
implement the same tick model with no shared kernel code:

* per-tick counters of the two engines are identical, and so are the final
  received / crashed bitsets (SHA-256);
* counter identities: received == popcount(received bitset), crashed ==
  popcount(crashed bitset), messages <= delivered sends, every fired
  broadcast is a scheduled one (pending never negative, 0 at quiescence);
* the overlay respects fanout <= len(friends) <= fanin (simulator.go:68,80,96).
Node-range shards at full size (G in-process shards on the one GPU: the
owner-expand flood with its all-to-all of messages, the push-pull replica +
sharded bottom-up rounds) against the unsharded run, per tick and on the
final bitsets.
Push-pull at N = 1e9: monotone informed set, pending == received, float32
99 % reached, delivered <= calls; with a 1 % pre-failed mask the per-round
counters and final bitsets are identical across the round selections auto /
dense / topdown / bottom / answer (independent kernels: sparse informed-list
rounds, streamed top-down rounds with atomics, bottom-up in-edge scans,
pull-answer in-edge scans of the informed).  The flood
with the same 1 % mask: window engine vs tick engine, bit-exact per tick.
"""
from __future__ import annotations

import hashlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N = 1_000_000_000


def popcount(words: np.ndarray) -> int:
    return int(np.bitwise_count(words).sum())


def sha(words: np.ndarray) -> str:
    return hashlib.sha256(words.tobytes()).hexdigest()


def failed_mask(frac: float, seed: int) -> np.ndarray:
    """round(frac * N) node ids drawn uniformly (bench.py's failed_mask)."""
    rng = np.random.default_rng(seed)
    idx = rng.integers(0, N, size=int(round(frac * N)), dtype=np.int64)
    w = np.zeros((N + 63) // 64, dtype=np.uint64)
    np.bitwise_or.at(w, idx >> 6, np.left_shift(np.uint64(1), (idx & 63).astype(np.uint64)))
    return w


def flood(engine: str, mask=None, shards: int = 0):
    import gossip_simulator_amd as gs
    gs.load()
    cfg = gs.Config(n=N, fanout=5, fanin=6, droprate=0.1, crashrate=0.01, seed=0x5EED,
                    engine=engine)
    with gs.Simulator(cfg, devices=[0] * shards if shards else None) as sim:
        _, stab = sim.build_overlay()
        if mask is not None:
            sim.set_failed(mask)
        if engine == "window" and not shards:
            deg, _ = sim.read_peers()
            assert deg.min() >= 5 and deg.max() <= 6
            del deg
        sim.broadcast_begin(-1)
        rows = []
        while True:
            r = sim.step(10)
            rows.append(r)
            if gs.covered(int(r[-1][4]), N) or int(r[-1][6]) == 0:
                break
        rows = np.concatenate(rows)
        rec, cra = sim.received(), sim.crashed()
        return stab, rows, sha(rec), sha(cra), popcount(rec), popcount(cra), sim.totals()


def test_c5_window_vs_tick_engine_bit_exact():
    a = flood("window")
    b = flood("tick")
    assert a[0] == b[0]  # same overlay stabilisation tick
    assert np.array_equal(a[1], b[1]), "per-tick counters differ between the engines"
    assert a[2] == b[2] and a[3] == b[3], "final bitsets differ between the engines"
    stab, rows, _, _, nrec, ncra, tot = a
    assert nrec == int(rows[-1][4]) == tot["received"]
    assert ncra == int(rows[-1][5]) == tot["crashed"]
    assert (rows[:, 3] <= rows[:, 2]).all()              # counted <= delivered
    assert (rows[:, 6].astype(np.int64) >= 0).all()
    assert int(rows[:, 1].sum()) == int(tot["fired"]) and int(rows[:, 2].sum()) == int(tot["sent"])
    assert 0.98 < nrec / N < 0.995                       # ~1 % crash on the first receipt


def test_c5_pushpull_properties():
    import gossip_simulator_amd as gs
    gs.load()
    cfg = gs.Config(n=N, fanout=5, fanin=6, droprate=0.1, crashrate=0.0, seed=0x5EED,
                    model="pushpull")
    with gs.Simulator(cfg) as sim:
        sim.build_overlay()
        sim.broadcast_begin(-1)
        rows = sim.step(60)
        rec = np.asarray(rows[:, 4], dtype=np.int64)
        assert (np.diff(rec) >= 0).all() and (rows[:, 6] == rows[:, 4]).all()
        assert (rows[:, 3] <= rows[:, 2]).all() and (rows[:, 2] <= rows[:, 1]).all()
        assert gs.covered(int(rec[-1]), N)
        assert popcount(sim.received()) == int(rec[-1])


def test_c5_flood_failed_mask_window_vs_tick():
    """C5's flood with 1 % of the nodes pre-failed (gs_set_failed): the two
    engines agree per tick and on the final bitsets; failed nodes never count
    nor forward (the crashed bitset holds the mask)."""
    mask = failed_mask(0.01, 0x5EED + 1)
    a = flood("window", mask)
    b = flood("tick", mask)
    assert np.array_equal(a[1], b[1]), "per-tick counters differ between the engines"
    assert a[2] == b[2] and a[3] == b[3], "final bitsets differ between the engines"
    nfail = popcount(mask)
    assert a[5] >= nfail and 0.97 < a[4] / N < 0.99


def pushpull_failed(pp_rounds: str, mask, shards: int = 0):
    import gossip_simulator_amd as gs
    gs.load()
    cfg = gs.Config(n=N, fanout=5, fanin=6, droprate=0.1, crashrate=0.0, seed=0x5EED,
                    model="pushpull", pp_rounds=pp_rounds)
    with gs.Simulator(cfg, devices=[0] * shards if shards else None) as sim:
        sim.build_overlay()
        sim.set_failed(mask)
        sim.broadcast_begin(-1)
        rows = []
        while True:
            r = sim.step(5)
            rows.append(r)
            if gs.covered(int(r[-1][4]), N) or len(rows) > 20:
                break
        tm = sim.timing()
        rec = sim.received()
        return np.concatenate(rows), sha(rec), popcount(rec), tm


def test_c5_pushpull_failed_mask_round_modes_bit_exact():
    mask = failed_mask(0.01, 0x5EED + 1)
    ref = pushpull_failed("auto", mask)
    rows, h, nrec, tm = ref
    assert tm["pp_early_rounds"] > 0 and tm["pp_bottom_rounds"] > 0  # both special kernels ran
    assert gs_covered(int(rows[-1][4]))
    assert nrec == int(rows[-1][4])
    rec = np.asarray(rows[:, 4], dtype=np.int64)
    assert (np.diff(rec) >= 0).all() and (rows[:, 3] <= rows[:, 2]).all()
    for mode in ("dense", "topdown", "bottom", "answer"):
        got = pushpull_failed(mode, mask)
        assert np.array_equal(got[0], rows), f"pp_rounds={mode}: per-round counters differ"
        assert got[1] == h, f"pp_rounds={mode}: final informed set differs"
        if mode == "dense":
            assert got[3]["pp_early_rounds"] == 0 and got[3]["pp_bottom_rounds"] == 0


def gs_covered(recv: int) -> bool:
    return np.float32(recv) / np.float32(N) >= np.float32(0.99)


def test_c5_flood_shards_vs_unsharded_bit_exact():
    """C5's flood at N = 1e9 in 8 node-range shards (owner expand, messages to
    their targets' owners) and in 3 (ragged ranges, a partial coarse bin per
    shard) with the 1 % mask: identical to the unsharded window engine per tick
    and on the final bitsets."""
    mask = failed_mask(0.01, 0x5EED + 1)
    a = flood("window", mask)
    for G in (8, 3):
        b = flood("window", mask, shards=G)
        assert a[0] == b[0]
        assert np.array_equal(a[1], b[1]), f"G={G}: per-tick counters differ from the unsharded run"
        assert a[2] == b[2] and a[3] == b[3], f"G={G}: final bitsets differ from the unsharded run"


def test_c5_pushpull_shards_vs_unsharded_bit_exact():
    """C5 as named (push-pull, N = 1e9) with the 1 % mask in 8 node-range
    shards (the replica's sparse early rounds, then sharded bottom-up rounds):
    identical to the unsharded run per round and on the informed set."""
    mask = failed_mask(0.01, 0x5EED + 1)
    rows, h, nrec, _ = pushpull_failed("auto", mask)
    got = pushpull_failed("auto", mask, shards=8)
    assert np.array_equal(got[0], rows), "per-round counters differ from the unsharded run"
    assert got[1] == h and got[2] == nrec
    assert got[3]["pp_early_rounds"] > 0 and got[3]["pp_bottom_rounds"] > 0
