"""World-size-2 gloo tests of the multi-GPU logic on CPU.

* Trial sharding: dist.run_trials (the product's host code) over gloo, with the
  oracle behind the batch interface the HIP engine exposes -- must reproduce
  the serial trials.
* Node-range sharding: the library's window protocol (gs_api.cpp
  shard_windows: the same window cut on every shard from the gathered fire
  counts, every message of the window delivered to the shard that owns its
  target, per-poll sum of the counters) restated over oracle shards and gloo
  collectives -- must be bit-identical to the unsharded run.  The HIP path
  moves the messages themselves (owner expand + all-to-all); the restatement
  all-gathers the firing sets and lets each shard deliver to its own nodes,
  which is the same multiset of messages per shard.  The HIP path is checked
  on the GPU (tests/test_gpu_multi.py, and with two processes exchanging
  through gloo in tests/test_rank_exchange.py).
* Push-pull node-range sharding (config C5): the sharded rounds of
  gs_api.cpp pp_shard_step -- bottom-up on the shard's own nodes against the
  replicated informed set, then an all-gather of the owned words; and
  pull-answer, the shard's informed nodes informing nodes anywhere, whose
  bits go to their owners -- restated in numpy over gloo; each must equal the
  oracle's unsharded pushpull_step per round.
"""
from __future__ import annotations

import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class OracleBatch:
    """A batch of trials (oracle overlay + engine per trial) behind the
    interface dist.run_trials drives (the HIP engine's Simulator)."""

    def __init__(self, O, cfg):
        self.O, self.cfg = O, cfg
        self.trials = []

    def build_overlay(self):
        c = self.cfg
        for t in range(c.trials):
            p = self.O.make_params(n=c.n, fanout=c.fanout, fanin=c.fanin, delay_low=c.delaylow,
                                   delay_high=c.delayhigh, drop_rate=c.droprate,
                                   crash_rate=c.crashrate, seed=c.seed, trial=c.trial + t)
            deg, ids, _, _ = self.O.overlay(p)
            self.trials.append((p, deg, ids))

    def broadcast_begin(self, sender=-1):
        pass

    def run(self, poll=10, max_ticks=1_000_000):
        self.rows = []
        for p, deg, ids in self.trials:
            rows, _ = self.O.run_to_coverage(p, deg, ids, poll=poll, max_ticks=max_ticks)
            tick99 = next((int(r[0]) for r in rows if self.O.covered(int(r[4]), p.n)), 0)
            last = rows[-1]
            status = 0 if self.O.covered(int(last[4]), p.n) else 1 if int(last[6]) == 0 else 2
            self.rows.append([p.trial, tick99, int(last[0]), *[int(x) for x in rows[:, 1:4].sum(0)],
                              int(last[4]), int(last[5]), status])

    def trial_results(self):
        return np.array(self.rows, dtype=np.int64)


def run_sharded_model(O, p, deg, ids, rank, world, poll=10):
    """The window protocol of the sharded engine (gs_api.cpp shard_windows),
    restated over oracle shards: a window of L = min(max(delaylow,1), 10)
    ticks (never crossing a poll) starts by all-gathering every shard's firing
    sets of its L ticks -- all already scheduled, since a Broadcast fires at
    least delaylow ticks after its cause -- then each shard delivers to its own
    nodes; the per-tick counters are summed over shards at every poll."""
    from gossip_simulator_amd import dist as gd
    lo, hi = gd.shard_range(p.n, rank, world)
    e = O.Engine(p, deg, ids)
    e.set_range(lo, hi)
    e.begin(-1)
    L = min(max(p.delay_low, 1), 10)
    polls, acc = [], np.zeros(7, dtype=np.int64)
    while True:
        rows = []
        while len(rows) < poll:
            n = min(L, poll - len(rows))
            for k in range(n):  # the window's firing sets, all-gathered
                t = e.tick + 1 + k
                mine = np.zeros_like(e.get_slot(t))
                w = e.get_slot(t)
                mine[lo // 64:-(-hi // 64)] = w[lo // 64:-(-hi // 64)]
                full = torch.from_numpy(mine.view(np.int64).copy())
                gathered = [torch.zeros_like(full) for _ in range(world)]
                dist.all_gather(gathered, full)
                e.set_slot(t, np.bitwise_or.reduce([g.numpy().view(np.uint64) for g in gathered]))
            rows.extend(e.step(n).astype(np.int64))
        rows = np.array(rows)
        local = torch.tensor([*rows[:, 1:4].sum(0), rows[-1, 4], rows[-1, 5], rows[-1, 6]], dtype=torch.int64)
        dist.all_reduce(local)
        g = local.numpy()
        acc[0] = rows[-1, 0]
        acc[1:4] += g[:3]
        acc[4:7] = g[3:]
        polls.append(acc.copy())
        if O.covered(int(acc[4]), p.n) or int(acc[6]) == 0:
            return np.array(polls), e


def _sharded_worker(rank, world, port, kw, out_dir):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import pyoracle as O
    p = O.make_params(**kw)
    deg, ids, _, _ = O.overlay(p)
    polls, e = run_sharded_model(O, p, deg, ids, rank, world)
    np.save(os.path.join(out_dir, f"polls{rank}.npy"), polls)
    np.save(os.path.join(out_dir, f"recv{rank}.npy"), e.received())
    np.save(os.path.join(out_dir, f"crash{rank}.npy"), e.crashed())
    dist.destroy_process_group()


def pp_round_shard(O, p, deg, ids, inf, dead, t, lo, hi, rev):
    """One sharded push-pull round restated (k_ppb_round on nodes [lo, hi)):
    returns this shard's newly informed nodes and its (fired, sent, msgs)."""
    key = [int(p.seed) & 0xFFFFFFFF, int(p.seed) >> 32]
    kd = O.threshold(p.drop_rate)
    c3 = (9 << 24) | int(p.trial)

    def call(v):  # v's keyed pick slot and whether the call is kept
        r = O.philox([v, t, 0, c3], key)
        return (r[0] * int(deg[v])) >> 32, ((r[1] * 100) >> 32) >= kd

    fired = sent = msgs = 0
    new = []
    for v in range(lo, hi):
        if dead[v]:
            continue
        d = int(deg[v])
        if d:
            fired += 1
            j, kept = call(v)
            if inf[v]:
                if kept:  # a push: counted by the caller, found by the receiver's owner
                    sent += 1
                    msgs += 0 if dead[int(ids[v, j])] else 1
                continue
            u = int(ids[v, j])
            if kept and inf[u]:  # a pull from an informed friend
                sent += 1
                msgs += 1
                new.append(v)
                continue
        if inf[v]:
            continue
        for (w, jw) in rev.get(v, ()):  # pushes v receives: its in-edges
            if inf[w] and int(deg[w]) and call(w) == (jw, True):
                new.append(v)
                break
    return new, fired, sent, msgs


def pp_round_shard_answer(O, p, deg, ids, inf, dead, t, lo, hi, rev):
    """One sharded pull-answer round restated (k_ppa_round on nodes [lo, hi)):
    each own informed node pushes (its own row) and answers the pulls among its
    in-edges; returns the nodes it informs ANYWHERE (they go to their owners)
    and this shard's (fired, sent, msgs)."""
    key = [int(p.seed) & 0xFFFFFFFF, int(p.seed) >> 32]
    kd = O.threshold(p.drop_rate)
    c3 = (9 << 24) | int(p.trial)

    def call(v):
        r = O.philox([v, t, 0, c3], key)
        return (r[0] * int(deg[v])) >> 32, ((r[1] * 100) >> 32) >= kd

    fired = sent = msgs = 0
    new = []
    for u in range(lo, hi):
        if dead[u]:
            continue
        d = int(deg[u])
        fired += d > 0
        if not inf[u]:
            continue
        if d:
            j, kept = call(u)
            if kept:
                sent += 1
                w = int(ids[u, j])
                if not dead[w]:
                    msgs += 1
                    new.append(w)
        for (v, jv) in rev.get(u, ()):  # the pulls u answers: callers v anywhere
            if not inf[v] and not dead[v] and call(v) == (jv, True):
                sent += 1
                msgs += 1
                new.append(v)
    return new, fired, sent, msgs


def _pp_answer_worker(rank, world, port, kw, out_dir):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import pyoracle as O
    from gossip_simulator_amd import dist as gd
    p = O.make_params(**kw)
    deg, ids, _, _ = O.overlay(p)
    n = int(p.n)
    lo, hi = gd.shard_range(n, rank, world)
    dead = np.random.default_rng(3).random(n) < 0.02
    rev = {}
    for v in range(n):
        for j in range(int(deg[v])):
            u = int(ids[v, j])
            if lo <= u < hi:
                rev.setdefault(u, []).append((v, j))
    inf = np.zeros(n, bool)
    s = int(O.pick_sender(p))
    inf[s] = not dead[s]
    rows, recv = [], int(inf.sum())
    for t in range(1, 31):
        new, fired, sent, msgs = pp_round_shard_answer(O, p, deg, ids, inf, dead, t, lo, hi, rev)
        mark = np.zeros(n, np.uint8)
        mark[np.array(new, dtype=np.int64)] = 1
        g = torch.from_numpy(mark)
        dist.all_reduce(g, op=dist.ReduceOp.MAX)  # the bits every shard set, at their owners
        nxt = inf | g.numpy().astype(bool)
        c = torch.tensor([fired, sent, msgs], dtype=torch.int64)
        dist.all_reduce(c)
        recv += int((nxt & ~inf).sum())
        inf = nxt
        rows.append([t, *c.tolist(), recv, 0, recv])
    np.save(os.path.join(out_dir, f"pa{rank}.npy"), np.array(rows, dtype=np.int64))
    dist.destroy_process_group()


def _pp_sharded_worker(rank, world, port, kw, out_dir):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import pyoracle as O
    from gossip_simulator_amd import dist as gd
    p = O.make_params(**kw)
    deg, ids, _, _ = O.overlay(p)
    n = int(p.n)
    lo, hi = gd.shard_range(n, rank, world)
    dead = np.random.default_rng(3).random(n) < 0.02
    rev = {}
    for v in range(n):
        for j in range(int(deg[v])):
            u = int(ids[v, j])
            if lo <= u < hi:
                rev.setdefault(u, []).append((v, j))
    inf = np.zeros(n, bool)
    s = int(O.pick_sender(p))
    inf[s] = not dead[s]
    rows, recv = [], int(inf.sum())
    for t in range(1, 31):
        new, fired, sent, msgs = pp_round_shard(O, p, deg, ids, inf, dead, t, lo, hi, rev)
        mine = np.zeros(hi - lo, bool)
        mine[np.array(new, dtype=np.int64) - lo] = True
        mine |= inf[lo:hi]
        seg = gd.shard_range(n, 0, world)[1]  # every segment padded to the first (full) shard's size
        part = torch.from_numpy(np.pad(mine, (0, seg - (hi - lo))))
        got = [torch.zeros_like(part) for _ in range(world)]
        dist.all_gather(got, part)
        nxt = np.concatenate([g.numpy() for g in got])[:n]
        c = torch.tensor([fired, sent, msgs], dtype=torch.int64)
        dist.all_reduce(c)
        recv += int((nxt & ~inf).sum())
        inf = nxt
        rows.append([t, *c.tolist(), recv, 0, recv])
    np.save(os.path.join(out_dir, f"pp{rank}.npy"), np.array(rows, dtype=np.int64))
    np.save(os.path.join(out_dir, f"ppinf{rank}.npy"), inf)
    dist.destroy_process_group()


def _trials_worker(rank, world, port, out_dir):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import pyoracle as O
    from gossip_simulator_amd import dist as gd
    from gossip_simulator_amd.engine import Config
    cfg = Config(n=3000, crashrate=0.01, seed=5)
    res = gd.run_trials(lambda c: OracleBatch(O, c), cfg, total=7, rank=rank, world=world)
    np.save(os.path.join(out_dir, f"trials{rank}.npy"), res)
    dist.destroy_process_group()


@pytest.mark.parametrize("kw", [
    dict(n=50000, fanout=5, fanin=6, delay_low=10, delay_high=20, drop_rate=0.1, crash_rate=0.02,
         seed=0x5EED, trial=0),
    dict(n=12345, fanout=3, fanin=6, delay_low=10, delay_high=11, drop_rate=0.2, crash_rate=0.0,
         seed=3, trial=2),
])
def test_node_range_sharding_world2_bit_identical(oracle, tmp_path, kw):
    world = 2
    mp.start_processes(_sharded_worker, args=(world, free_port(), kw, str(tmp_path)),
                       nprocs=world, join=True, start_method="spawn")
    p = oracle.make_params(**kw)
    deg, ids, _, _ = oracle.overlay(p)
    rows, e = oracle.run_to_coverage(p, deg, ids)
    polls0 = np.load(tmp_path / "polls0.npy")
    polls1 = np.load(tmp_path / "polls1.npy")
    assert np.array_equal(polls0, polls1)  # every rank sees the same global stats
    # per-poll: tick, summed fired/sent/messages, cumulative received/crashed/pending
    want = []
    for i in range(0, len(rows), 10):
        blk = rows[i:i + 10].astype(np.int64)
        want.append([blk[-1, 0], *blk[:, 1:4].sum(0), blk[-1, 4], blk[-1, 5], blk[-1, 6]])
    want = np.array(want)
    want[:, 1:4] = np.cumsum(want[:, 1:4], axis=0)
    assert np.array_equal(polls0, want)
    recv = np.load(tmp_path / "recv0.npy") | np.load(tmp_path / "recv1.npy")
    crash = np.load(tmp_path / "crash0.npy") | np.load(tmp_path / "crash1.npy")
    assert np.array_equal(recv, e.received()) and np.array_equal(crash, e.crashed())
    assert not (np.load(tmp_path / "recv0.npy") & np.load(tmp_path / "recv1.npy")).any()


def test_pushpull_node_range_sharding_world2_bit_identical(oracle, tmp_path):
    """Config C5's push-pull in two node-range shards (bottom-up rounds on the
    own nodes, all-gather of the owned informed words): every round equals
    the oracle's unsharded pushpull_step, 2 % of the nodes failed."""
    kw = dict(n=20000, fanout=5, fanin=6, delay_low=10, delay_high=20, drop_rate=0.1, crash_rate=0.0,
              seed=0x5EED, trial=0, model=1)
    world = 2
    mp.start_processes(_pp_sharded_worker, args=(world, free_port(), kw, str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    a, b = np.load(tmp_path / "pp0.npy"), np.load(tmp_path / "pp1.npy")
    assert np.array_equal(a, b)
    p = oracle.make_params(**kw)
    deg, ids, _, _ = oracle.overlay(p)
    n = int(p.n)
    dead = np.random.default_rng(3).random(n) < 0.02
    w = np.zeros((n + 63) // 64, np.uint64)
    idx = np.nonzero(dead)[0]
    np.bitwise_or.at(w, idx // 64, np.left_shift(np.uint64(1), (idx % 64).astype(np.uint64)))
    e = oracle.Engine(p, deg, ids)
    e.set_failed(w)
    e.begin(-1)
    want = e.step(30).astype(np.int64)
    want[:, 5] = 0
    assert np.array_equal(a, want)
    inf = np.load(tmp_path / "ppinf0.npy")
    rec = e.received()
    bits = (rec[np.arange(n) // 64] >> (np.arange(n) % 64).astype(np.uint64)) & np.uint64(1)
    assert np.array_equal(inf, bits.astype(bool))


def test_pushpull_pull_answer_sharding_world2_bit_identical(oracle, tmp_path):
    """The sharded pull-answer round (gs_api.cpp pp_shard_step, k_ppa_round on
    each shard's informed nodes, their bits in other ranges sent to the owners)
    restated over gloo, every round pull-answer: equal to the oracle's
    unsharded pushpull_step per round, 2 % failed."""
    kw = dict(n=20000, fanout=5, fanin=6, delay_low=10, delay_high=20, drop_rate=0.1, crash_rate=0.0,
              seed=0x5EED, trial=0, model=1)
    world = 2
    mp.start_processes(_pp_answer_worker, args=(world, free_port(), kw, str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    a, b = np.load(tmp_path / "pa0.npy"), np.load(tmp_path / "pa1.npy")
    assert np.array_equal(a, b)
    p = oracle.make_params(**kw)
    deg, ids, _, _ = oracle.overlay(p)
    n = int(p.n)
    dead = np.random.default_rng(3).random(n) < 0.02
    w = np.zeros((n + 63) // 64, np.uint64)
    idx = np.nonzero(dead)[0]
    np.bitwise_or.at(w, idx // 64, np.left_shift(np.uint64(1), (idx % 64).astype(np.uint64)))
    e = oracle.Engine(p, deg, ids)
    e.set_failed(w)
    e.begin(-1)
    want = e.step(30).astype(np.int64)
    want[:, 5] = 0
    assert np.array_equal(a, want)


def test_trial_sharding_world2_matches_serial(oracle, tmp_path):
    world = 2
    mp.start_processes(_trials_worker, args=(world, free_port(), str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    a = np.load(tmp_path / "trials0.npy")
    b = np.load(tmp_path / "trials1.npy")
    assert np.array_equal(a, b)
    from gossip_simulator_amd import dist as gd
    from gossip_simulator_amd.engine import Config
    serial = gd.run_trials(lambda c: OracleBatch(oracle, c), Config(n=3000, crashrate=0.01, seed=5),
                           total=7)
    assert np.array_equal(a, serial)
    assert list(a[:, 0]) == list(range(7))
    assert set(a[:, 8]) <= {0, 1}  # covered, or the flood died out (crash 1 %)
    assert (a[a[:, 8] == 0, 1] > 0).all()


def test_shard_ranges_cover_and_align():
    from gossip_simulator_amd import dist as gd
    for n in (20000, 50000, 10**6, 10**8 + 7):
        for world in (1, 2, 3, 8):
            rs = [gd.shard_range(n, r, world) for r in range(world)]
            if rs[-1][0] == n:  # a shard of whole buckets would be empty: gs_create_* refuses
                continue
            assert rs[0][0] == 0 and rs[-1][1] == n
            for (lo, hi), (lo2, _) in zip(rs, rs[1:]):
                assert hi == lo2 and lo % 16384 == 0 and hi > lo


def test_trial_ranges_partition():
    from gossip_simulator_amd import dist as gd
    for total in (1, 7, 10000):
        for world in (1, 2, 8):
            rs = [gd.trial_range(total, r, world) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
