"""World-size-2 gloo tests of the multi-GPU logic on CPU.

* Trial sharding: dist.run_trials (the product's host code) over gloo, with the
  oracle behind the batch interface the HIP engine exposes -- must reproduce
  the serial trials.
* Node-range sharding: the library's window protocol (gs_api.cpp
  shard_windows: per-window all-gather of the firing sets, per-poll sum of
  the counters) restated over oracle shards and gloo collectives -- must be
  bit-identical to the unsharded run.  The HIP path of the same protocol is
  checked on the GPU (tests/test_gpu_multi.py).
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
