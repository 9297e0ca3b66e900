"""Multi-GPU execution: one process per GPU, torch.distributed (RCCL on ROCm,
gloo for CPU tests).

Two partitionings; neither exists in the reference, whose
only concurrency is goroutines in one process (simulator.go:214-217):

* ``run_trials`` -- independent Monte Carlo trials (config C3).  Trial k runs
  on rank k mod world with its own keyed overlay and broadcast; nothing is
  exchanged until the per-trial results are summed at the end.

* ``run_sharded`` -- one huge-N broadcast with the node range split over
  ranks (config C4).  Rank r owns nodes [lo_r, hi_r) (4096-node aligned), its
  received/crashed bits and its fire-ring bits.  Before every tick the ranks
  all-gather their owned words of the fire slot, so every rank sees the full
  firing set; each rank then evaluates every firing node's sends with the same
  keyed Philox draws but delivers only to targets it owns.  The union over
  ranks is bit-identical to the unsharded run, and the only per-tick traffic
  is the N/8-byte frontier all-gather (plus a 6-counter all-reduce per poll).

Engines are duck-typed so the same host logic drives the HIP engine
(``HipShard``) and, in CPU tests, the oracle.
"""
from __future__ import annotations

from dataclasses import replace

import numpy as np
import torch
import torch.distributed as dist

from .engine import Config, Simulator, covered

CHUNK = 4096  # nodes per chunk = 64 bitset words; shard boundaries align to it

TRIAL_FIELDS = ("trial", "tick_99", "poll_99", "sent", "messages", "crashed", "received",
                "status")


def trials_of(total: int, rank: int, world: int) -> range:
    return range(rank, total, world)


def shard_range(n: int, rank: int, world: int):
    """Rank r's owned nodes [lo, hi) and the padded words per rank."""
    per = -(-n // world)
    per = -(-per // CHUNK) * CHUNK
    lo = min(rank * per, n)
    hi = min(lo + per, n)
    return lo, hi, per // 64


# ---------------------------------------------------------------------------
# independent trials
# ---------------------------------------------------------------------------
def run_one_trial(sim, n: int, poll: int = 10, max_ticks: int = 100000) -> list:
    """Overlay + broadcast to the first 99 % poll; exact first tick kept."""
    sim.build_overlay()
    sim.broadcast_begin(-1)
    tick99 = -1
    sent = 0
    status = 2
    while True:
        rows = sim.step(poll)
        sent += int(rows[:, 2].sum())
        msgs_last = rows[-1]
        if tick99 < 0:
            for r in rows:
                if covered(int(r[4]), n):
                    tick99 = int(r[0])
                    break
        if covered(int(msgs_last[4]), n):
            status = 0
            break
        if int(msgs_last[6]) == 0:
            status = 1
            break
        if int(msgs_last[0]) >= max_ticks:
            break
    tot = sim.totals()
    return [tick99, int(tot["tick"]), sent, tot["messages"], tot["crashed"], tot["received"], status]


def run_trials(make_sim, cfg: Config, total: int, rank: int = 0, world: int = 1,
               device: str = "cpu", poll: int = 10, concurrency: int = 1) -> np.ndarray:
    """Run trials rank, rank+world, ...; returns the full [total, 8] table on
    every rank (one all-reduce of the per-rank rows at the end).

    concurrency > 1 runs that many trials at once on the rank's GPU, one
    context (own HIP stream) per host thread: a trial at N = 1e5 launches
    small grids, so one stream alone leaves most CUs idle.  ctypes releases
    the GIL inside every C-ABI call, so the threads overlap on the device."""
    out = torch.zeros((total, len(TRIAL_FIELDS)), dtype=torch.int64)

    def one(t):
        sim = make_sim(replace(cfg, trial=t))
        try:
            return t, [t] + run_one_trial(sim, cfg.n, poll)
        finally:
            close = getattr(sim, "close", None)
            if close:
                close()

    mine = list(trials_of(total, rank, world))
    if concurrency > 1:
        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(max_workers=concurrency) as ex:
            rows = list(ex.map(one, mine))
    else:
        rows = [one(t) for t in mine]
    for t, row in rows:
        out[t] = torch.tensor(row, dtype=torch.int64)
    if world > 1:
        buf = out.to(device)
        dist.all_reduce(buf, op=dist.ReduceOp.SUM)
        out = buf.cpu()
    return out.numpy()


# ---------------------------------------------------------------------------
# node-range sharding
# ---------------------------------------------------------------------------
class HipShard:
    """Adapter: a Simulator that owns nodes [lo, hi) and exchanges its fire
    slot through torch tensors on the engine's own stream."""

    def __init__(self, cfg: Config, lo: int, hi: int, stream=None):
        self.sim = Simulator(cfg, node_range=(lo, hi))
        if stream is not None:
            self.sim.set_stream(stream)
        self.W = self.sim.words

    def build_overlay(self):
        return self.sim.build_overlay()

    def load_peers(self, deg, ids):
        self.sim.load_peers(deg, ids)

    def begin(self, sender=-1):
        self.sim.broadcast_begin(sender)

    def export_slot(self, tick: int, dst: torch.Tensor, word_lo: int, nwords: int):
        self.sim.frontier_export(tick, dst.data_ptr(), word_lo, nwords)

    def import_slot(self, tick: int, src: torch.Tensor):
        self.sim.frontier_import(tick, src.data_ptr())

    def step(self, ticks: int):
        return self.sim.step(ticks)

    @property
    def tick(self):
        return self.sim.totals()["tick"]

    def received(self):
        return self.sim.received()

    def close(self):
        self.sim.close()


def run_sharded(shard, n: int, rank: int, world: int, device: str = "cpu", poll: int = 10,
                max_ticks: int = 1_000_000, sender: int = -1):
    """Drive one node-range-sharded broadcast to the first 99 % poll.

    ``shard`` exposes begin(), export_slot(tick, tensor, word_lo, nwords),
    import_slot(tick, tensor), step(1) -> stats rows (this rank's share) and
    ``tick``.  Returns (per-poll global stats rows, status)."""
    lo, hi, wpr = shard_range(n, rank, world)
    W = (n + 63) // 64
    word_lo = lo // 64
    nwords = max(0, min(W, -(-hi // 64)) - word_lo)
    mine = torch.zeros(wpr, dtype=torch.int64, device=device)
    full = torch.zeros(wpr * world, dtype=torch.int64, device=device)
    shard.begin(sender)
    polls = []
    totals = np.zeros(7, dtype=np.int64)  # tick fired sent msgs recv crashed pending
    status = 2
    while True:
        acc = np.zeros(6, dtype=np.int64)  # fired sent msgs recv_new crash_new pending_delta
        for _ in range(poll):
            t = shard.tick + 1
            mine.zero_()
            shard.export_slot(t, mine, word_lo, nwords)
            if world > 1:
                dist.all_gather_into_tensor(full, mine)
            else:
                full.copy_(mine)
            shard.import_slot(t, full)
            row = shard.step(1)[0].astype(np.int64)
            acc += [row[1], row[2], row[3], 0, 0, 0]
            totals[0] = row[0]
        # this rank's cumulative received/crashed/pending are in the last row
        local = torch.tensor([acc[0], acc[1], acc[2], int(row[4]), int(row[5]), int(row[6])],
                             dtype=torch.int64, device=device)
        if world > 1:
            dist.all_reduce(local, op=dist.ReduceOp.SUM)
        g = local.cpu().numpy()
        totals[1:4] += g[0:3]
        totals[4:7] = g[3:6]
        polls.append(totals.copy())
        if covered(int(totals[4]), n):
            status = 0
            break
        if int(totals[6]) == 0:
            status = 1
            break
        if int(totals[0]) >= max_ticks:
            break
    return np.array(polls), status
