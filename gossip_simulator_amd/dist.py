"""Multi-GPU execution: one process per GPU, torch.distributed for the host-side
hand-offs (RCCL on ROCm, gloo for CPU tests); the data path's collectives run
inside libgossip_hip.so.

Two partitionings; neither exists in the reference, whose
only concurrency is goroutines in one process (simulator.go:214-217):

* ``run_trials`` -- independent Monte Carlo trials (config C3).  Rank r runs
  the contiguous trials ``trial_range(total, r, world)`` as ONE batched
  context (all its trials' overlays and broadcasts at once on its GPU);
  nothing is exchanged until the per-trial rows are summed at the end.

* ``open_shard`` -- one huge-N broadcast with the node range split over ranks
  (configs C4 and C5).  Rank 0 makes an RCCL unique id, torch.distributed
  ships it to every rank, and each rank opens its shard with gs_create_rank.
  From then on the library runs the data path's exchange itself over RCCL:
  the flood expands each rank's own fires and sends every message to its
  target's owner (grouped ncclSend/ncclRecv, one all-to-all per window, with
  the window cut agreed from an all-gather of the per-rank fire counts);
  push-pull all-gathers the informed set's owned words per bottom-up round;
  the per-tick counters are summed, so gs_run on every rank returns the
  global counters.  In one process, ``Simulator(cfg, devices=[...])`` does
  the same over several devices (gs_create_multi).

* ``open_shard_exchange`` -- the same shard with the exchange done by the
  caller (gs_create_rank_exchange) over a torch.distributed CPU group
  (gloo).  It runs every multi-rank code path of the library except the
  RCCL transport, so several processes can share one GPU (RCCL refuses two
  ranks on one device): tests/test_rank_exchange.py and bench.py
  ``--transport gloo``.
"""
from __future__ import annotations

from dataclasses import replace

import numpy as np
import torch
import torch.distributed as dist

from .engine import TRIAL_FIELDS, Config, Simulator, comm_unique_id

FINE = 16384  # nodes per fine bucket; shard boundaries align to it


def trial_range(total: int, rank: int, world: int):
    """Rank r's trials [t0, t1) -- the split gs_create_rank makes."""
    return total * rank // world, total * (rank + 1) // world


def shard_range(n: int, rank: int, world: int):
    """Rank r's owned nodes [lo, hi) -- the split gs_create_multi /
    gs_create_rank make (whole 16384-node buckets per shard)."""
    per = -(-n // world)
    per = -(-per // FINE) * FINE
    lo = min(rank * per, n)
    return lo, min(lo + per, n)


def run_trials(make_batch, cfg: Config, total: int, rank: int = 0, world: int = 1,
               device: str = "cpu", poll: int = 10, max_ticks: int = 1_000_000) -> np.ndarray:
    """Trials cfg.trial .. cfg.trial+total-1 split over the ranks; returns the
    full [total, len(TRIAL_FIELDS)] table on every rank.  make_batch(cfg)
    opens one batch of cfg.trials trials starting at cfg.trial (the HIP
    engine: ``Simulator``)."""
    out = torch.zeros((total, len(TRIAL_FIELDS)), dtype=torch.int64)
    t0, t1 = trial_range(total, rank, world)
    if t1 > t0:
        sim = make_batch(replace(cfg, trial=cfg.trial + t0, trials=t1 - t0))
        try:
            sim.build_overlay()
            sim.broadcast_begin(-1)
            sim.run(poll=poll, max_ticks=max_ticks)
            out[t0:t1] = torch.from_numpy(np.asarray(sim.trial_results(), dtype=np.int64))
        finally:
            close = getattr(sim, "close", None)
            if close:
                close()
    if world > 1:
        buf = out.to(device)
        dist.all_reduce(buf, op=dist.ReduceOp.SUM)
        out = buf.cpu()
    return out.numpy()


def comm_id(rank: int, world: int) -> bytes:
    """Rank 0's RCCL unique id, shipped to every rank over torch.distributed."""
    box = [comm_unique_id() if rank == 0 else None]
    if world > 1:
        dist.broadcast_object_list(box, src=0)
    return box[0]


def open_shard(cfg: Config, rank: int, world: int) -> Simulator:
    """This rank's shard of one node-range-sharded broadcast (gs_create_rank)."""
    return Simulator.rank(cfg, world, rank, comm_id(rank, world))


def gloo_exchange(world: int, group=None):
    """The three host exchange callbacks of gs_create_rank_exchange over a
    torch.distributed CPU (gloo) group: all_gather of equal byte blocks,
    element-wise u64 sum, all_to_allv of byte blocks (rank-major)."""

    def all_gather(send: np.ndarray) -> np.ndarray:
        t = torch.from_numpy(send)
        out = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(out, t, group=group)
        return torch.cat(out).numpy()

    def all_reduce(x: np.ndarray) -> np.ndarray:
        t = torch.from_numpy(x.view(np.int64).copy())
        dist.all_reduce(t, group=group)
        return t.numpy().view(np.uint64)

    def all_to_allv(send: np.ndarray, send_sizes, recv_sizes) -> np.ndarray:
        out = torch.empty(sum(recv_sizes), dtype=torch.uint8)
        dist.all_to_all_single(out, torch.from_numpy(send), output_split_sizes=list(recv_sizes),
                               input_split_sizes=list(send_sizes), group=group)
        return out.numpy()

    return all_gather, all_reduce, all_to_allv


def open_shard_exchange(cfg: Config, rank: int, world: int, group=None) -> Simulator:
    """This rank's shard with the exchange through the caller over gloo
    (gs_create_rank_exchange): the library's per-rank logic is the RCCL
    path's; only the transport differs."""
    return Simulator.rank_exchange(cfg, world, rank, *gloo_exchange(world, group))
