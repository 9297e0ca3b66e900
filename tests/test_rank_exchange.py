"""Multi-process node-range shards with more than one rank:
two processes, one shard each, on one GPU, exchanging through the caller
(gs_create_rank_exchange; the callbacks use torch.distributed on gloo).  The
library's per-rank logic -- window cut from the gathered fire counts, segment
sizes, the fire-list all-gather, the counter sums, push-pull's informed-set
exchange -- runs exactly as under RCCL; only the transport differs.  Both
ranks must report the unsharded run's per-tick counters, gs_run's polls and
status, and together its bitsets (each rank holds its own nodes' words).
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("model,n,fanout,fanin,crash,drop,ticks,fail", [
    ("flood", 1_000_000, 18, 19, 0.02, 0.1, 120, 0.0),     # config C4's row shape
    ("pushpull", 1_000_000, 5, 6, 0.0, 0.1, 40, 0.01),     # config C5's model, 1 % failed
])
def test_two_ranks_match_unsharded(tmp_path, model, n, fanout, fanin, crash, drop, ticks, fail):
    import gossip_simulator_amd as gs
    gs.load()
    cfg = gs.Config(n=n, fanout=fanout, fanin=fanin, crashrate=crash, droprate=drop, seed=0x5EED, model=model)
    failed = None
    if fail:
        bits = np.random.default_rng(5).random(n) < fail
        failed = np.zeros((n + 63) // 64, np.uint64)
        idx = np.nonzero(bits)[0]
        np.bitwise_or.at(failed, idx // 64, np.left_shift(np.uint64(1), (idx % 64).astype(np.uint64)))
    with gs.Simulator(cfg) as sim:
        sim.build_overlay()
        deg, ids = sim.read_peers()
        if failed is not None:
            sim.set_failed(failed)
        sim.broadcast_begin(-1)
        rows = sim.step(ticks)
        rec, cra = sim.received(), sim.crashed()
        sim.reset()
        sim.broadcast_begin(-1)
        polls, status = sim.run(poll=10)
    extra = {"failed": failed} if failed is not None else {}
    np.savez(tmp_path / "table.npz", deg=deg, ids=ids, n=n, fanout=fanout, fanin=fanin, crashrate=crash,
             droprate=drop, ticks=ticks, **extra)
    port = free_port()
    procs = [subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "exchange_worker.py"), str(r), "2",
                               str(port), str(tmp_path), model], stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
             for r in range(2)]
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append(out.decode(errors="replace"))
    for r, p in enumerate(procs):
        assert p.returncode == 0, f"rank {r} failed:\n{outs[r][-3000:]}"
    got = [np.load(tmp_path / f"rank{r}.npz") for r in range(2)]
    orr, orc = np.zeros_like(rec), np.zeros_like(cra)
    for r, g in enumerate(got):
        assert np.array_equal(g["rows"], rows), f"rank {r}: per-tick counters differ"
        assert np.array_equal(g["polls"], polls) and int(g["status"]) == status, f"rank {r}: gs_run differs"
        orr |= g["rec"]
        if model == "flood":
            orc |= g["cra"]
    assert np.array_equal(orr, rec), "the ranks' received words do not make up the unsharded bitset"
    if model == "flood":
        assert np.array_equal(orc, cra)


def test_one_rank_overflows_both_return_eoverflow(tmp_path):
    """a receipt-count overflow on ONE rank (the hub's owner) must
    end the step with GS_EOVERFLOW on every rank -- device-driven windows and
    host-driven (GS_SYNC_WINDOWS=1) alike -- instead of leaving the other rank
    waiting in a collective."""
    from test_overflow import star32_table
    n, deg, ids = star32_table()
    np.savez(tmp_path / "table.npz", deg=deg, ids=ids, n=n)
    port = free_port()
    procs = [subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "exchange_worker.py"), str(r), "2",
                               str(port), str(tmp_path), "overflow"], stdout=subprocess.PIPE,
                              stderr=subprocess.STDOUT) for r in range(2)]
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append(out.decode(errors="replace"))
    for r, p in enumerate(procs):
        assert p.returncode == 0, f"rank {r} failed:\n{outs[r][-3000:]}"
        codes = np.load(tmp_path / f"rank{r}.npz")["codes"]
        assert list(codes) == [-6, -6], f"rank {r}: {list(codes)}"

