"""One rank of a multi-process node-range-sharded run whose exchange goes
through the caller (gs_create_rank_exchange): the callbacks move host bytes
with torch.distributed on the gloo backend.  Launched by
tests/test_rank_exchange.py, two processes on one GPU.

Usage: python tests/exchange_worker.py <rank> <world> <port> <dir> <model>
Reads <dir>/table.npz (deg, ids[, failed]) and writes <dir>/rank<r>.npz."""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    rank, world, port, d, model = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4], sys.argv[5]
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    import gossip_simulator_amd as gs

    def all_gather(send: np.ndarray) -> np.ndarray:
        t = torch.from_numpy(send)
        out = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(out, t)
        return torch.cat(out).numpy()

    def all_reduce(x: np.ndarray) -> np.ndarray:
        t = torch.from_numpy(x.view(np.int64).copy())
        dist.all_reduce(t)
        return t.numpy().view(np.uint64)

    def all_to_allv(send: np.ndarray, send_sizes, recv_sizes) -> np.ndarray:
        out = torch.empty(sum(recv_sizes), dtype=torch.uint8)
        dist.all_to_all_single(out, torch.from_numpy(send), output_split_sizes=list(recv_sizes),
                               input_split_sizes=list(send_sizes))
        return out.numpy()

    z = np.load(os.path.join(d, "table.npz"))
    if model == "overflow":  # only the rank that owns the hub overflows; every rank must return GS_EOVERFLOW
        codes = []
        for mode in ("dd", "host"):
            if mode == "host":
                os.environ["GS_SYNC_WINDOWS"] = "1"
            cfg = gs.Config(n=int(z["n"]), fanout=32, fanin=32, delaylow=10, delayhigh=11, droprate=0.0,
                            crashrate=0.01, seed=0x5EED, device=0)
            sim = gs.Simulator.rank_exchange(cfg, world, rank, all_gather, all_reduce, all_to_allv)
            code = 0
            try:
                sim.load_peers(z["deg"], z["ids"])
                sim.broadcast_begin(0)
                sim.step(45)
            except gs.GossipError as e:
                code = e.code
            finally:
                sim.close()
            codes.append(code)
        np.savez(os.path.join(d, f"rank{rank}.npz"), codes=np.array(codes))
        dist.destroy_process_group()
        return
    kw = {k: (z[k].item()) for k in ("n", "fanout", "fanin", "crashrate", "droprate")}
    cfg = gs.Config(n=int(kw["n"]), fanout=int(kw["fanout"]), fanin=int(kw["fanin"]),
                    crashrate=float(kw["crashrate"]), droprate=float(kw["droprate"]), seed=0x5EED,
                    model=model, device=0)
    sim = gs.Simulator.rank_exchange(cfg, world, rank, all_gather, all_reduce, all_to_allv)
    try:
        sim.load_peers(z["deg"], z["ids"])
        if "failed" in z:
            sim.set_failed(z["failed"])
        sim.broadcast_begin(-1)
        rows = sim.step(int(z["ticks"]))
        polls_rows, status = None, None
        rec, cra = sim.received(), sim.crashed()
        sim.reset()
        sim.broadcast_begin(-1)
        polls_rows, status = sim.run(poll=10)
        np.savez(os.path.join(d, f"rank{rank}.npz"), rows=rows, rec=rec, cra=cra, polls=polls_rows,
                 status=status, info=np.array(sim.shard_info(), dtype=np.uint64))
    finally:
        sim.close()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
