#!/usr/bin/env python3
"""Benchmark: gossip messages delivered per second in the broadcast phase.

Workload (BASELINE.json metric "gossip messages delivered/sec at N=1e9"): one
push-flooding broadcast over a GPU-built overlay of N = 1e9 nodes, fanout 5,
fanin 6, delays 10-20 ms, droprate 0.1, crashrate 0.01 (config C5's loss and
crash settings, reference model; the push-pull and failure-mask extensions are
not in this line).  A "step" is one whole broadcast: gs_broadcast_begin, ticks
until a 10-tick poll sees float32(received)/float32(N) >= 0.99
(simulator.go:239-253), then gs_reset.  Inputs (peer table, state) are resident
in HBM before the timed region; the overlay build is timed separately.

Multi-GPU: one process per GPU; each rank runs an independent trial (its own
overlay, trial = rank) -- batched Monte Carlo trials with no data-path
collective, so "scaling" is weak and value = all ranks' counted messages / the
slowest rank's time.  BASELINE.json's 8-GPU target is ONE N = 1e9 run across
the GPUs: the line's top-level `strong_scaling` block reports exactly that --
the C5 flood and the C5 push-pull broadcast node-range sharded over the ranks
(one run, total work fixed), with every rank's device time beside the wall;
at --gpus 1 the block holds the same workloads on the one GPU (the headline
broadcast and the unsharded push-pull), so the 1 -> N ratio is explicit.  `value` counts the reference's TotalMessage
(simulator.go:111: a receipt counted at a live node, config.messages_per_step);
delivered sends (friend slots not dropped, :144-145) are 2 % more -- they also
reach crashed nodes -- and are config.delivered_per_s / delivered_per_step.

Extensions in the same line: config C3 (10,000 trials of N = 1e5, batched
contexts, split over the ranks), config C4 (N = 1e8, fanout 18, fanin 19,
one broadcast node-range sharded over the ranks: each rank expands its own
fires and an all-to-all per window inside libgossip_hip.so moves every message
to its target's owner; one shard at --gpus 1), and config C5's push-pull and
failure-mask runs.  `--transport gloo` runs the world > 1 legs with the
exchange over a gloo group instead of RCCL, so two ranks can rehearse them on
one GPU (tests/test_bench_ranks.py).

Roofline: HBM-bound; 12 algorithmic bytes per delivered send (4-B friend id +
4-B read and 4-B write of the target's state word), divided by
the device time of the tick kernels measured with HIP events on the engine's
own stream (an extra, instrumented broadcast after the timed steps).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
BYTES_PER_SEND = 12


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    # --nodes: the same, unambiguous behind torch.distributed.run (whose own options --nnodes,
    # --nproc-per-node, ... make a bare --n ambiguous there)
    ap.add_argument("--n", "--nodes", dest="n", type=int, default=1_000_000_000)
    ap.add_argument("--fanout", type=int, default=5)
    ap.add_argument("--fanin", type=int, default=6)
    ap.add_argument("--delaylow", type=int, default=10)
    ap.add_argument("--delayhigh", type=int, default=20)
    ap.add_argument("--droprate", type=float, default=0.1)
    ap.add_argument("--crashrate", type=float, default=0.01)
    ap.add_argument("--seed", type=int, default=0x5EED)
    ap.add_argument("--cpu-n", type=int, default=100_000_000,
                    help="nodes in the bounded CPU-baseline sample (0 = skip)")
    ap.add_argument("--cpu-cap", type=float, default=40.0, help="seconds the CPU-baseline broadcast may run")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--no-c3", action="store_true", help="skip the C3 batched-trials run")
    ap.add_argument("--no-c4", action="store_true", help="skip the C4 node-range-sharded run")
    ap.add_argument("--c3-trials", type=int, default=10_000)
    ap.add_argument("--c3-batch", type=int, default=5000, help="trials per batched context")
    ap.add_argument("--c3-members", type=int, default=4,
                    help="C3: contexts of one rank's trials run at once on its GPU (gs_create_multi with the "
                         "device repeated: every member builds and runs its batch on its own stream); 1 = "
                         "one batch context renumbered batch after batch")
    ap.add_argument("--no-extensions", action="store_true",
                    help="skip the C5 extension runs (1%% failed mask, push-pull)")
    ap.add_argument("--shard-scaling", action="store_true",
                    help="at --gpus 1: per-shard device time of G = 1/2/4/8 in-process shards (C4 at N=1e8, "
                         "C5's flood at N=1e9 with G=8)")
    ap.add_argument("--pp-shards", type=int, default=8, help="in-process push-pull shards at --gpus 1")
    ap.add_argument("--ext-deadline", type=float, default=300.0,
                    help="seconds the extension legs may take before the line is printed without the rest")
    ap.add_argument("--transport", choices=("rccl", "gloo"), default="rccl",
                    help="world > 1: the ranks' exchange -- RCCL inside the library (one GPU per rank), or "
                         "host callbacks over a gloo group (gs_create_rank_exchange; ranks may share a GPU)")
    ap.add_argument("--c4-n", type=int, default=100_000_000, help="nodes of the C4 leg")
    return ap.parse_args()


def log(msg):
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


_DIST = ["cuda"]  # device of the bench's own host-side reductions: "cuda" (RCCL) or "cpu" (gloo)


def allreduce(dist, vals, op):
    """Element-wise sum or max of a few floats over the ranks (on the GPU for
    RCCL, on the host for gloo)."""
    import torch
    t = torch.tensor([float(v) for v in vals], dtype=torch.float64, device=_DIST[0])
    dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM)
    return [float(x) for x in t.cpu()]


def open_rank_shard(a, gd, cfg, rank, world):
    """This rank's shard of one node-range-sharded broadcast: RCCL inside the
    library (gs_create_rank), or the gloo host exchange (--transport gloo)."""
    if a.transport == "gloo":
        return gd.open_shard_exchange(cfg, rank, world)
    return gd.open_shard(cfg, rank, world)


DEADLINE_EXIT = 3  # exit status after the extension deadline fired
_LEG = ["headline"]  # the leg running now (for the deadline watchdog)


def devmem_delta(before):
    """The library's device-memory figures since `before` (gs_memory_stats):
    time inside hipMalloc / hipFree, the longest single hipMalloc so far, and
    the buffers served from its cache of large blocks."""
    import gossip_simulator_amd as gs
    now = gs.memory_stats()
    return {"alloc_ms": round(now["alloc_ms"] - before["alloc_ms"], 3),
            "free_ms": round(now["free_ms"] - before["free_ms"], 3),
            "largest_alloc_ms_so_far": round(now["largest_alloc_ms"], 3),
            "hip_mallocs": int(now["alloc_calls"] - before["alloc_calls"]),
            "cache_hits": int(now["alloc_cache_hits"] - before["alloc_cache_hits"]),
            "cached_gb_after": round(now["cached_bytes"] / 1e9, 3)}


def guarded(name, fn):
    """An extension leg that raises is recorded as {"error": ...} so the
    headline line still prints (every rank runs the same legs, so a
    parameter error raises on all of them alike).  A leg's result carries
    its device-memory figures (devmem_delta)."""
    import gossip_simulator_amd as gs
    _LEG[0] = name
    before = gs.memory_stats()
    try:
        out = fn()
    except Exception as e:  # noqa: BLE001 -- reported in the line, not hidden
        log(f"{name} failed: {type(e).__name__}: {e}")
        return {"error": f"{type(e).__name__}: {e}"}
    if isinstance(out, dict):
        out["devmem"] = devmem_delta(before)
    return out


class Emitter:
    """Rank 0 prints the ONE JSON line exactly once.  The extension legs run
    under a deadline (--ext-deadline s): a leg that blocks -- e.g. a
    collective of a multi-rank path waiting on a peer that failed -- must not
    swallow the headline, so when the deadline passes rank 0 prints the line
    with the unfinished leg marked and every rank exits at once, with status
    DEADLINE_EXIT: the line is there, but the run did not finish, and the
    exit status says so (torchrun, CI and the evidence scripts see a failure)."""

    def __init__(self, rank):
        import threading
        self.rank = rank
        self.lock = threading.Lock()
        self.done = False
        self.line = None
        self.timer = None

    def emit(self):
        with self.lock:
            if self.done:
                return
            self.done = True
            if self.rank == 0 and self.line is not None:
                try:
                    text = json.dumps(self.line)
                except RuntimeError:  # a leg changed the extensions dict meanwhile
                    text = json.dumps(dict(self.line, extensions={"error": "deadline while a leg was writing"}))
                print(text, flush=True)

    def arm(self, seconds, ext):
        import threading

        def fire():
            log(f"extension deadline ({seconds:.0f} s) passed in leg {_LEG[0]}: printing the line and exiting")
            if ext is not None:
                ext[_LEG[0]] = {"error": f"deadline: unfinished after {seconds:.0f} s of extension legs"}
            self.emit()
            sys.stdout.flush()
            sys.stderr.flush()
            os._exit(DEADLINE_EXIT)

        self.timer = threading.Timer(seconds, fire)
        self.timer.daemon = True
        self.timer.start()

    def disarm(self):
        if self.timer is not None:
            self.timer.cancel()


def main():
    a = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        if a.transport == "gloo":
            # ranks may share a GPU (a one-GPU rehearsal of the multi-rank legs)
            local = local % max(torch.cuda.device_count(), 1)
            torch.cuda.set_device(local)
            dist.init_process_group("gloo")
            _DIST[0] = "cpu"
        else:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
            _DIST[0] = "cuda"

    import gossip_simulator_amd as gs

    cfg = gs.Config(n=a.n, fanout=a.fanout, fanin=a.fanin, delaylow=a.delaylow,
                    delayhigh=a.delayhigh, droprate=a.droprate, crashrate=a.crashrate,
                    seed=a.seed, trial=rank, device=local)
    mem0 = gs.memory_stats()
    sim = gs.Simulator(cfg)
    t0 = time.perf_counter()
    wins, stab = sim.build_overlay()
    overlay_s = time.perf_counter() - t0
    # the build's wait inside hipMalloc: on a box whose previous process freed
    # most of the HBM, the first large allocations wait seconds for that memory
    # (DESIGN.md section 9); reported beside the wall time, not hidden
    overlay_alloc_ms = gs.memory_stats()["alloc_ms"] - mem0["alloc_ms"]
    otm = sim.timing()
    ov_ticks = {"partition": int(otm["ov_part_ticks"]), "sort": int(otm["ov_sort_ticks"]),
                "partition_fallbacks": int(otm["ov_part_fallbacks"])}
    log(f"rank {rank}: overlay n={a.n} stabilised at {stab} ms simulated, {overlay_s:.2f} s wall, ticks {ov_ticks}")

    def one_step():
        sim.reset()
        sim.broadcast_begin(-1)
        polls, status = sim.run(poll=10)
        tot = sim.totals()
        return tot, status

    for _ in range(a.warmup):
        tot, status = one_step()
        log(f"rank {rank}: warmup ticks={tot['tick']} sent={tot['sent']} status={status}")

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    barrier()
    t1 = time.perf_counter()
    sent = counted = 0
    ticks = []
    for _ in range(a.steps):
        tot, status = one_step()
        sent += tot["sent"]
        counted += tot["messages"]
        ticks.append(tot["tick"])
    recv_last = tot["received"]
    barrier()
    elapsed = time.perf_counter() - t1
    msgs = tot["messages"]
    if dist is not None:
        elapsed = allreduce(dist, [elapsed], "max")[0]
        sent_all, counted_all = (int(x) for x in allreduce(dist, [sent, counted], "sum"))
    else:
        sent_all, counted_all = sent, counted
    # value: the reference's TotalMessage (simulator.go:111, a receipt counted at a
    # live node) per second; delivered sends (:144-145, what the kernels move and
    # the roofline prices) are 2 % more and reported as config.delivered_per_s
    value = counted_all / elapsed

    roof = None
    if not a.no_roofline:
        sim.set_flags(True)
        sim.reset()
        sim.broadcast_begin(-1)
        sim.run(poll=10)
        tm = sim.timing()
        tot_r = sim.totals()
        kern_ms = tm["deliver_ms"] + tm["resolve_ms"]
        launches = int(tm["resolve_launches"])
        achieved = BYTES_PER_SEND * tot_r["sent"] / (kern_ms * 1e-3) / 1e9
        per = {"k_expand": tm["expand_ms"], "k_plan+k_part2": tm["part_ms"],
               "k_resolve": tm["resolve_ms"]}
        traffic, tnote = pmc_traffic()
        alg = int(BYTES_PER_SEND * tot_r["sent"] / max(launches, 1))
        roof = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                "traffic_ratio": round(traffic / alg, 3) if traffic and alg else None,
                "traffic_note": tnote + "; traffic_ratio = PMC bytes / algorithmic bytes per launch",
                "kernel": "window pipeline k_expand -> k_plan/k_part2 -> k_resolve "
                          "(one launch of each per window)",
                "avg_launch_us": round(kern_ms * 1e3 / max(launches, 1), 2),
                "launches": launches,
                "bytes_per_launch": alg,
                "kernels_avg_us": {k: round(v * 1e3 / max(launches, 1), 2) for k, v in per.items()},
                "kernels_total_ms": {k: round(v, 3) for k, v in per.items()},
                "exact_redos": int(tm["exact_redos"]),
                "broadcast_device_ms": round(kern_ms, 3)}
        sim.set_flags(False)

    ext = None if a.no_extensions else {}
    out = Emitter(rank)
    out.line = {
        "metric": "gossip messages delivered/sec (node) at N=1e9; rounds-to-coverage parity",
        "value": round(value, 1),
        "unit": "msgs/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(elapsed * 1e3 / a.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (GPU-built overlay, keyed Philox)",
        "config": {"workload": "C5-reference-model: single push-flood broadcast per GPU",
                   "value_counts": "TotalMessage (simulator.go:111: receipts counted at live nodes); "
                                   "delivered sends (:144-145) in delivered_per_s",
                   "delivered_per_s": round(sent_all / elapsed, 1),
                   "n": a.n, "fanout": a.fanout, "fanin": a.fanin,
                   "delaylow": a.delaylow, "delayhigh": a.delayhigh,
                   "droprate": a.droprate, "crashrate": a.crashrate,
                   # a step ends at the first 10-tick poll with float32 coverage
                   # >= 99 % (covered) or with no broadcast pending (quiescent:
                   # with crashrate 0.01 about 1 % of the nodes crash on their
                   # first receipt, so 99 % can be out of reach)
                   "ticks": ticks[-1], "status": STATUS[status],
                   "coverage": round(recv_last / a.n, 6),
                   "delivered_per_step": sent // a.steps,
                   "messages_per_step": msgs, "overlay_s": round(overlay_s, 3),
                   "overlay_alloc_ms": round(overlay_alloc_ms, 3), "overlay_ticks": ov_ticks,
                   "overlay_stabilised_ms": stab, "parallelism": f"trials{world}",
                   "transport": a.transport if world > 1 else None},
        "roofline": roof,
        "devmem": {"headline": devmem_delta(mem0)},
        "cpu_baseline": None,
        "extensions": ext,
    }
    if ext is not None:
        out.arm(a.ext_deadline, ext)
        ext["flood_failed_1pct"] = guarded("flood_failed_1pct", lambda: flood_failed(a, sim))
    sim.close()
    if not a.no_extensions:
        # round 5 put C3 and C4 before push-pull when allocations after ~100 GB
        # of frees ran seconds slow; the library's cache
        # of large device blocks (gs_devmem.cpp) now keeps freed blocks mapped
        # for the next context, and every leg reports its hipMalloc time
        # (`devmem`)
        if not a.no_c3:
            ext["c3_trials"] = guarded("c3_trials", lambda: c3_trials(a, gs, rank, world, local, dist))
        if not a.no_c4:
            ext["c4_sharded"] = guarded("c4_sharded", lambda: c4_sharded(a, gs, rank, world, local, dist))
        pp = guarded("pushpull", lambda: pushpull_runs(a, gs, rank, local))
        dm = pp.pop("devmem", None)
        ext.update(pp if "error" not in pp else {"pushpull": pp})
        if dm is not None and isinstance(ext.get("pushpull"), dict):
            ext["pushpull"]["devmem"] = dm
        if world > 1:
            ext["c5_flood_sharded"] = guarded("c5_flood_sharded",
                                              lambda: c5_flood_sharded(a, gs, rank, world, local, dist))
        ext["c5_pushpull_sharded"] = guarded("c5_pushpull_sharded",
                                             lambda: pushpull_sharded(a, gs, rank, world, local, dist))
        if world == 1 and a.shard_scaling:
            ext["c4_shards_inproc"] = guarded("c4_shards_inproc", lambda: shards_inproc(a, gs))
        out.line["strong_scaling"] = strong_scaling_block(world, out.line, ext)
    out.disarm()
    out.line["devmem"]["process"] = devmem_delta({k: 0 for k in gs.memory_stats()})

    cpu = None
    if rank == 0 and world == 1 and a.cpu_n > 0:
        cpu = cpu_baseline(a, gs)
    out.line["cpu_baseline"] = cpu
    gs.trim()  # (see cpu_baseline) every rank gives its cached device blocks back before it exits
    out.emit()
    if dist is not None:
        dist.destroy_process_group()


def strong_scaling_block(world, line, ext):
    """BASELINE.json's multi-GPU target as measured: ONE N = 1e9 broadcast over
    `world` GPUs (total work fixed), beside the weak-scaling headline.  At
    world > 1: the flood and the push-pull runs node-range sharded over the
    ranks (c5_flood_sharded, c5_pushpull_sharded: wall time = the slowest
    rank's, device time of every rank from its GS_FLAG_TIMING run); at
    world == 1 the same workloads on the one GPU (the headline broadcast and
    the unsharded push-pull) -- the 1-GPU end of the curve."""
    ext = ext or {}
    out = {"n_gpus": world, "scaling": "strong",
           "workload": "one N=1e9 broadcast (C5 parameters) node-range sharded over the GPUs"}
    if world > 1:
        fl, pp = ext.get("c5_flood_sharded") or {}, ext.get("c5_pushpull_sharded") or {}
        out["flood"] = {k: fl.get(k) for k in ("value", "unit", "ms_per_step", "device_ms_per_step",
                                               "device_ms_per_rank", "wall_over_device", "status", "error")
                        if k in fl}
        out["pushpull"] = {k: pp.get(k) for k in ("value", "unit", "ms_per_step", "rounds_to_99", "rounds_run",
                                                  "status", "placement", "error") if k in pp}
    else:
        roof = line.get("roofline") or {}
        out["flood"] = {"value": line.get("value"), "unit": line.get("unit"), "ms_per_step": line.get("ms_per_step"),
                        "device_ms_per_step": roof.get("broadcast_device_ms"),
                        "device_ms_per_rank": [roof.get("broadcast_device_ms")], "status": line["config"].get("status")}
        pp = ext.get("pushpull") or {}
        out["pushpull"] = {k: pp.get(k) for k in ("value", "unit", "ms_per_step", "rounds_to_99", "rounds_run",
                                                  "status", "error") if k in pp}
    return out


def failed_mask(n, frac, seed):
    """Pre-failed node mask: round(frac * n) node ids drawn uniformly (with
    replacement, so slightly fewer distinct nodes), as ceil(n/64) words."""
    import numpy as np
    rng = np.random.default_rng(seed)
    idx = rng.integers(0, n, size=int(round(frac * n)), dtype=np.int64)
    w = np.zeros((n + 63) // 64, dtype=np.uint64)
    np.bitwise_or.at(w, idx >> 6, np.left_shift(np.uint64(1), (idx & 63).astype(np.uint64)))
    return w


def timed_broadcast(sim, poll=10):
    import torch
    sim.reset()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    sim.broadcast_begin(-1)
    _, status = sim.run(poll=poll)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    tot = sim.totals()
    return tot, status, dt


STATUS = {0: "covered", 1: "quiescent", 2: "max_ticks"}


def flood_failed(a, sim):
    """C5 extension: the reference's flood with 1 % of the nodes pre-failed
    (gs_set_failed); the crashrate still applies, so 99 % is out of reach and
    the run ends when no broadcast is pending."""
    sim.reset()
    sim.set_failed(failed_mask(a.n, 0.01, a.seed + 1))
    tot, status, dt = timed_broadcast(sim)
    log(f"flood+1% failed: ticks={tot['tick']} sent={tot['sent']} {dt * 1e3:.1f} ms {STATUS[status]}")
    return {"value": round(tot["messages"] / dt, 1), "unit": "msgs/s", "ms": round(dt * 1e3, 3),
            "delivered_per_s": round(tot["sent"] / dt, 1), "messages": tot["messages"],
            "ticks": tot["tick"], "delivered": tot["sent"], "received": tot["received"],
            "status": STATUS[status]}


def pushpull_runs(a, gs, rank, local):
    """C5 extension: push-pull gossip over the same
    overlay (same seed -> the same table, rebuilt in a push-pull context),
    without and with 1 % pre-failed nodes.  value = delivered transmissions / s
    (calls not lost, whose receiver is live); the round's roofline (all its
    kernels: sparse k_ppe_round, top-down k_pp_round or bottom-up k_ppb_round,
    summaries, commit) at SURVEY.md 8(d)'s 8 algorithmic bytes per delivered
    message, with `traffic` / `traffic_ratio` from the committed PMC passes of
    one such broadcast (profiles/pmc_pp_traffic.json, scripts/pmc_pp.sh).
    prep_ms: the reverse-table build (first broadcast on a new table) and, in
    the 1 %-failed leg, the failed-slot mask and failed-caller bits; both sit
    inside the timed broadcast that needed them."""
    cfg = gs.Config(n=a.n, fanout=a.fanout, fanin=a.fanin, delaylow=a.delaylow,
                    delayhigh=a.delayhigh, droprate=a.droprate, crashrate=a.crashrate,
                    seed=a.seed, trial=rank, device=local, model="pushpull")
    out = {}
    with gs.Simulator(cfg) as sim:
        sim.build_overlay()
        timed_broadcast(sim)  # warmup (builds the reverse table)
        rev_ms = sim.timing()["prep_ms"]
        rev_passes = int(sim.timing()["pp_rev_part"])
        runs = [timed_broadcast(sim) for _ in range(max(a.steps, 1))]
        dt = sum(r[2] for r in runs)
        tot, status, _ = runs[-1]
        sim.set_flags(True)
        timed_broadcast(sim)
        tm = sim.timing()
        sim.set_flags(False)
        rounds = int(tm["deliver_launches"])
        ms = tm["deliver_ms"]
        # 8 algorithmic bytes per delivered push-pull message
        ach = 8 * tot["messages"] / (ms * 1e-3) / 1e9
        log(f"push-pull: rounds={tot['tick']} sent={tot['sent']} {dt * 1e3 / len(runs):.1f} ms/run")
        out["pushpull"] = {
            "value": round(sum(r[0]["messages"] for r in runs) / dt, 1), "unit": "msgs/s",
            "ms_per_step": round(dt * 1e3 / len(runs), 3), "poll": 10, "rounds_run": tot["tick"],
            "calls_per_s": round(sum(r[0]["fired"] for r in runs) / dt, 1),
            "messages_per_step": tot["messages"], "received": tot["received"],
            "status": STATUS[status],
            "roofline": {"bound": "hbm", "kernel": "one push-pull round (k_ppe_round | k_pp_round | k_ppb_round)",
                         "bytes": "8 per delivered message (SURVEY.md 8(d))",
                         "achieved": round(ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(ach / HBM_PEAK_GBS, 5),
                         "avg_launch_us": round(ms * 1e3 / max(rounds, 1), 2), "launches": rounds,
                         **pp_pmc_traffic()},
            "rev_table_prep_ms": round(rev_ms, 3),
            # passes of the partition build over the coarse bins (sized to the largest block the
            # device allocator can give without a hipFree; 0 = the atomic build)
            "rev_table_passes": rev_passes}
        # the same broadcast polled after every round instead of main's 10-tick
        # poll (simulator.go:243): push-pull is round-synchronous, so this is its
        # exact rounds-to-99 % and the rounds the 10-tick poll adds past it
        # (late bottom-up rounds, ~1.8 ms each); ms_per_step above keeps poll 10
        tot1, st1, dt1 = timed_broadcast(sim, poll=1)
        out["pushpull"]["poll_every_round"] = {"ms": round(dt1 * 1e3, 3), "rounds_to_99": tot1["tick"],
                                               "messages": tot1["messages"], "status": STATUS[st1]}
        # the exact rounds to 99 % (rounds_run: where the 10-round poll stopped)
        out["pushpull"]["rounds_to_99"] = tot1["tick"]
        sim.reset()
        sim.set_failed(failed_mask(a.n, 0.01, a.seed + 1))
        tot, status, dt = timed_broadcast(sim)
        log(f"push-pull+1% failed: rounds={tot['tick']} {dt * 1e3:.1f} ms {STATUS[status]}")
        out["pushpull_failed_1pct"] = {
            "value": round(tot["messages"] / dt, 1), "unit": "msgs/s", "ms": round(dt * 1e3, 3),
            "rounds": tot["tick"], "received": tot["received"], "status": STATUS[status],
            "prep_ms": round(sim.timing()["prep_ms"], 3)}
    return out


def c3_trials(a, gs, rank, world, local, dist):
    """Config C3: a.c3_trials trials at N = 1e5 (reference defaults), each its
    own GPU-built overlay and broadcast to its 99 % poll, split over the ranks.
    A rank runs its trials as batched contexts: one context of up to
    a.c3_members * a.c3_batch trials whose a.c3_members members (gs_create_multi
    with the rank's device repeated) each build all their trials' overlays and
    then run all their broadcasts at once, on their own streams, concurrently
    (the per-tick kernels of a batched overlay leave the GPU half idle: four
    members measured 0.91-0.97 s against 1.09 s for one 5,000-trial context
    renumbered batch after batch, profiles/r06d_c3_members.txt).  Timed: every
    batch's renumbering (gs_set_trial), overlay, broadcast and results.  The
    contexts are created and run twice before the timer, like the headline's
    warmup steps; create_s / warmup_s report that setup and s_end_to_end adds
    the creation to the batches."""
    import numpy as np
    import torch
    from dataclasses import replace
    from gossip_simulator_amd import dist as gd
    t0, t1 = gd.trial_range(a.c3_trials, rank, world)
    cfg = gs.Config(n=100_000, seed=a.seed, device=local)

    # one context per batch size, renumbered batch after batch (gs_set_trial);
    # with --c3-members M a batch is M * c3_batch trials in ONE context whose M
    # members (the same device repeated) build and run concurrently
    M = max(1, a.c3_members)
    step = a.c3_batch * M

    def open_batch(b, T):
        m = min(M, T)
        c = replace(cfg, trial=b, trials=T)
        return gs.Simulator(c, devices=[local] * m) if m > 1 else gs.Simulator(c)

    sims = {}
    create_s = warm_s = 0.0
    warm_passes = []  # each untimed pass (overlay + broadcast) of each context, s
    for b in range(t0, t1, step):  # warmup: contexts, workspaces, code objects
        T = min(b + step, t1) - b
        if T not in sims:
            tw = time.perf_counter()
            sims[T] = open_batch(b, T)
            create_s += time.perf_counter() - tw
            for rep in range(2):  # two passes: the members' buffers settle in the block cache
                tp = time.perf_counter()
                if rep:
                    sims[T].reset()
                    sims[T].set_trial(b)
                sims[T].build_overlay()
                sims[T].broadcast_begin(-1)
                sims[T].run(poll=10)
                torch.cuda.synchronize()
                warm_passes.append(round(time.perf_counter() - tp, 3))
            warm_s += time.perf_counter() - tw
            log(f"C3 warmup: context of {T} trials created and run twice in {time.perf_counter() - tw:.2f} s "
                f"(passes {warm_passes[-2:]} s)")
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    start = time.perf_counter()
    rows = []
    try:
        for b in range(t0, t1, step):
            T = min(b + step, t1) - b
            sim = sims[T]
            sim.reset()
            sim.set_trial(b)
            tb = time.perf_counter()
            sim.build_overlay()
            tm = sim.timing()
            sim.broadcast_begin(-1)
            sim.run(poll=10)
            rows.append(sim.trial_results())
            log(f"C3 batch {b}: {T} trials, overlay {tm['overlay_ms']:.0f} ms (ticks partitioned "
                f"{tm['ov_part_ticks']}, sorted {tm['ov_sort_ticks']}, fallbacks {tm['ov_part_fallbacks']}), "
                f"batch {(time.perf_counter() - tb) * 1e3:.0f} ms")
        torch.cuda.synchronize()
        dt = time.perf_counter() - start
    finally:
        for s_ in sims.values():
            s_.close()
    res = np.concatenate(rows) if rows else np.zeros((0, 9), np.int64)
    tot = [float(dt), float(res[:, 4].sum()), float(res[:, 5].sum()), float(len(res)),
           float((res[:, 8] == 0).sum())]
    if dist is not None:
        mx = allreduce(dist, [dt, create_s, warm_s], "max")
        tot = allreduce(dist, tot, "sum")
        tot[0], create_s, warm_s = mx
    dt, sent, msgs, ntr, ncov = tot
    cov = res[res[:, 8] == 0]
    log(f"C3: {int(ntr)} trials in {dt:.2f} s ({int(ncov)} covered)")
    return {"trials": int(ntr), "n": 100_000, "batch": a.c3_batch, "members": M, "s_total": round(dt, 3),
            "trials_per_s": round(ntr / dt, 1), "delivered_per_s": round(sent / dt, 1),
            "messages_per_s": round(msgs / dt, 1), "covered": int(ncov),
            "median_tick_99_rank0": int(np.median(cov[:, 1])) if len(cov) else None,
            "mean_messages_per_trial": round(msgs / max(ntr, 1), 1),
            # setup outside s_total: gs_create of the batch contexts (create_s) and their
            # two untimed passes of overlay + broadcast (warmup_s includes create_s;
            # warmup_passes_s each pass, rank 0); s_end_to_end = the contexts' creation +
            # every batch, round 4's end-to-end timer
            "create_s": round(create_s, 3), "warmup_s": round(warm_s, 3), "warmup_passes_s": warm_passes,
            "s_end_to_end": round(dt + create_s, 3),
            "note": "s_total: every batch's renumbering (gs_set_trial), overlay, broadcast to its stopping poll "
                    "and results on contexts created and run twice before the timer; s_end_to_end adds "
                    "the contexts' creation (create_s)"}


def flood_sharded(a, gs, rank, world, local, dist, n, fanout, fanin, crashrate, name):
    """ONE flood broadcast whose node range is sharded over the ranks
    (gs_create_rank: each rank expands its own fires and the messages move to
    their targets' owners by an RCCL all-to-all per window; per-step RCCL sum
    of the counters) -- one shard through the same window driver at --gpus 1.
    value = counted messages (TotalMessage) / wall time of the broadcast (max over ranks)."""
    import torch
    from gossip_simulator_amd import dist as gd
    cfg = gs.Config(n=n, fanout=fanout, fanin=fanin, delaylow=a.delaylow, delayhigh=a.delayhigh,
                    droprate=a.droprate, crashrate=crashrate, seed=a.seed, device=local)
    sim = open_rank_shard(a, gd, cfg, rank, world) if world > 1 else gs.Simulator(cfg, devices=[local])
    try:
        t0 = time.perf_counter()
        sim.build_overlay()
        ov = time.perf_counter() - t0
        steps = max(a.steps // 4, 2)
        for _ in range(2):
            sim.reset()
            sim.broadcast_begin(-1)
            sim.run(poll=10)
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(steps):
            sim.reset()
            sim.broadcast_begin(-1)
            _, status = sim.run(poll=10)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t1
        tot = sim.totals()  # global counters on every rank
        if dist is not None:
            dt = allreduce(dist, [dt], "max")[0]
        sim.set_flags(True)
        sim.reset()
        sim.broadcast_begin(-1)
        sim.run(poll=10)
        tm = sim.timing()
        sim.set_flags(False)
        kern = tm["deliver_ms"] + tm["resolve_ms"]
        launches = max(int(tm["resolve_launches"]), 1)
        per_rank = [round(kern, 3)]
        if dist is not None:
            kt = [0.0] * world
            kt[rank] = kern
            per_rank = [round(x, 3) for x in allreduce(dist, kt, "sum")]
        shard_sent = tot["sent"] / world  # a shard's share of the deliveries (balanced ranges)
        ach = BYTES_PER_SEND * shard_sent / (kern * 1e-3) / 1e9 if kern > 0 else 0.0
        log(f"{name} sharded x{world}: {dt * 1e3 / steps:.1f} ms per broadcast, "
            f"{tot['messages'] / (dt / steps):.3e} msgs/s")
        # value counts TotalMessage (simulator.go:111) like the headline
        return {"value": round(tot["messages"] * steps / dt, 1), "unit": "msgs/s", "shards": world,
                "delivered_per_s": round(tot["sent"] * steps / dt, 1),
                "ms_per_step": round(dt * 1e3 / steps, 3), "steps": steps, "n": cfg.n, "fanout": fanout,
                # wall (device-driven windows) over this rank's kernel time (GS_FLAG_TIMING run)
                "device_ms_per_step": round(kern, 3), "wall_over_device": round(dt * 1e3 / steps / kern, 4) if kern else None,
                "device_ms_per_rank": per_rank,
                "fanin": fanin, "ticks": tot["tick"], "status": STATUS[status],
                "coverage": round(tot["received"] / cfg.n, 6),
                "delivered_per_step": tot["sent"], "messages_per_step": tot["messages"],
                "overlay_s": round(ov, 3),
                "roofline": {"bound": "hbm", "kernel": "shard window pipeline k_expand (owner bins) -> k_pack -> "
                             "all-to-all -> k_plan/k_part2 -> k_resolve (rank 0; timed with GS_FLAG_TIMING, "
                             "which synchronises every window)", "achieved": round(ach, 2),
                             "peak": HBM_PEAK_GBS,
                             "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 5),
                             "avg_launch_us": round(kern * 1e3 / launches, 2), "launches": launches,
                             "kernels_total_ms": {"k_expand": round(tm["expand_ms"], 3),
                                                  "k_pack+k_plan+k_part2": round(tm["part_ms"], 3),
                                                  "k_resolve": round(tm["resolve_ms"], 3)}}}
    finally:
        sim.close()


def c4_sharded(a, gs, rank, world, local, dist):
    """Config C4: N = 1e8, fanout 18 (floor(ln 1e8)), fanin 19, reference
    defaults otherwise (crashrate 0.001 -> threshold 0), sharded over the
    ranks (flood_sharded)."""
    return flood_sharded(a, gs, rank, world, local, dist, a.c4_n, 18, 19, 0.001, "C4")


def c5_flood_sharded(a, gs, rank, world, local, dist):
    """The headline workload (C5's flood at N = 1e9) as ONE broadcast sharded
    over the ranks (--gpus > 1 only: at one GPU it is the headline itself)."""
    return flood_sharded(a, gs, rank, world, local, dist, a.n, a.fanout, a.fanin, a.crashrate, "C5 flood")


def pushpull_sharded(a, gs, rank, world, local, dist):
    """Config C5 as BASELINE.json names it: ONE N = 1e9 push-pull run whose
    node range is sharded -- over the ranks (gs_create_rank: bottom-up rounds
    on each rank's own nodes, an all-gather of the informed set's owned words
    per round over RCCL), or at --gpus 1 over a.pp_shards in-process shards on
    the one GPU (the same per-shard kernels; the shards share the device's
    copy of the informed set).  value = delivered messages / wall time."""
    import torch
    from gossip_simulator_amd import dist as gd
    cfg = gs.Config(n=a.n, fanout=a.fanout, fanin=a.fanin, delaylow=a.delaylow, delayhigh=a.delayhigh,
                    droprate=a.droprate, crashrate=0.0, seed=a.seed, device=local, model="pushpull")
    G = world if world > 1 else a.pp_shards
    sim = open_rank_shard(a, gd, cfg, rank, world) if world > 1 else gs.Simulator(cfg, devices=[local] * G)
    out = {}
    try:
        t0 = time.perf_counter()
        sim.build_overlay()
        ov = time.perf_counter() - t0
        for tag, mask in (("", None), ("_failed_1pct", failed_mask(a.n, 0.01, a.seed + 1))):
            if mask is not None:
                sim.reset()
                sim.set_failed(mask)
            runs = []
            for i in range(1 + max(a.steps // 4, 2)):
                sim.reset()
                if dist is not None:
                    dist.barrier()
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                sim.broadcast_begin(-1)
                _, status = sim.run(poll=10)
                torch.cuda.synchronize()
                dt = time.perf_counter() - t1
                if i:  # the first run warms up
                    runs.append(dt)
            dt = sum(runs) / len(runs)
            if dist is not None:
                dt = allreduce(dist, [dt], "max")[0]
            tot = sim.totals()  # global counters on every rank
            log(f"push-pull sharded x{G}{tag}: {dt * 1e3:.1f} ms, rounds={tot['tick']} {STATUS[status]}")
            out["value" if not tag else "failed_1pct"] = (
                round(tot["messages"] / dt, 1) if not tag else
                {"value": round(tot["messages"] / dt, 1), "ms": round(dt * 1e3, 3), "rounds": tot["tick"],
                 "received": tot["received"], "status": STATUS[status]})
            if not tag:
                # rounds_run: where the 10-round poll stopped; rounds_to_99: one more
                # broadcast polled every round (push-pull is round-synchronous)
                sim.reset()
                sim.broadcast_begin(-1)
                sim.run(poll=1)
                exact = sim.totals()["tick"]
                out.update({"unit": "msgs/s", "shards": G, "placement": "ranks" if world > 1 else "one GPU",
                            "ms_per_step": round(dt * 1e3, 3), "steps": len(runs), "poll": 10,
                            "rounds_run": tot["tick"], "rounds_to_99": exact,
                            "messages_per_step": tot["messages"], "received": tot["received"],
                            "status": STATUS[status], "overlay_s": round(ov, 3)})
    finally:
        sim.close()
    return out


def shards_inproc(a, gs):
    """In-process scaling proxy (one GPU): G = 1/2/4/8 node-range shards of
    config C4 (N = 1e8, fanout 18 / fanin 19) and G = 8 of C5's flood
    (N = 1e9), each shard's window pipeline run alone on the device
    (GS_SHARD_SERIAL=1) with HIP-event timing: per shard, the device time of
    one broadcast (expand of its own fires, pack, partition and resolve of
    what it receives); the slowest shard bounds a G-GPU run (plus its
    all-to-all transfers, not measured here: in-process shards read each
    other's blocks in place).  DESIGN.md section 6 compares it with the
    per-rank bytes model."""
    os.environ["GS_SHARD_SERIAL"] = "1"
    out = {}
    try:
        for name, n, fo, fi, crash, Gs in (("c4", 100_000_000, 18, 19, 0.001, (1, 2, 4, 8)),
                                           ("c5", a.n, a.fanout, a.fanin, a.crashrate, (8,))):
            for G in Gs:
                cfg = gs.Config(n=n, fanout=fo, fanin=fi, crashrate=crash, droprate=a.droprate, seed=a.seed,
                                device=0)
                with gs.Simulator(cfg, devices=[0] * G) as sim:
                    sim.build_overlay()
                    sim.broadcast_begin(-1)
                    sim.run(poll=10)  # warm-up
                    sim.set_flags(True)
                    sim.reset()
                    sim.broadcast_begin(-1)
                    sim.run(poll=10)
                    tot = sim.totals()
                    per = []
                    for i in range(G):
                        tm = sim.shard_timing(i)
                        per.append(round(tm["expand_ms"] + tm["part_ms"] + tm["resolve_ms"], 3))
                    sim.set_flags(False)
                    t0 = sim.shard_timing(0)
                    # the same broadcast device-driven (one stream, no serial syncs): its wall
                    os.environ.pop("GS_SHARD_SERIAL", None)
                    walls = []
                    for _ in range(2):
                        sim.reset()
                        sim.broadcast_begin(-1)
                        w0 = time.perf_counter()
                        sim.run(poll=10)
                        walls.append(time.perf_counter() - w0)
                    os.environ["GS_SHARD_SERIAL"] = "1"
                    key = f"{name}_G{G}"
                    out[key] = {"n": n, "shard_ms": per, "max_ms": max(per), "sum_ms": round(sum(per), 3),
                                "dd_wall_ms": round(min(walls) * 1e3, 3),
                                "dd_wall_over_sum": round(min(walls) * 1e3 / sum(per), 4),
                                "delivered": tot["sent"], "windows": int(t0["windows"]),
                                "shard0_phases_ms": {"expand": round(t0["expand_ms"], 3),
                                                     "pack+plan+part2": round(t0["part_ms"], 3),
                                                     "resolve": round(t0["resolve_ms"], 3)}}
                    log(f"in-process shards {key}: per-shard device ms {per}")
    finally:
        os.environ.pop("GS_SHARD_SERIAL", None)
    return out


def pmc_traffic():
    """HBM bytes per window launch (k_expand + k_part2 + k_resolve*) from the
    committed PMC passes (scripts/pmc.sh + scripts/pmc_traffic.py): reads =
    the L2's memory read requests by size (every one was 128 B on gfx950,
    calibrated on known byte counts: profiles/r03_fetch_calibration.json),
    writes = WRITE_SIZE (exact in the same calibration); counters cannot be
    read from inside the timed process, so this is the profile of the same
    workload at this commit's kernels, not this run."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None, "no PMC profile committed"
    d = json.load(open(path))
    return int(d["bytes_per_launch"]), (f"{os.path.relpath(path, ROOT)} (from {d['source']}): calibrated "
                                        f"read requests + WRITE_SIZE over {d['launches']} window launches "
                                        f"of one broadcast")


def pp_pmc_traffic():
    """HBM bytes of one C5 push-pull broadcast's round kernels from the
    committed PMC passes (scripts/pmc_pp.sh -> scripts/pmc_pp_traffic.py; the
    same calibrated read requests + WRITE_SIZE as pmc_traffic) against SURVEY.md
    8(d)'s 8 B per delivered message: the profile of the same workload at this
    commit's kernels, not of this run."""
    path = os.path.join(ROOT, "profiles", "pmc_pp_traffic.json")
    if not os.path.exists(path):
        return {"traffic": None, "traffic_note": "no push-pull PMC profile committed"}
    d = json.load(open(path))
    return {"traffic": int(d["round_bytes"]), "traffic_unit": "bytes per broadcast", "traffic_ratio": d["traffic_ratio"],
            "traffic_note": (f"{os.path.relpath(path, ROOT)} (from {d['source']}): bytes per broadcast over "
                             f"{d['rounds']} rounds; traffic_ratio = PMC bytes / (8 B x {d['messages']} messages)")}


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_limits():
    """What this host lets the process use: affinity and the cgroup CPU quota."""
    out = {"nproc": os.cpu_count()}
    try:
        out["affinity"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        pass
    try:
        q = open("/sys/fs/cgroup/cpu.max").read().split()
        if q and q[0] != "max":
            out["cgroup_cpus"] = round(int(q[0]) / int(q[1]), 2)
    except (OSError, ValueError, IndexError):
        pass
    return out


def cpu_threads():
    """The all-core thread count this host allows: the CPUs in the process's
    affinity mask, capped by the cgroup CPU quota when one is set (the GPU box
    gives each GPU a 16-CPU quota out of 256 CPUs: more threads than the quota
    are throttled, not faster)."""
    lim = cpu_limits()
    n = lim.get("affinity") or lim.get("nproc") or 1
    if lim.get("cgroup_cpus"):
        n = min(n, max(1, int(lim["cgroup_cpus"])))
    return n, lim


def cpu_baseline(a, gs):
    """The all-core OpenMP port of the tick model (oracle/gsomp.c, bit-exact to
    the restatement, checked in tests/test_omp_port.py) on this host: one whole
    broadcast at n = cpu_n with the same parameters, over a table the GPU
    overlay built (copied to the host); times only the port's tick loop,
    capped at --cpu-cap s.  Threads: cpu_threads() (affinity, capped by the
    cgroup quota).  msgs/s as the headline: delivered sends / time
    (simulator.go:252-253 divides TotalMessage by the broadcast's time)."""
    from oracle import pyoracle as O
    O.build()
    n = a.cpu_n
    cfg = gs.Config(n=n, fanout=a.fanout, fanin=a.fanin, delaylow=a.delaylow,
                    delayhigh=a.delayhigh, droprate=a.droprate, crashrate=a.crashrate,
                    seed=a.seed, trial=0, device=0)
    with gs.Simulator(cfg) as s:
        s.build_overlay()
        deg, ids = s.read_peers()
    # the GPU legs are over: hand the library's cached blocks back now, so the
    # driver clears them while the CPU runs, not while the next process waits
    # for its first allocations
    gs.trim()
    p = O.make_params(n=n, fanout=a.fanout, fanin=a.fanin, delay_low=a.delaylow,
                      delay_high=a.delayhigh, drop_rate=a.droprate, crash_rate=a.crashrate,
                      seed=a.seed, trial=0)
    threads, lim = cpu_threads()
    e = O.OmpEngine(p, deg, ids, threads=threads)
    del deg, ids
    e.begin(-1)
    sent = msgs = 0
    t0 = time.perf_counter()
    capped = False
    while True:
        st = e.step(10)
        sent += int(st[:, 2].sum())
        msgs += int(st[:, 3].sum())
        if O.covered(int(st[-1, 4]), n) or int(st[-1, 6]) == 0:
            break
        if time.perf_counter() - t0 > a.cpu_cap:
            capped = True
            break
    dt = time.perf_counter() - t0
    log(f"cpu baseline: {e.threads} threads, n={n}: {msgs / dt:.3e} msgs/s ({dt:.1f} s)")
    # value counts TotalMessage like the headline; delivered sends in delivered_per_s
    return {"value": round(msgs / dt, 1), "unit": "msgs/s", "cores": e.threads, "kind": "port",
            "delivered_per_s": round(sent / dt, 1), "cpu_model": cpu_model(), **lim,
            "s": round(dt, 3), "capped": capped,
            "sample": f"oracle/gsomp.c (OpenMP port of the tick model), one broadcast at n={n} to "
                      f"{'the %.0f s cap' % a.cpu_cap if capped else '99% / quiescence'} ({sent} delivered sends "
                      f"in {dt:.2f} s) with {e.threads} threads (the affinity mask capped by the cgroup quota), "
                      f"same params, GPU-built overlay"}


if __name__ == "__main__":
    main()
