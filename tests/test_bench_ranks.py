"""bench.py's world > 1 legs, rehearsed on one GPU (verdict r05 item 4).

Two ranks launched the way the driver launches the 8-GPU scaling run
(`torch.distributed.run --nproc-per-node 2 ... bench.py --gpus 2`), with
`--transport gloo`: the ranks share the one GPU and exchange through
gs_create_rank_exchange's host callbacks instead of RCCL (RCCL refuses two
ranks on one device).  Every multi-rank leg runs -- the per-rank headline,
C3 split over the ranks, C4 and the C5 flood node-range sharded, the
push-pull shards -- at a small N, and rank 0's line must carry every leg
without an error, two per-rank device times in `strong_scaling`, and the
same counters as a one-process run of the same workloads (simulator.go:214-217
is the single process these shards replace).
"""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--nodes", "2000000", "--c4-n", "2000000", "--c3-trials", "200", "--c3-batch", "100",
         "--steps", "2", "--warmup", "1", "--cpu-n", "0", "--pp-shards", "2", "--ext-deadline", "240"]


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def run_bench(args, nproc):
    if nproc == 1:
        cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1"] + args
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
               "--master-addr", "127.0.0.1", f"--master-port={free_port()}", os.path.join(ROOT, "bench.py"),
               "--gpus", str(nproc), "--transport", "gloo"] + args
    env = dict(os.environ, OMP_NUM_THREADS="4")
    p = subprocess.run(cmd, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=300, env=env)
    err = p.stderr.decode(errors="replace")
    assert p.returncode == 0, f"bench x{nproc} rc={p.returncode}:\n{err[-4000:]}"
    lines = [ln for ln in p.stdout.decode().splitlines() if ln.startswith("{")]
    assert len(lines) == 1, f"expected one JSON line, got {len(lines)}:\n{p.stdout.decode()[-2000:]}"
    return json.loads(lines[0]), err


def errors(d, path=""):
    out = []
    if isinstance(d, dict):
        for k, v in d.items():
            if k == "error" and v:
                out.append(f"{path}: {v}")
            else:
                out += errors(v, f"{path}.{k}")
    return out


@pytest.mark.timeout(700)
def test_two_gloo_ranks_run_every_leg():
    two, err2 = run_bench(SMALL, 2)
    one, _ = run_bench(SMALL, 1)
    assert two["n_gpus"] == 2 and two["config"]["transport"] == "gloo"
    assert not errors(two), errors(two)
    ext2, ext1 = two["extensions"], one["extensions"]
    for leg in ("c3_trials", "c4_sharded", "c5_flood_sharded", "c5_pushpull_sharded", "pushpull",
                "flood_failed_1pct"):
        assert leg in ext2, f"leg {leg} missing at world 2"
    ss = two["strong_scaling"]
    assert len(ss["flood"]["device_ms_per_rank"]) == 2
    assert all(x > 0 for x in ss["flood"]["device_ms_per_rank"])
    # rank 0's headline is trial 0, the one-process run's broadcast
    assert two["config"]["delivered_per_step"] == one["config"]["delivered_per_step"]
    # the C5 flood sharded over 2 ranks = the unsharded headline broadcast
    fl = ext2["c5_flood_sharded"]
    assert fl["shards"] == 2
    assert fl["delivered_per_step"] == one["config"]["delivered_per_step"]
    assert fl["messages_per_step"] == one["config"]["messages_per_step"]
    assert fl["ticks"] == one["config"]["ticks"]
    # C4 over 2 ranks = C4 as one shard
    for k in ("delivered_per_step", "messages_per_step", "ticks", "status"):
        assert ext2["c4_sharded"][k] == ext1["c4_sharded"][k], k
    assert ext2["c4_sharded"]["shards"] == 2
    # push-pull over 2 ranks = the unsharded push-pull (crashrate is unused by push-pull)
    pp2 = ext2["c5_pushpull_sharded"]
    assert pp2["placement"] == "ranks" and pp2["shards"] == 2
    assert pp2["messages_per_step"] == ext1["pushpull"]["messages_per_step"]
    assert pp2["rounds_to_99"] == ext1["pushpull"]["rounds_to_99"]
    assert pp2["failed_1pct"]["received"] == ext1["pushpull_failed_1pct"]["received"]
    # C3: the 200 trials split over 2 ranks = the same 200 trials on one
    c3a, c3b = ext2["c3_trials"], ext1["c3_trials"]
    assert c3a["trials"] == c3b["trials"] == 200
    assert c3a["covered"] == c3b["covered"]
    assert c3a["mean_messages_per_trial"] == c3b["mean_messages_per_trial"]
    assert c3a["create_s"] >= 0 and c3a["s_end_to_end"] >= c3a["s_total"]
