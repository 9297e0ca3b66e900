"""Push-pull node-range shards at N = 1e9 on one GPU: bench.py's
c5_pushpull_sharded leg alone (8 in-process shards; the replica's early
rounds, then sharded bottom-up rounds), one JSON line.
Usage: python scripts/pp_shard_probe.py [shards]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import gossip_simulator_amd as gs  # noqa: E402

import torch  # noqa: E402

torch.cuda.synchronize()  # the HIP runtime is up before the library's first call
G = int(sys.argv[1]) if len(sys.argv) > 1 else 8
a = argparse.Namespace(n=1_000_000_000, fanout=5, fanin=6, delaylow=10, delayhigh=20, droprate=0.1,
                       seed=0x5EED, steps=8, pp_shards=G)
gs.load()
print(json.dumps(bench.pushpull_sharded(a, gs, 0, 1, 0, None)), flush=True)
