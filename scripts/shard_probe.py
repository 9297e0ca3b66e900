"""In-process shard scaling probe: bench.py's shards_inproc leg alone (C4 G =
1/2/4/8 and C5's flood at G = 8), printing one JSON line."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import gossip_simulator_amd as gs  # noqa: E402

a = argparse.Namespace(n=1_000_000_000, fanout=5, fanin=6, crashrate=0.01, droprate=0.1, seed=0x5EED)
gs.load()
print(json.dumps(bench.shards_inproc(a, gs)), flush=True)
