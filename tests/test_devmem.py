"""The library's device-memory cache (gs_devmem.cpp, DESIGN.md section 9;
verdict r05 item 2).

A hipMalloc right after tens of GB of hipFree waited for seconds on this
pool, so the product must not free and re-allocate large buffers in its
steady state.  Pinned here on the GPU:

* after a context's first broadcast, further broadcasts (gs_reset +
  gs_broadcast_begin + gs_run) make no device allocation at all -- neither a
  hipMalloc nor a block from the cache -- for the flood (window engine) and
  for push-pull, whose first broadcast builds the reverse table;
* a destroyed context's large blocks serve the next context of the same
  shape from the cache (no hipMalloc), and gs_trim gives them back;
* results do not depend on the cache: the same broadcast with
  GS_DEVMEM_CACHE=0 (every buffer a plain hipMalloc) gives the same counters
  and bitsets (a subprocess: the switch is read once per process).

The reference allocates its nodes once per process (simulator.go:208-212).
"""
from __future__ import annotations

import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def gs():
    import gossip_simulator_amd as mod
    mod.load()
    return mod


def allocs(gs):
    m = gs.memory_stats()
    return int(m["alloc_calls"]), int(m["alloc_cache_hits"])


@pytest.mark.parametrize("model", ["flood", "pushpull"])
def test_no_device_allocation_after_the_first_broadcast(gs, model):
    cfg = gs.Config(n=4_000_000, fanout=5, fanin=6, droprate=0.1, crashrate=0.01 if model == "flood" else 0.0,
                    seed=0x5EED, model=model)
    with gs.Simulator(cfg) as sim:
        sim.build_overlay()
        sim.broadcast_begin(-1)
        first = sim.run(poll=10)
        before = allocs(gs)
        for _ in range(3):
            sim.reset()
            sim.broadcast_begin(-1)
            again = sim.run(poll=10)
            assert np.array_equal(again[0], first[0]) and again[1] == first[1]
        assert allocs(gs) == before, f"device allocations in a later broadcast: {before} -> {allocs(gs)}"


def test_destroyed_context_blocks_serve_the_next(gs):
    cfg = gs.Config(n=8_000_000, fanout=5, fanin=6, droprate=0.1, crashrate=0.01, seed=0x5EED)
    with gs.Simulator(cfg) as sim:
        sim.build_overlay()
        sim.broadcast_begin(-1)
        a = sim.run(poll=10)
    _, hits0 = allocs(gs)
    assert gs.memory_stats()["cached_bytes"] > 0
    with gs.Simulator(cfg) as sim:
        sim.build_overlay()
        sim.broadcast_begin(-1)
        b = sim.run(poll=10)
    _, hits1 = allocs(gs)
    assert hits1 > hits0, "the second context took no block from the cache"
    assert np.array_equal(a[0], b[0]) and a[1] == b[1]
    # gs_trim hands back whole free slabs: exactly that many cached bytes go
    cached = int(gs.memory_stats()["cached_bytes"])
    released = gs.trim()
    assert released > 0
    assert int(gs.memory_stats()["cached_bytes"]) == cached - released


_CHILD = r"""
import json, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
import gossip_simulator_amd as gs
out = {}
for model in ("flood", "pushpull"):
    cfg = gs.Config(n=2_000_000, fanout=5, fanin=6, droprate=0.1, crashrate=0.01 if model == "flood" else 0.0,
                    seed=0x5EED, model=model)
    with gs.Simulator(cfg) as sim:
        sim.build_overlay()
        sim.broadcast_begin(-1)
        rows, status = sim.run(poll=10)
        out[model] = {"rows": np.asarray(rows).tolist(), "status": int(status),
                      "recv": int(np.unpackbits(sim.received().view(np.uint8)).sum())}
out["cached"] = int(gs.memory_stats()["cached_bytes"])
print("JSON" + json.dumps(out))
"""


def test_results_do_not_depend_on_the_cache():
    runs = {}
    for mode in ("1", "0"):
        env = dict(os.environ, GS_DEVMEM_CACHE=mode)
        p = subprocess.run([sys.executable, "-c", _CHILD, ROOT], capture_output=True, text=True, timeout=300, env=env)
        assert p.returncode == 0, p.stderr[-3000:]
        line = next(ln for ln in p.stdout.splitlines() if ln.startswith("JSON"))
        runs[mode] = json.loads(line[4:])
    assert runs["0"]["cached"] == 0 and runs["1"]["cached"] > 0
    for model in ("flood", "pushpull"):
        assert runs["0"][model] == runs["1"][model], model
