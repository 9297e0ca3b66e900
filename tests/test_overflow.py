"""Receipt-count overflow: a node that gets more than 65535 messages in one
tick overflows the 16-bit receipt count the tick engine and the CPU
restatements pack (receipts | crash rolls << 16).  Every engine that packs it
must refuse such a run (GS_EOVERFLOW / OverflowError) instead of mixing the
receipt count into the roll count.  The reference's counts are unbounded
(one channel receive per message, simulator.go:107-123); its channels hold
1024 messages (:51-54), so such a hub would block senders there instead.

The table is an injected star: the sender (node 0) lists 255 relays; each
relay lists 255 leaves; each leaf lists the hub T twice (duplicates are
separate sends, simulator.go:97-101, 143-147).  With a constant 10-ms delay
every leaf fires at tick 30, so T gets ~2 x 65025 messages in one tick.
"""
from __future__ import annotations

import numpy as np
import pytest

RELAYS, FAN = 255, 255


def star_table():
    leaves0 = 1 + RELAYS
    nleaves = RELAYS * FAN
    hub = leaves0 + nleaves
    n = hub + 1
    stride = FAN
    deg = np.zeros(n, dtype=np.uint8)
    ids = np.zeros((n, stride), dtype=np.uint32)
    deg[0] = RELAYS
    ids[0, :RELAYS] = np.arange(1, 1 + RELAYS)
    for r in range(RELAYS):
        deg[1 + r] = FAN
        ids[1 + r, :FAN] = leaves0 + r * FAN + np.arange(FAN)
    deg[leaves0:hub] = 2
    ids[leaves0:hub, 0] = hub
    ids[leaves0:hub, 1] = hub
    deg[hub] = 1
    ids[hub, 0] = 0
    return n, deg, ids


KW = dict(fanout=FAN, fanin=FAN, delay_low=10, delay_high=11, drop_rate=0.0, crash_rate=0.01,
          seed=0x5EED, trial=0)


def test_oracles_refuse_receipt_overflow(oracle):
    n, deg, ids = star_table()
    p = oracle.make_params(n=n, **KW)
    e = oracle.Engine(p, deg, ids)
    e.begin(0)
    e.step(29)  # relays and leaves informed; nothing has reached the hub yet
    with pytest.raises(OverflowError):
        e.step(1)
    o = oracle.OmpEngine(p, deg, ids, threads=4)
    o.begin(0)
    o.step(29)
    with pytest.raises(OverflowError):
        o.step(1)


def test_oracle_counts_below_the_limit(oracle):
    """The same star with one copy of the hub per leaf: 65025 < 65536 receipts
    (minus crashed leaves) is in range, and every receipt is accounted for."""
    n, deg, ids = star_table()
    deg[1 + RELAYS:n - 1] = 1
    p = oracle.make_params(n=n, **KW)
    e = oracle.Engine(p, deg, ids)
    e.begin(0)
    rows = e.step(31)
    assert int(rows[29, 2]) > 60_000  # tick 30: the leaves' sends to the hub


@pytest.mark.gpu
def test_tick_engine_returns_overflow():
    import gossip_simulator_amd as gs
    n, deg, ids = star_table()
    cfg = gs.Config(n=n, fanout=FAN, fanin=FAN, delaylow=10, delayhigh=11, droprate=0.0,
                    crashrate=0.01, seed=0x5EED, engine="tick")
    with gs.Simulator(cfg) as sim:
        sim.load_peers(deg, ids)
        sim.broadcast_begin(0)
        sim.step(29)
        with pytest.raises(gs.GossipError) as ei:
            sim.step(1)
        assert ei.value.code == -6  # GS_EOVERFLOW
        # the context stays usable: a reset clears the overflow, and a second
        # broadcast that stops before the hub's tick runs clean
        sim.reset()
        sim.broadcast_begin(0)
        rows = sim.step(29)
        assert int(rows[-1][0]) == 29 and int(rows[:, 2].sum()) > 0


def star32_table(copies=4):
    """The same hub overflow within the window engine's 32-slot rows: three
    levels of 32 relays (32768 leaves), each leaf lists the hub `copies`
    times.  With crashrate 0.01 the hub holds about 1300 crash-roll receipts,
    so k_resolve takes its per-node 16-bit counters (the rolled list holds
    1024) and ~127000 receipts overflow them at tick 40."""
    L1, L2, L3 = 32, 32 * 32, 32 * 32 * 32
    n = 1 + L1 + L2 + L3 + 1
    hub = n - 1
    deg = np.zeros(n, dtype=np.uint8)
    ids = np.zeros((n, 32), dtype=np.uint32)
    deg[0] = 32
    ids[0] = 1 + np.arange(32)
    lv1, lv2, lv3 = 1, 1 + L1, 1 + L1 + L2
    for i in range(L1):
        deg[lv1 + i] = 32
        ids[lv1 + i] = lv2 + i * 32 + np.arange(32)
    for i in range(L2):
        deg[lv2 + i] = 32
        ids[lv2 + i] = lv3 + i * 32 + np.arange(32)
    deg[lv3:hub] = copies
    ids[lv3:hub, :copies] = hub
    deg[hub] = 1
    ids[hub, 0] = 0
    return n, deg, ids


@pytest.mark.gpu
@pytest.mark.parametrize("G", [0, 2])
def test_window_engine_returns_overflow(G):
    """The window engine (unsharded, device-driven) and in-process shards
    return GS_EOVERFLOW for the 32-slot star."""
    import gossip_simulator_amd as gs
    n, deg, ids = star32_table()
    cfg = gs.Config(n=n, fanout=32, fanin=32, delaylow=10, delayhigh=11, droprate=0.0, crashrate=0.01,
                    seed=0x5EED)
    with (gs.Simulator(cfg, devices=[0] * G) if G else gs.Simulator(cfg)) as sim:
        sim.load_peers(deg, ids)
        sim.broadcast_begin(0)
        with pytest.raises(gs.GossipError) as ei:
            sim.step(45)
        assert ei.value.code == -6  # GS_EOVERFLOW

