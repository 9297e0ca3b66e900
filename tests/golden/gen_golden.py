"""Generates the committed golden fixtures under tests/golden/ from the CPU
restatement (oracle/gsoracle.c).

The reference (simulator.go) has no tests or fixtures and cannot be run here
(no Go toolchain), so these vectors pin the tick-model specification itself:
they freeze the oracle's outputs so that (a) the oracle cannot drift silently
and (b) the HIP engine is checked against the same data on the GPU box, where
/root/reference does not exist.

Run from the repo root:  python tests/golden/gen_golden.py
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import pyoracle as O  # noqa: E402

CASES = {
    # name: params, plus the sender (-1 = keyed pick) and max ticks
    "a_n100_tick": dict(n=100, fanout=3, fanin=4, delay_low=1, delay_high=4,
                        drop_rate=0.1, crash_rate=0.05, seed=7, trial=0),
    "b_n1000_default": dict(n=1000, fanout=5, fanin=6, delay_low=10, delay_high=20,
                            drop_rate=0.1, crash_rate=0.001, seed=0x5EED, trial=0),
    "c_n4133_hop": dict(n=4133, fanout=3, fanin=6, delay_low=10, delay_high=11,
                        drop_rate=0.2, crash_rate=0.02, seed=3, trial=5),
    "d_n10000_crash": dict(n=10000, fanout=5, fanin=6, delay_low=10, delay_high=20,
                           drop_rate=0.1, crash_rate=0.01, seed=0x5EED, trial=1),
}


def sha(words: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(words, dtype="<u8").tobytes()).hexdigest()


def masked(deg, ids):
    m = np.arange(ids.shape[1])[None, :] < deg[:, None]
    return np.where(m, ids, 0).astype(np.uint32)


def run_case(kw):
    p = O.make_params(**kw)
    deg, ids, wins, final = O.overlay(p)
    e = O.Engine(p, deg, ids)
    e.begin(-1)
    ticks = []
    while True:
        s = e.step(1)[0]
        ticks.append({"stats": [int(x) for x in s], "received_sha256": sha(e.received())})
        if O.covered(int(s[4]), p.n) or int(s[6]) == 0 or len(ticks) >= 5000:
            break
    return deg, masked(deg, ids), wins, final, ticks, sha(e.crashed()), O.pick_sender(p)


def main():
    index = {}
    for name, kw in CASES.items():
        deg, ids, wins, final, ticks, crash_sha, sender = run_case(kw)
        np.savez_compressed(os.path.join(HERE, f"{name}_peers.npz"), deg=deg, ids=ids)
        doc = {"params": kw, "sender": sender, "overlay_windows": wins,
               "overlay_final_tick": final, "ticks": ticks, "crashed_sha256_final": crash_sha,
               "stat_fields": list(O.STAT_FIELDS)}
        with open(os.path.join(HERE, f"{name}.json"), "w") as f:
            json.dump(doc, f, indent=0)
        index[name] = {"ticks": len(ticks), "final": ticks[-1]["stats"]}
        print(name, index[name])
    with open(os.path.join(HERE, "index.json"), "w") as f:
        json.dump(index, f, indent=1)


if __name__ == "__main__":
    main()
