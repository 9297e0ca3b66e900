"""Per-tick split of the LAST overlay build in a rocprofv3 kernel-trace .db:
a tick is everything from one k_process to the next (the sort and select
before it belong to it).  Prints per tick the summed kernel time by kernel
family and the span, then totals.  Usage: python scripts/ov_ticks.py <db>"""
import re
import sqlite3
import sys
from collections import defaultdict

db = sqlite3.connect(sys.argv[1])
rows = db.execute("select name, start, end from kernels order by start").fetchall()


def fam(n):
    if "k_ov_part" in n:
        return "part1" if "false" in n.lower() or "Lb0" in n else "part2"
    if "k_ov_fine" in n:
        return "fine"
    if "k_process" in n:
        return "process"
    if "k_scatter" in n:
        return "scatter"
    if "Select" in n or "select" in n:
        return "select"
    if "rocprim" in n or "hipcub" in n or "radix" in n.lower() or "onesweep" in n:
        return "sort"
    return "other"


# the last build starts at the last scatter that precedes the first k_process
# of a run of k_process launches: take every kernel after the second-to-last
# PickSource scatter pair (count + write of tick 0)
picks = [i for i, (n, _, _) in enumerate(rows) if "PickSource" in n]
start = picks[-2] if len(picks) >= 2 else 0
rows = rows[start:]
# host-side stalls: the largest idle gaps between consecutive kernels
gaps = sorted(((rows[i + 1][1] - rows[i][2]) / 1e6, rows[i][0][:60], rows[i + 1][0][:60]) for i in range(len(rows) - 1))[-8:]
for g, a, b in gaps:
    print(f"gap {g:.2f} ms after {a} before {b}")
ticks, cur = [], defaultdict(float)
span0 = rows[0][1]
for n, b, e in rows:
    f = fam(n)
    cur[f] += (e - b) / 1e6
    if f == "scatter" and "true" in n.lower() and cur.get("process"):
        ticks.append(cur)
        cur = defaultdict(float)
if cur:
    ticks.append(cur)
tot = defaultdict(float)
for i, t in enumerate(ticks):
    for k, v in t.items():
        tot[k] += v
    if i < 25 or sum(t.values()) > 5:
        print(f"tick-group {i}: " + "  ".join(f"{k} {v:.2f}" for k, v in sorted(t.items())) + f"  sum {sum(t.values()):.2f} ms")
print(f"{len(ticks)} groups; span {(rows[-1][2] - span0) / 1e6:.1f} ms; kernel totals: " +
      "  ".join(f"{k} {v:.1f}" for k, v in sorted(tot.items())) + f"  sum {sum(tot.values()):.1f} ms")
