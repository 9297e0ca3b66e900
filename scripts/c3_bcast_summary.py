"""Kernel totals of the last broadcast in a rocprofv3 .db of scripts/c3_bcast.py:
everything after the last host gap > 20 ms (the sleep before it).
Usage: python scripts/c3_bcast_summary.py <db>"""
import re
import sqlite3
import sys
from collections import defaultdict

rows = sqlite3.connect(sys.argv[1]).execute("select name, start, end from kernels order by start").fetchall()
cut = max(i for i in range(1, len(rows)) if rows[i][1] - rows[i - 1][2] > 20e6)
rows = rows[cut:]
tot, cnt = defaultdict(float), defaultdict(int)
for n, b, e in rows:
    m = re.search(r"(\w+)(<[^(]*>)?\(", n)
    k = m.group(1) if m else n[:40]
    tot[k] += (e - b) / 1e6
    cnt[k] += 1
span = (rows[-1][2] - rows[0][1]) / 1e6
busy = sum(tot.values())
print(f"last broadcast: {len(rows)} kernels, span {span:.2f} ms, kernel busy {busy:.2f} ms")
for k, v in sorted(tot.items(), key=lambda x: -x[1])[:20]:
    print(f"{k:40s} {cnt[k]:6d} {v:9.3f} ms")
