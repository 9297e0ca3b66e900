"""Kernel sequence of the last broadcast in a rocprofv3 .db (from the last
k_schedule_win): one line per window-engine launch group, durations in us.
Usage: python scripts/winseq.py <db>"""
import re
import sqlite3
import sys

rows = sqlite3.connect(sys.argv[1]).execute("select name, start, end from kernels order by start").fetchall()
names = []
for n, b, e in rows:
    m = re.search(r"gs::(?:\(anonymous namespace\)::)?(\w+)", n)
    names.append((m.group(1) if m else n.split("(")[0][:30], (e - b) / 1e3, b))
last = max(i for i, x in enumerate(names) if x[0] == "k_schedule_win")
seq = names[last:]
line, out = [], []
for k, us, b in seq:
    if k == "k_units" and line:
        out.append(line)
        line = []
    line.append(f"{k[2:] if k.startswith('k_') else k}={us:.0f}")
out.append(line)
for i, l in enumerate(out):
    print(i, " ".join(l))
