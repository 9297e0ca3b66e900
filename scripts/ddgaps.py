"""The last broadcast of a rocprofv3 kernel-trace .db (from its k_schedule_win
on, or from the last kernel named <mark>): kernel time by kernel, the idle
time before each kernel by kernel (the gap a launch waited for), span and
busy time.  Usage: python ddgaps.py <db> [mark]"""
import re
import sqlite3
import sys
from collections import defaultdict

db = sqlite3.connect(sys.argv[1])
rows = db.execute("select name, start, end from kernels order by start").fetchall()
mark = sys.argv[2] if len(sys.argv) > 2 else "k_schedule"  # the kernel that starts a broadcast
starts = [i for i, (n, _, _) in enumerate(rows) if mark in n]
rows = rows[starts[-1]:] if starts else rows


def short(n):
    m = re.search(r"gs::(?:\(anonymous namespace\)::)?(\w+)", n)
    return m.group(1) if m else n.split("(")[0][-40:]


busy = defaultdict(float)
cnt = defaultdict(int)
gap = defaultdict(float)
last_end = rows[0][1]
for n, b, e in rows:
    if not re.search(r"gs::|hipcub|rocprim|__amd_rocclr", n):
        break
    k = short(n)
    busy[k] += (e - b) / 1e3
    cnt[k] += 1
    if b > last_end:
        gap[k] += (b - last_end) / 1e3
    last_end = max(last_end, e)
span = (last_end - rows[0][1]) / 1e3
tb, tg = sum(busy.values()), sum(gap.values())
print(f"span {span:.1f} us  kernels {tb:.1f} us  idle {tg:.1f} us")
print(f"{'kernel':28s} {'calls':>6s} {'busy us':>10s} {'idle before us':>15s}")
for k in sorted(busy, key=lambda k: -(busy[k] + gap[k])):
    print(f"{k:28s} {cnt[k]:6d} {busy[k]:10.1f} {gap[k]:15.1f}")
