"""Per-window kernel durations (us) of the last broadcast in a rocprofv3 .db:
expand, part2, resolve (and a GS_PROBE diagnostic resolve, if any) in dispatch
order.  Usage: python scripts/perwindow.py <db> [nwin]"""
import re
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
rows = db.execute("select name, start, end from kernels order by start").fetchall()


def s(n):
    m = re.search(r"gs::(?:\(anonymous namespace\)::)?(\w+)(<\w+>)?", n)
    if not m:
        return ""
    if m.group(1) == "k_resolve" and m.group(2) and m.group(2) != "<0>":
        return "probe"
    if m.group(1) == "k_resolve_rolled" or (m.group(1) == "k_resolve_small" and m.group(2) == "<true>"):
        return "rolled"  # the rolled-node replay after k_resolve, same window
    return m.group(1)


seq = [(s(n), (e - b) / 1e3) for n, b, e in rows
       if s(n) in ("k_expand", "k_part2", "k_resolve_small", "k_resolve", "probe", "rolled")]
wins, cur = [], {}
for name, us in seq:
    if name == "rolled" and wins:
        wins[-1]["rolled"] = wins[-1].get("rolled", 0) + us
        continue
    cur[name] = cur.get(name, 0) + us
    if name == "k_resolve":
        wins.append(cur)
        cur = {}
nwin = int(sys.argv[2]) if len(sys.argv) > 2 else 40
tot = {}
for i, w in enumerate(wins[-nwin:]):
    extra = f"  probe {w['probe']:8.1f}" if "probe" in w else ""
    extra += f"  rolled {w['rolled']:6.1f}" if "rolled" in w else ""
    print(f"{i:3d} expand {w.get('k_expand', 0):8.1f}  part2 {w.get('k_part2', 0):8.1f}  "
          f"resolve {w.get('k_resolve', 0):8.1f}  small {w.get('k_resolve_small', 0):6.1f}{extra}")
    for k, v in w.items():
        tot[k] = tot.get(k, 0) + v
print("sum(ms)", {k: round(v / 1e3, 2) for k, v in tot.items()})
