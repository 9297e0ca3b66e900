"""Per-round push-pull kernel time (us) of the last N rounds in a rocprofv3
.db: rounds start at k_pp_mode; each row sums the round's kernels
(dense: summaries + k_pp_round + k_pp_commit; early: k_ppe_round +
k_ppe_commit).  Usage: python scripts/pprounds.py <db> [nrounds]"""
import re
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
rows = db.execute("select name, start, end from kernels order by start").fetchall()
rounds, cur = [], None
for n, b, e in rows:
    m = re.search(r"gs::(?:\(anonymous namespace\)::)?(\w+)", n)
    k = m.group(1) if m else ""
    if k == "k_pp_mode":
        if cur:
            rounds.append(cur)
        cur = {"t0": b, "t1": e}
        continue
    if cur is None or not k.startswith("k_pp") and not k.startswith("k_ppe"):
        continue
    cur[k] = cur.get(k, 0) + (e - b) / 1e3
    cur["t1"] = e
if cur:
    rounds.append(cur)
nr = int(sys.argv[2]) if len(sys.argv) > 2 else 40
tot = 0.0
for i, r in enumerate(rounds[-nr:]):
    span = (r["t1"] - r["t0"]) / 1e3
    tot += span
    parts = " ".join(f"{k[2:]}={v:.0f}" for k, v in r.items() if k not in ("t0", "t1") and v >= 1)
    print(f"{i:3d} span {span:8.1f}  {parts}")
print(f"total span {tot / 1e3:.1f} ms over {min(nr, len(rounds))} rounds")
