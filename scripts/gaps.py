"""GPU busy time vs wall span of the last broadcast in a rocprofv3 .db: the
span from the last broadcast's first k_units to its last kernel, the summed
kernel time (overlaps merged) and the idle gaps.  Usage: python gaps.py <db>"""
import re
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
rows = db.execute("select name, start, end from kernels order by start").fetchall()
# broadcasts start with the sender's k_schedule_win; take the last one
starts = [i for i, (n, _, _) in enumerate(rows) if "k_schedule" in n]
rows = rows[starts[-1]:] if starts else rows
# stop at the first kernel that is not part of the window engine (next phase)
span0, span1 = rows[0][1], rows[0][2]
busy, cur_s, cur_e, gaps = 0, rows[0][1], rows[0][2], []
for n, b, e in rows[1:]:
    if not re.search(r"gs::|hipcub|rocprim|__amd_rocclr", n):
        break
    if b > cur_e:
        busy += cur_e - cur_s
        gaps.append(b - cur_e)
        cur_s, cur_e = b, e
    else:
        cur_e = max(cur_e, e)
    span1 = max(span1, e)
busy += cur_e - cur_s
span = span1 - span0
big = sorted(gaps)[-5:]
print(f"span {span / 1e6:.3f} ms  busy {busy / 1e6:.3f} ms  idle {(span - busy) / 1e6:.3f} ms in {len(gaps)} gaps "
      f"(largest us: {[round(g / 1e3, 1) for g in big]})")
