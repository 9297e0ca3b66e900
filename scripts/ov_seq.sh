#!/bin/bash
# rocprofv3 kernel trace of one N = 1e9 overlay build (scripts/ov_once.py):
# the kernel sequence of its densest ticks with durations and grid sizes.
# Usage: bash scripts/ov_seq.sh <tag>
set -o pipefail
o=gpurun_out/$1; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 rocprofv3 --kernel-trace -d $o/prof -o run -- python3 scripts/ov_once.py > $o/prof.log 2>&1 || { tail -20 $o/prof.log; exit 1; }
f=$(find $o/prof -name '*.db' | head -1)
python3 - "$f" > $o/ov_seq.txt <<'PY'
import re, sqlite3, sys
db = sqlite3.connect(sys.argv[1])
cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
g = [c for c in cols if "grid" in c.lower()]
sel = "name, start, end" + (", " + ", ".join(g) if g else "")
rows = db.execute(f"select {sel} from kernels order by start").fetchall()
print("columns:", sel)
for r in rows[:400]:
    m = re.search(r"(\w+)(<[^(]*>)?\(", r[0])
    nm = (m.group(1) + (m.group(2) or "")) if m else r[0][:50]
    print(f"{(r[2] - r[1]) / 1e3:9.1f} us  {nm[:60]:60s} {r[3:]}")
PY
find $o/prof -name '*.db' -delete
head -5 $o/ov_seq.txt
