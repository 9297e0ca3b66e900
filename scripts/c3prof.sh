#!/bin/bash
# rocprofv3 kernel trace of scripts/c3_after.py <mode> [GiB]: kernel summary + gaps
set -o pipefail
o=gpurun_out/$1; shift
mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $o/prof -o run -- python3 scripts/c3_after.py "$@" > $o/prof.log 2>&1 || { tail -20 $o/prof.log; exit 1; }
f=$(find $o/prof -name '*.db' | head -1)
python3 tools_profsummary.py "$f" 16 > $o/kernel_summary.txt
python3 - "$f" > $o/gaps.txt <<'PY'
import sqlite3, sys
rows = sqlite3.connect(sys.argv[1]).execute("select name, start, end from kernels order by start").fetchall()
gaps = sorted(((rows[i + 1][1] - rows[i][2]) / 1e6, rows[i][0][:50], rows[i + 1][0][:50]) for i in range(len(rows) - 1))
print(f"kernels {len(rows)}, span {(rows[-1][2] - rows[0][1]) / 1e6:.1f} ms, busy {sum(e - b for _, b, e in rows) / 1e6:.1f} ms")
print(f"gaps > 1 ms: {sum(g for g, _, _ in gaps if g > 1):.1f} ms in {sum(1 for g, _, _ in gaps if g > 1)}")
for g, a, b in gaps[-10:]:
    print(f"gap {g:.1f} ms after {a} before {b}")
PY
find $o/prof -name '*.db' -delete
grep "C3" $o/prof.log; head -3 $o/gaps.txt; head -8 $o/kernel_summary.txt
