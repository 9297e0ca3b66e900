#!/bin/bash
# rocprofv3 kernel trace of one C5 flood broadcast: per-window split + kernel summary.
# Usage (inside gpurun): bash scripts/pw.sh <tag>
set -o pipefail
o=gpurun_out/${1:-pw}; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prof -o run -- python3 bench.py --steps 1 --warmup 1 --cpu-n 0 --no-roofline --no-extensions --no-c3 --no-c4 > $o/prof.log 2>&1 || { tail -20 $o/prof.log; exit 1; }
f=$(find $o/prof -name '*.db' | head -1)
python3 tools_profsummary.py "$f" 14 > $o/kernel_summary.txt && python3 scripts/perwindow.py "$f" 28 > $o/perwindow.txt && python3 scripts/ov_ticks.py "$f" > $o/ov_ticks.txt
python3 - "$f" > $o/sequence.txt <<'PY'
import re, sqlite3, sys
rows = sqlite3.connect(sys.argv[1]).execute("select name, start, end from kernels order by start").fetchall()
i0 = max(i for i, r in enumerate(rows) if "k_schedule_win" in r[0])  # the last broadcast's begin
for n, b, e in rows[i0:i0 + 400]:
    m = re.search(r"(\w+)(<[^(]*>)?\(", n)
    print(f"{(e - b) / 1e3:9.1f} {(m.group(1) + (m.group(2) or '')) if m else n[:60]}")
PY
find $o/prof -name '*.db' -delete
tail -12 $o/perwindow.txt; head -16 $o/kernel_summary.txt
