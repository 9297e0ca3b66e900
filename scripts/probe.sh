#!/bin/bash
# k_resolve phase probes: one rocprof run per GS_PROBE level (1..4), one broadcast each.
set -o pipefail
o=gpurun_out/probe; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for p in 1 2 3 4; do
  GS_PROBE=$p timeout -k 10 200 rocprofv3 --kernel-trace -d $o/p$p -o run -- python3 bench.py --steps 1 --warmup 0 --cpu-n 0 --no-roofline > $o/p$p.log 2>&1 || { tail -5 $o/p$p.log; exit 1; }
  f=$(find $o/p$p -name '*.db' | head -1)
  python3 scripts/perwindow.py "$f" 40 > $o/probe$p.txt; rm -rf $o/p$p
  echo "probe $p: $(tail -1 $o/probe$p.txt)"
done
