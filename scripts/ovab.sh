#!/bin/bash
# overlay build A/B: kernel sums of one N=1e9 build per variant, interleaved
set -o pipefail
o=gpurun_out/$1; shift; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for rep in 1 2; do
  for v in "$@"; do
    tag=$(echo "$v" | tr '=, /' '____' | tail -c 40)
    timeout -k 10 240 env $v rocprofv3 --kernel-trace -d $o/p_$tag -o run -- python3 scripts/ov_once.py > $o/l_$tag.log 2>&1 || { tail -5 $o/l_$tag.log; exit 1; }
    f=$(find $o/p_$tag -name '*.db' | head -1)
    python3 scripts/ov_ticks.py $f > $o/t_${rep}_$tag.txt
    echo "$rep [$v] $(tail -1 $o/t_${rep}_$tag.txt)"
    rm -rf $o/p_$tag
  done
done
