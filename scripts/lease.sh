#!/bin/bash
# One evidence pass inside a gpurun call, in the order given; every GPU step
# runs under its own time limit and the pass stops at the first failure.
# Outputs under gpurun_out/<tag>/.
# Usage: bash scripts/lease.sh <tag> <step> [<step> ...]
#   tests[=pytest args]  the -m gpu suite (or the given targets), scripts/gtest.sh
#   smoke                __graft_entry__.smoke()
#   bench[=bench args]   bench.py (default args), the JSON line in bench.json
#   pw                   rocprofv3 kernel trace of one broadcast: per-window split (scripts/pw.sh)
#   prof[=bench args]    rocprofv3 kernel trace of a short bench (scripts/prof.sh)
#   pmc                  PMC passes over one broadcast (scripts/pmc.sh)
#   pmcpp                PMC passes over one C5 push-pull broadcast (scripts/pmc_pp.sh)
#   pool                 the stream-ordered pool reproducer in its diagnosis modes (scripts/micro/pool_repro.hip)
#   ab=ENV_A,ENV_B,...   interleaved A/B/... benches (scripts/abn.sh)
set -o pipefail
tag=${1:?tag}; shift
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/$tag; mkdir -p "$o"
for step in "$@"; do
  name=${step%%=*}; arg=""; [ "$name" != "$step" ] && arg=${step#*=}
  echo "[lease] $tag: $name $arg"
  case $name in
    tests)
      # shellcheck disable=SC2086
      bash scripts/gtest.sh 900 $arg > /dev/null || { tail -30 gpurun_out/gtest.log; exit 1; }
      cp gpurun_out/gtest.log "$o/tests.log"; tail -1 "$o/tests.log" ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$o/smoke.log" 2>&1 \
        || { tail -20 "$o/smoke.log"; exit 1; }
      tail -1 "$o/smoke.log" ;;
    bench)
      # shellcheck disable=SC2086
      timeout -k 10 900 python -u bench.py $arg > "$o/bench.json" 2> "$o/bench.err" || { tail -20 "$o/bench.err"; exit 1; }
      cut -c1-400 "$o/bench.json"; grep "\[bench\]" "$o/bench.err" ;;
    pw)
      bash scripts/pw.sh "$tag/pw" > /dev/null || exit 1
      tail -1 "$o/pw/perwindow.txt"; head -14 "$o/pw/kernel_summary.txt" ;;
    prof)
      # shellcheck disable=SC2086
      bash scripts/prof.sh "$tag/prof" $arg || exit 1 ;;
    pmc)
      bash scripts/pmc.sh "$o/pmc" || exit 1 ;;
    pmcpp)
      bash scripts/pmc_pp.sh "$o/pmc_pp" 1e9 0 || exit 1 ;;
    pool)
      hipcc -O2 --offload-arch=gfx950 -o "$o/pool_repro" scripts/micro/pool_repro.hip || exit 1
      for args in "5 6 pool memcpy nosync" "5 6 pool memcpy sync" "5 6 pool kcopy nosync" "5 6 pool kcopy sync" \
                  "5 6 malloc memcpy nosync" "5 6 malloc memcpy sync" "5 6 malloc kcopy nosync" \
                  "5 6 malloc kcopy sync" "1 6 pool memcpy nosync"; do
        echo "== pool_repro $args"
        # shellcheck disable=SC2086
        timeout -k 10 180 "$o/pool_repro" $args; rc=$?
        [ $rc -le 1 ] || { echo "pool_repro rc=$rc"; exit 1; }
      done > "$o/pool_repro.txt" 2>&1
      grep -E "^==|REPRODUCED|no mismatch" "$o/pool_repro.txt" ;;
    ab)
      IFS=',' read -r -a envs <<< "$arg"
      bash scripts/abn.sh "${envs[@]}" || exit 1 ;;
    *) echo "[lease] unknown step $name"; exit 2 ;;
  esac
done
