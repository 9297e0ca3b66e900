#!/bin/bash
# Per-round push-pull kernel time for each round mode at N = 1e9 (inside gpurun).
# Usage: bash scripts/ppprof.sh [modes...]   (default: topdown bottom)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
modes=${*:-topdown bottom}
for m in $modes; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/pp_$m -o run -- python3 scripts/pp_time.py 1e9 $m nofail > gpurun_out/pp_$m.log 2>&1 || exit 1
  f=$(find gpurun_out/pp_$m -name "*.db" | head -1)
  python3 scripts/pprounds.py "$f" 40 > gpurun_out/pprounds_$m.txt || exit 1
  find gpurun_out/pp_$m -name "*.db" -delete
done
