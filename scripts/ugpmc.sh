#!/bin/bash
# uncached_gather timings per allocation mode, then the L2 -> memory read
# request sizes of one run per mode (rocprofv3 --pmc).  Usage: bash scripts/ugpmc.sh <tag>
set -o pipefail
o=gpurun_out/$1; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
hipcc -O3 --offload-arch=gfx950 -o $o/ug scripts/micro/uncached_gather.hip || exit 1
for m in coarse; do
  timeout -k 10 120 $o/ug 25.6 $m 64 || exit 1
done
for m in coarse; do
  timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum \
    --output-format csv -d $o/pmc_$m -o run -- $o/ug 25.6 $m 64 > $o/pmc_$m.log 2>&1 || { tail -5 $o/pmc_$m.log; exit 1; }
  f=$(find $o/pmc_$m -name '*counter_collection.csv' | head -1)
  echo "== $m"; python3 - "$f" <<'PY'
import csv, sys, collections
tot = collections.defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    if "k_gather" in r.get("Kernel_Name", ""):
        tot[r["Counter_Name"]] += float(r["Counter_Value"])
print({k: f"{v:.4g}" for k, v in sorted(tot.items())})
PY
done
