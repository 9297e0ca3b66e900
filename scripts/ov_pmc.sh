#!/bin/bash
# PMC counters per dispatch of one N = 1e9 overlay build (scripts/ov_once.py):
# one kernel's launches side by side, by grid size (default the emitted
# events' k_scatter).  Usage: bash scripts/ov_pmc.sh <tag> [kernel substring] [wide]
# (wide: the instruction-mix passes instead of the L2 ones)
set -o pipefail
o=gpurun_out/$1; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ksub=${2:-OutSource}
i=0
groups=("SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU"
        "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_HIT_sum TCC_MISS_sum"
        "TCC_EA0_RDREQ_sum TCC_EA0_ATOMIC_sum TCP_TCC_WRITE_REQ_sum TCP_TCC_ATOMIC_WITH_RET_REQ_sum")
[ "${3:-}" = wide ] && groups=("SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU"
        "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
        "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum")
for grp in "${groups[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $o/p$i -o run -- python3 scripts/ov_once.py > $o/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $o/p$i.log; exit 1; }
  echo "pass $i ok"
done
python3 - $o "$ksub" > $o/kernel_pmc.txt <<'PY'
import csv, glob, sys, collections
rows = collections.defaultdict(dict)
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if sys.argv[2] not in r["Kernel_Name"]:
            continue
        key = (int(r.get("Grid_Size", 0) or 0))
        rows[key][r["Counter_Name"]] = rows[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
for g in sorted(rows, key=lambda k: -k)[:16]:
    print(g, {k: f"{v:.4g}" for k, v in sorted(rows[g].items())})
PY
rm -rf $o/p[0-9]*/
cat $o/kernel_pmc.txt | head -20
