#!/bin/bash
# PMC passes over ONE C5 push-pull broadcast (scripts/pp_once.py), one
# rocprofv3 run per counter group; then the per-round-kernel traffic
# (scripts/pmc_pp_traffic.py).  Usage: scripts/pmc_pp.sh <outdir> [n] [failed_fraction]
set -u
out=${1:-gpurun_out/pmc_pp}; n=${2:-1e9}; frac=${3:-0}
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
i=0
for grp in \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES" \
  "FETCH_SIZE" "WRITE_SIZE" \
  "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d "$out/p$i" -o run -- python3 scripts/pp_once.py "$n" "$frac" > "$out/p$i.log" 2>&1 || { echo "pass $i ($grp) failed rc=$?"; tail -5 "$out/p$i.log"; exit 1; }
  echo "pass $i ok: $grp"; tail -1 "$out/p$i.log"
done
python3 scripts/pmc_summary.py "$out" > "$out/summary.csv" && rm -rf "$out"/p[0-9]*/ && python3 scripts/pmc_pp_traffic.py "$out/summary.csv" "$out/pmc_pp_traffic.json" "$out/p1.log"
