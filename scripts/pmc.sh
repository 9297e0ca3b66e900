#!/bin/bash
# PMC passes over one N=1e9 broadcast (bench.py --steps 1 --warmup 0), one
# rocprofv3 run per counter group (rocprofv3 does not split passes itself).
# Usage: scripts/pmc.sh <outdir> [extra bench args]
set -u
out=${1:-gpurun_out/pmc}; shift || true
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
args="--steps 1 --warmup 0 --no-roofline --no-extensions --cpu-n 0 $*"  # no extensions: the C3 host threads crash the profiler
i=0
for grp in \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES" \
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
  "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
  "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" \
  "TCC_EA0_RDREQ_DRAM_32B_sum TCC_BUBBLE_sum" \
  "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_WRITE_DRAM_32B_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$out/p$i" -o run -- python3 bench.py $args > "$out/p$i.log" 2>&1 || { echo "pass $i ($grp) failed rc=$?"; tail -5 "$out/p$i.log"; exit 1; }
  echo "pass $i ok: $grp"
done
python3 scripts/pmc_summary.py "$out" > "$out/summary.csv" && rm -rf "$out"/p[0-9]*/ && python3 scripts/pmc_traffic.py "$out/summary.csv" "$out/pmc_traffic.json" $i ${PMC_WINDOWS:-28} > /dev/null  # 28: the C5 broadcast's windows (gs_timing.windows)
