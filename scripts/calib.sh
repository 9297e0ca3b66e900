#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration (MI355X_MICROARCH.md HBM section): the
# known-byte micro kernels of scripts/micro/fetch_calib.hip under one
# rocprofv3 pass per counter group, then the per-pattern byte factors.
# Usage (inside gpurun): bash scripts/calib.sh <outdir>
set -u
out=${1:-gpurun_out/calib}
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bin=scripts/micro/fetch_calib
timeout -k 10 60 $bin > "$out/plain.txt" 2>&1 || { echo "calib binary failed"; tail -5 "$out/plain.txt"; exit 1; }
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
  "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" \
  "TCC_EA0_RDREQ_DRAM_32B_sum TCC_BUBBLE_sum" \
  "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_WRITE_DRAM_32B_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d "$out/p$i" -o run -- $bin > "$out/p$i.log" 2>&1 || { echo "pass $i ($grp) failed"; tail -5 "$out/p$i.log"; exit 1; }
  echo "pass $i ok: $grp"
done
python3 scripts/pmc_summary.py "$out" > "$out/summary.csv" && rm -rf "$out"/p[0-9]*/
python3 scripts/calib_summary.py "$out/plain.txt" "$out/summary.csv" > "$out/calibration.json"
cat "$out/calibration.json"
