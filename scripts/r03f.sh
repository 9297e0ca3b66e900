#!/bin/bash
# Round-3 GPU call F: PMC passes over one C5 broadcast at HEAD (calibrated request-size counters).
cd "$GRAFT_REPO_ROOT"
bash scripts/pmc.sh gpurun_out/r03f > gpurun_out/r03f.log 2>&1; rc=$?; tail -12 gpurun_out/r03f.log; exit $rc
