#!/bin/bash
# Round-3 GPU call M: kernel trace of the headline workload alone (C5 flood,
# N = 1e9, bench.py --steps 2 --warmup 1, no extensions).
cd "$GRAFT_REPO_ROOT"
bash scripts/prof.sh r03m
