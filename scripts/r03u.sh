#!/bin/bash
# Round-3 GPU call O: evidence pass at HEAD final pass of the session
# (every GPU test, smoke, the default bench line, a kernel trace of the bench).
cd "$GRAFT_REPO_ROOT"
bash scripts/round.sh r03u
