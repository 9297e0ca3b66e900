#!/bin/bash
# Round-3 GPU call O: evidence pass at HEAD after the packed rows and one-draw drop/crash
# (every GPU test, smoke, the default bench line, a kernel trace of the bench).
cd "$GRAFT_REPO_ROOT"
bash scripts/round.sh r03s
