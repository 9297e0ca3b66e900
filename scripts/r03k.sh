#!/bin/bash
# Round-3 GPU call K: evidence pass at HEAD (every GPU test, smoke, the default
# bench line, a kernel trace).
cd "$GRAFT_REPO_ROOT"
bash scripts/round.sh r03k
