#!/bin/bash
# Runs "name|seconds|command" steps in order inside one gpurun call, each under
# its own time limit; a step that fails is reported and the next one runs,
# but a step ending in a timeout, abort or crash (124, 137, 134, 139) stops
# the call (nothing more touches the GPU after a possible fault).
# Output of step <name> in gpurun_out/<tag>/<name>.log.
# Usage: bash scripts/steps.sh <tag> "name|seconds|command" ...
tag=${1:?tag}; shift
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/$tag; mkdir -p "$o"
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}; secs=${rest%%|*}; cmd=${rest#*|}
  echo "[steps] $name ($secs s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "$o/$name.log" 2>&1
  rc=$?
  echo "[steps] $name rc=$rc"; tail -4 "$o/$name.log"
  case $rc in 124|137|134|139) echo "[steps] stopping after $name"; exit $rc ;; esac
done
