#!/bin/bash
# Runs GPU steps in order, each under its own time limit.  A step that ends by a signal,
# a time limit or a crash (exit >= 124) stops the sequence: nothing more touches the GPU.
# Usage: scripts/gpu_steps.sh "<limit> <name> <command...>" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for spec in "$@"; do
  limit=${spec%% *}; rest=${spec#* }; name=${rest%% *}; cmd=${rest#* }
  echo "=== [$name] (limit ${limit}s): $cmd"
  timeout -k 10 "$limit" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc"
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ge 124 ]; then echo "=== stopping: $name ended with $rc"; exit $rc; fi
done
exit 0
