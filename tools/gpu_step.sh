#!/bin/bash
# Run GPU steps in order; each under its own time limit; stop after a fault / abort / timeout
# (exit codes other than 0 and 1: 124/137 time limit, 134 abort, 139 segfault, ...).
# usage: tools/gpu_step.sh "<seconds> <log> <command...>" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
for spec in "$@"; do
  secs=${spec%% *}; rest=${spec#* }; log=${rest%% *}; cmd=${rest#* }
  echo "=== [$(date +%T)] $cmd (limit ${secs}s) -> gpurun_out/$log"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$log" 2>&1
  rc=$?
  echo "=== rc=$rc"
  tail -3 "gpurun_out/$log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: rc=$rc"; exit $rc; fi
done
