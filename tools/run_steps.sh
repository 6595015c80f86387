#!/bin/bash
# Run GPU steps in order; a step that fails with a test failure (rc 1) lets the next run, anything
# else (fault, abort, segfault, timeout) stops the call.  Usage: run_steps.sh 'cmd1' 'cmd2' ...
mkdir -p gpurun_out
for cmd in "$@"; do
  echo "[step] $cmd"
  bash -c "$cmd"
  rc=$?
  echo "[step rc=$rc]"
  if [ $rc -gt 1 ]; then exit $rc; fi
done
