#!/bin/bash
# GPU suite, then the search A/B: host-side partial reduction off / on, alternating, two passes each.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05e}
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gpu_suite.log 2>&1 || exit $?
OUT=gpurun_out/${TAG}_search_ab.jsonl
: > $OUT
for pass in 1 2; do
  for hr in 0 1; do
    SR_AMD_HOST_REDUCE=$hr timeout -k 10 300 python3 tools/search_ab.py C3 C5 share >> $OUT 2>> gpurun_out/${TAG}_search_ab.err || exit $?
  done
done
timeout -k 10 300 python3 tools/share_probe.py > gpurun_out/${TAG}_share_probe.jsonl 2> gpurun_out/${TAG}_share_probe.err || exit $?
