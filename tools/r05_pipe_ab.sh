#!/bin/bash
# GPU suite, then the search A/B: the lanes' pipeline (SR_AMD_SEARCH_PIPELINE) off / on, alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05i}
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gpu_suite.log 2>&1 || exit $?
OUT=gpurun_out/${TAG}_search_ab.jsonl
: > $OUT
for pass in 1 2; do
  for pp in 0 1; do
    SR_AMD_SEARCH_PIPELINE=$pp timeout -k 10 300 python3 tools/search_ab.py C1 C3 C5 share >> $OUT 2>> gpurun_out/${TAG}_search_ab.err || exit $?
  done
done
