#!/bin/bash
# GPU suite, then the exact-sum pass tree list read from pinned memory (default) vs uploaded first
# (SR_AMD_EXACT_LIST_HOST=0) on C2 and the tree-sharding share (tools/share_probe.py), three alternating passes.  Tag $1.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05q}
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gpu_suite.log 2>&1 || exit $?
OUT=gpurun_out/${TAG}_ab.jsonl
: > $OUT
for pass in 1 2 3; do
  for v in "X=0" "SR_AMD_EXACT_LIST_HOST=0"; do
    echo "{\"variant\": \"$v\", \"pass\": $pass}" >> $OUT
    env $v timeout -k 10 240 python3 -u tools/share_probe.py >> $OUT 2>> gpurun_out/${TAG}_ab.err || exit $?
  done
done
