#!/bin/bash
# Host wait mode A/B (how HIP waits for the device: ROC_ACTIVE_WAIT_TIMEOUT, hipSetDeviceFlags through
# SR_AMD_SCHED): the tree-sharding share + C2 (tools/share_probe.py) and the C3 / C5 searches
# (tools/search_ab.py), alternating, two passes.  Tag $1.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05w}
mkdir -p gpurun_out
OUT=gpurun_out/${TAG}_wait_ab.jsonl
: > $OUT
for pass in 1 2; do
  for v in "X=0" "ROC_ACTIVE_WAIT_TIMEOUT=100" "ROC_ACTIVE_WAIT_TIMEOUT=5000" "SR_AMD_SCHED=spin" "SR_AMD_SCHED=yield"; do
    echo "{\"variant\": \"$v\", \"pass\": $pass}" >> $OUT
    env $v timeout -k 10 240 python3 -u tools/share_probe.py >> $OUT 2>> gpurun_out/${TAG}_wait_ab.err || exit $?
    env $v ITERS=30 timeout -k 10 300 python3 -u tools/search_ab.py C3 C5 >> $OUT 2>> gpurun_out/${TAG}_wait_ab.err || exit $?
  done
done
