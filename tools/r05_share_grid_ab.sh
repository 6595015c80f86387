#!/bin/bash
# Tree-sharding share vs C2 (tools/share_probe.py) under grid variants: trees per workgroup (SR_AMD_TREES_PER_BLOCK)
# and row blocks (SR_AMD_MAX_ROW_BLOCKS), two alternating passes.  Tag $1.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05x2}
mkdir -p gpurun_out
OUT=gpurun_out/${TAG}_ab.jsonl
: > $OUT
for pass in 1 2; do
  for v in "X=0" "SR_AMD_TREES_PER_BLOCK=64" "SR_AMD_TREES_PER_BLOCK=32" "SR_AMD_MAX_ROW_BLOCKS=1024"; do
    echo "{\"variant\": \"$v\", \"pass\": $pass}" >> $OUT
    env $v timeout -k 10 240 python3 -u tools/share_probe.py >> $OUT 2>> gpurun_out/${TAG}_ab.err || exit $?
  done
done
