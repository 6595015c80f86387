#!/bin/bash
# Search latency A/B over launch-shape knobs (environment), tools/search_ab.py C3 C5, 30 iterations,
# two alternating passes.  Tag $1, then the variants ("X=0" = default).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; shift
mkdir -p gpurun_out
OUT=gpurun_out/${TAG}_knobs.jsonl
: > $OUT
for pass in 1 2; do
  for v in "$@"; do
    echo "{\"variant\": \"$v\", \"pass\": $pass}" >> $OUT
    env $v ITERS=30 timeout -k 10 300 python3 -u tools/search_ab.py C3 C5 >> $OUT 2>> gpurun_out/${TAG}_knobs.err || exit $?
  done
done
