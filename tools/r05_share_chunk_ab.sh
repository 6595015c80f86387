#!/bin/bash
# Tree-sharding share vs C2 (tools/share_probe.py) under two-chunk pipeline variants: the share's 1,250 trees
# run as one chunk by default (1/6 of them is below SR_AMD_CHUNK_MIN), so its compile is exposed; lower
# thresholds and other first-chunk fractions let the first chunk's kernel hide the rest's compile.  Two
# alternating passes.  Tag $1.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05sc}
mkdir -p gpurun_out
OUT=gpurun_out/${TAG}_ab.jsonl
: > $OUT
for pass in 1 2; do
  for v in "X=0" "SR_AMD_CHUNK_MIN=100" "SR_AMD_CHUNK_MIN=100 SR_AMD_FIRST_CHUNK=3" "SR_AMD_CHUNK_MIN=100 SR_AMD_FIRST_CHUNK=10"; do
    echo "{\"variant\": \"$v\", \"pass\": $pass}" >> $OUT
    env $v timeout -k 10 240 python3 -u tools/share_probe.py >> $OUT 2>> gpurun_out/${TAG}_ab.err || exit $?
  done
done
